"""VALU instruction counts per normals launch from tools/pmc_normals_bench.sh's counter CSVs.

SQ_INSTS_VALU counts wave-level VALU instructions (one per 64-lane issue). The bench's roofline
for the normals kernels divides the per-step count by the step's normals time and compares it
with the chip's VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave instruction
(a wave issues a VALU instruction over 2 cycles, MI355X_MICROARCH.md 'Wave scheduling') =
1228.8 G wave-instructions/s. SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* count quad-cycles
(MI355X_MICROARCH.md constants table); they are reported per kernel as fractions of the waves'
lifetime.
"""
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import PMC_KERNELS, kernel_sha, source_sha  # noqa: E402

out = sys.argv[1]
workload = sys.argv[2] if len(sys.argv) > 2 else "hdl64_seq"
bench = None
for line in open(os.path.join(out, "sq.log")):
    if line.startswith("{"):
        bench = json.loads(line)
# the profiled run executes warmup + steps timed steps and one statistics step (bench.py's
# roofline_normals), each with the same normals work
nsteps = (bench["steps"] + bench["warmup"] + 1) if bench else 1


def kname(n):
    m = re.search(r"normals_(sparse_kernel|dense_kernel|refine_kernel|kernel)", n)
    return m.group(0) if m else n


per = {}
for sub in ("sq", "sq2"):
    fs = glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        continue
    for r in csv.DictReader(open(fs[0])):
        k = kname(r["Kernel_Name"])
        per.setdefault(k, {})
        c = r["Counter_Name"]
        per[k][c] = per[k].get(c, 0.0) + float(r["Counter_Value"])
kern = {}
for k, v in per.items():
    d = {c: x / nsteps for c, x in sorted(v.items())}
    wc = v.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
            if c in v:
                d[c + "_frac_of_wave_cycles"] = v[c] / wc
    if v.get("SQ_WAVES"):
        d["valu_per_wave"] = v.get("SQ_INSTS_VALU", 0.0) / v["SQ_WAVES"]
    kern[k] = d
tot = sum(d.get("SQ_INSTS_VALU", 0.0) for d in kern.values())
mode = bench["config"]["normals"].split(", ")[-1] if bench else None
print(json.dumps({
    "workload": workload,
    "source_sha256": source_sha(),
    "kernel_sha": kernel_sha(tuple(PMC_KERNELS["normals_valu.json"])),
    "kernel": "every normals launch of a step (split launch: normals_sparse_kernel + "
              "normals_dense_kernel + normals_refine_kernel, each finishing its small "
              "neighbourhoods in Open3D's arithmetic)",
    "source": "rocprofv3 --kernel-trace --pmc SQ_* (two passes of 8), bench.py --workload "
              f"{workload} --steps 2 --warmup 1 (tools/pmc_normals_bench.sh)",
    "steps_profiled": nsteps, "normals_mode": mode,
    "pairs_per_gpu": bench["config"].get("pairs_per_gpu") if bench else None,
    "per_kernel_per_step": kern,
    "valu_per_step": tot,
}, indent=1))
