"""VALU instruction counts per normals launch from tools/pmc_normals_bench.sh's counter CSV.

SQ_INSTS_VALU counts wave-level VALU instructions (one per 64-lane issue). The bench's roofline
for the normals kernel divides this per-launch count by the launch's live duration and compares
it with the chip's VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave instruction
(a wave issues a VALU instruction over 2 cycles, MI355X_MICROARCH.md 'Wave scheduling') =
1228.8 G wave-instructions/s.
"""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
f = glob.glob(os.path.join(out, "sq", "**", "*counter_collection.csv"), recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    d = int(r["Dispatch_Id"])
    per.setdefault(d, {})
    per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
bench = None
for line in open(os.path.join(out, "sq.log")):
    if line.startswith("{"):
        bench = json.loads(line)
n = len(per)
# the profiled run executes warmup + steps timed steps and one statistics step (bench.py's
# roofline_normals), each with the same normals work
nsteps = (bench["steps"] + bench["warmup"] + 1) if bench else 1
tot = {c: sum(v.get(c, 0.0) for v in per.values())
       for c in sorted({c for v in per.values() for c in v})}
mode = bench["config"]["normals"].split(", ")[-1] if bench else None
print(json.dumps({
    "kernel": "every normals launch of a step (normals_kernel eager; lazy_normals_kernel per "
              "ICP pass when lazy)",
    "source": "rocprofv3 --kernel-trace --pmc SQ_* (one pass), bench.py --steps 2 --warmup 1, "
              "default workload (tools/pmc_normals_bench.sh)",
    "dispatches": n, "steps_profiled": nsteps, "normals_mode": mode,
    "pairs_per_gpu": bench["config"].get("pairs_per_gpu") if bench else None,
    "per_step": {c: v / nsteps for c, v in tot.items()},
    "valu_per_step": tot.get("SQ_INSTS_VALU", 0.0) / nsteps,
    "valu_per_wave": tot.get("SQ_INSTS_VALU", 0.0) / max(tot.get("SQ_WAVES", 1.0), 1.0),
}, indent=1))
