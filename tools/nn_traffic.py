"""Per-pass HBM traffic of the correspondence pass from tools/pmc_nn.sh's counter CSVs.

FETCH_SIZE is doubled (gfx950 reports half the bytes of wide coalesced reads,
MI355X_MICROARCH.md HBM section); WRITE_SIZE is taken as read. Both are in KB. A pass = one
nn_kernel launch plus its nn_fallback launch; the algorithmic bytes come from the same run's
bench JSON line (SURVEY.md §8d model, averaged per pass).
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import PMC_KERNELS, kernel_sha, source_sha  # noqa: E402

out = sys.argv[1]
workload = sys.argv[2] if len(sys.argv) > 2 else "hdl64_seq"


def total(counter):
    f = glob.glob(os.path.join(out, counter, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    names = {}
    for r in csv.DictReader(open(f)):
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    passes = sum(1 for d in per if "nn_fallback" in names[d])
    return sum(per.values()), passes, len(per)


fetch_kb, passes, n1 = total("FETCH_SIZE")
write_kb, passes2, n2 = total("WRITE_SIZE")
bench = None
for line in open(os.path.join(out, "FETCH_SIZE.log")):
    if line.startswith("{"):
        bench = json.loads(line)
algo = bench["roofline"]["algo_bytes_per_launch"] if bench else None
hbm = (2.0 * fetch_kb + write_kb) * 1024.0 / max(passes, 1)
print(json.dumps({
    "workload": workload,
    "source_sha256": source_sha(),
    "kernel_sha": kernel_sha(tuple(PMC_KERNELS["nn_traffic.json"])),
    "kernel": "correspondence pass (nn_kernel + nn_fallback)",
    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
              f"bench.py --workload {workload} --steps 2 --warmup 1 (tools/pmc_nn.sh)",
    "passes": passes, "dispatches": [n1, n2],
    "pairs_per_gpu": bench["config"].get("pairs_per_gpu") if bench else None,
    "fetch_size_kb_per_pass": fetch_kb / max(passes, 1),
    "write_size_kb_per_pass": write_kb / max(passes2, 1),
    "correction": "gfx950 FETCH_SIZE counts 1/2 of wide coalesced reads: fetch doubled; "
                  "WRITE_SIZE as read",
    "hbm_bytes_per_launch": hbm,
    "algo_bytes_per_launch": algo,
    "traffic_over_algorithmic": hbm / algo if algo else None,
}, indent=1))
