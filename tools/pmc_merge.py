"""Merge one PMC summary (tools/nn_traffic.py / tools/normals_valu.py output) into a per-workload
file: python tools/pmc_merge.py SUMMARY.json TARGET.json (TARGET: {workload: summary, ...}; a
file in the older single-summary format is replaced)."""
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
with open(src) as f:
    entry = json.load(f)
data = {}
if os.path.exists(dst):
    with open(dst) as f:
        old = json.load(f)
    if isinstance(old, dict) and all(isinstance(v, dict) and "workload" in v for v in old.values()):
        data = old
data[entry["workload"]] = entry
with open(dst, "w") as f:
    json.dump(data, f, indent=1)
    f.write("\n")
