"""Per-kernel sums of the counter passes written by tools/pmc_probe.sh (rocprofv3 csv)."""
import csv
import glob
import os
import sys
from collections import defaultdict

KEYS = ["nn_kernel<true", "nn_kernel<false", "nn_fallback", "normals_kernel", "accumulate"]
out = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = next((k for k in KEYS if k in r["Kernel_Name"]), None)
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((os.path.dirname(f), r["Dispatch_Id"]))
for k, v in agg.items():
    print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})
    w = v.get("SQ_WAVES", 0)
    if w:
        print(f"   per wave: VALU {v.get('SQ_INSTS_VALU', 0) / w:.0f} VMEM_RD "
              f"{v.get('SQ_INSTS_VMEM_RD', 0) / w:.0f} SALU {v.get('SQ_INSTS_SALU', 0) / w:.0f} "
              f"LDS {v.get('SQ_INSTS_LDS', 0) / w:.0f}; wave cycles: wait "
              f"{v.get('SQ_WAIT_ANY', 0) / max(v.get('SQ_WAVE_CYCLES', 1), 1):.2f} issue-stall "
              f"{v.get('SQ_WAIT_INST_ANY', 0) / max(v.get('SQ_WAVE_CYCLES', 1), 1):.2f} active "
              f"{v.get('SQ_ACTIVE_INST_ANY', 0) / max(v.get('SQ_WAVE_CYCLES', 1), 1):.2f}")
    h, m = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
    if h + m:
        print(f"   L2 hit {h / (h + m):.3f}; L1 accesses {v.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0):.4g}"
              f" L1->L2 reads {v.get('TCP_TCC_READ_REQ_sum', 0):.4g}")
