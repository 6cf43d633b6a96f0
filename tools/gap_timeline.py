"""Idle gaps of the GPU between consecutive kernels of a rocprofv3 kernel trace (host work the
device waits for), summed by the kernel they precede, over the last N ms of the trace -- or, with
a marker kernel name, over the window between its (2 per)-th- and per-th-last launches
(one step of a bench run that ends with an untimed statistics step; per = marker launches per
step). python tools/gap_timeline.py run_kernel_trace.csv[.gz] [window_ms | marker per]"""
import csv
import gzip
import sys
from collections import defaultdict

f = gzip.open(sys.argv[1], "rt") if sys.argv[1].endswith(".gz") else open(sys.argv[1])
rows = list(csv.DictReader(f))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
if len(sys.argv) > 3:
    marker, per = sys.argv[2], int(sys.argv[3])
    starts = [s for s, _, n in ev if marker in n]
    a, b = starts[-2 * per], starts[-per]
    ev = [x for x in ev if a <= x[0] < b]
elif len(sys.argv) > 2:
    window = float(sys.argv[2]) * 1e6
    t_end = max(e for _, e, _ in ev)
    ev = [x for x in ev if x[0] >= t_end - window]


def short(n):
    for k in ("radix_sort", "scan_impl", "lookback", "fillBuffer", "copyBuffer", "onesweep"):
        if k in n:
            return k
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    for c in "(<":
        n = n.split(c)[0]
    return n.split("::")[-1][:40]


gap = defaultdict(float)
cnt = defaultdict(int)
busy = defaultdict(float)
end = ev[0][1]
for s, e, n in ev:
    k = short(n)
    busy[k] += (e - s) / 1e6
    if s > end:
        gap[k] += (s - end) / 1e6   # idle before this kernel
        cnt[k] += 1
    end = max(end, e)
span = (ev[-1][1] - ev[0][0]) / 1e6
print(f"span {span:.2f} ms, busy {sum(busy.values()):.2f} ms, idle {sum(gap.values()):.2f} ms")
print("idle before kernel (ms, count):")
for k, v in sorted(gap.items(), key=lambda x: -x[1])[:20]:
    print(f"  {k:42s} {v:8.3f} {cnt[k]:6d}")
print("busy by kernel (ms):")
for k, v in sorted(busy.items(), key=lambda x: -x[1])[:20]:
    print(f"  {k:42s} {v:8.3f}")
