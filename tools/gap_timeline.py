"""Idle gaps of the GPU between consecutive kernels of a rocprofv3 kernel trace (host work the
device waits for), summed by the kernel that precedes the gap, over the last N ms of the trace.
python tools/gap_timeline.py run_kernel_trace.csv [window_ms]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
window = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else None
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
if window is not None:
    t_end = max(e for _, e, _ in ev)
    ev = [x for x in ev if x[0] >= t_end - window]


def short(n):
    n = n.split("(")[0]
    for k in ("radix_sort", "scan_impl", "lookback", "fillBuffer", "copyBuffer"):
        if k in n:
            return k
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
