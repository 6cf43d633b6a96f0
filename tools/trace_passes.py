"""Per-dispatch durations (us) of the kernels matching a substring, from a rocprofv3
kernel_trace.csv, in dispatch order: `python tools/trace_passes.py TRACE.csv nn_kernel [n]`."""
import csv
import sys

path, pat = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 64
rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print(len(d), "dispatches, mean", round(sum(d) / max(len(d), 1), 1), "us")
print([round(x) for x in d[:n]])
