"""Per-pass timeline of the ICP kernels from a rocprofv3 kernel trace (last step of the run):
python tools/trace_timeline.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
names = ["normals_kernel", "nn_kernel<true", "nn_kernel<false", "nn_fallback", "accumulate",
         "solve_kernel", "plan_kernel", "radix", "grid_scatter", "grid_fill"]


def short(n):
    return next((k for k in names if k in n), n[:24])


last = max(i for i, r in enumerate(rows) if "normals_kernel" in r["Kernel_Name"])
passes, cur = [], None
for r in rows[last + 1:]:
    k = short(r["Kernel_Name"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if k.startswith("nn_kernel"):
        cur = {"start": int(r["Start_Timestamp"])}
        passes.append(cur)
    if cur is not None:
        cur[k] = cur.get(k, 0.0) + d
        cur["end"] = int(r["End_Timestamp"])
tot = 0.0
for i, p in enumerate(passes):
    wall = (p["end"] - p["start"]) / 1e3
    tot += wall
    print(f"pass {i:2d}: wall {wall:8.1f} us  " + "  ".join(
        f"{k.split('<')[0]}{'*' if k.endswith('true') else ''} {v:7.1f}" for k, v in p.items()
        if k not in ("start", "end")))
print(f"total {tot / 1e3:.2f} ms over {len(passes)} passes")
