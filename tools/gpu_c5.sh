#!/bin/bash
# voxel / multi-scale tests and the C5 line (+ its rocprof stats). usage: bash tools/gpu_c5.sh TAG
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "voxel or multiscale or fpfh or grid or build_map" > "$OUT/pytest_sel.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_sel.log"; exit 1; }
tail -1 "$OUT/pytest_sel.log"
timeout -k 10 600 python bench.py --workload ouster_multiscale --no-c1 --no-cpu-baseline > "$OUT/bench_c5.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench_c5.log"; exit 1; }
tail -1 "$OUT/bench_c5.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('C5', j['value'], j['ms_per_step'], j['breakdown_ms_per_step'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5" -o run -- python3 bench.py --workload ouster_multiscale --no-cpu-baseline --no-c1 --steps 3 --warmup 1 > "$OUT/bench_c5_prof.log" 2>&1 || { echo "rocprof c5 failed"; tail -30 "$OUT/bench_c5_prof.log"; exit 1; }
find "$OUT/prof5" -name '*kernel_stats.csv' -exec cp {} "$OUT/c5_kernel_stats.csv" \;
rm -rf "$OUT/prof5"
python3 - "$OUT/c5_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    n = r["Name"]
    n = n.split("detail::")[2][:40] if "rocprim" in n else n.split("(")[0][-40:] if "(" in n[:60] else n[:40]
    print(f"{n:42s} {r['Calls']:>6s} {float(r['TotalDurationNs'])/1e6:9.3f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
