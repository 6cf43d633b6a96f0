#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel-trace stats.
# usage: bash tools/gpu_round.sh TAG [skip-tests]
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
  cat "$OUT/smoke.log"
fi
timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/bench_prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.log"; exit 1; }
tail -1 "$OUT/bench_prof.log"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"   # the traces exceed what gpurun copies back (64 MiB); the summary is kept
head -12 "$OUT/kernel_stats.csv" | cut -c1-220
