#!/bin/bash
# One measurement session on the box: GPU suite + smoke, the default bench line (CPU baseline,
# C1 and C2 lines) with its rocprof kernel stats, the C4 / C5 lines, the C4 sharding balance.
# usage: bash tools/gpu_measure.sh TAG [notests|tests] [nobalance]
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-}" != "notests" ]; then
  bash tools/gpu_tests.sh $TAG; rc=$?
  [ $rc -ne 0 ] && { echo "gpu tests rc $rc"; exit $rc; }
fi
timeout -k 10 900 python bench.py --seq-cache /tmp/lsm_hdl64_seq.npz > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz > "$OUT/bench_under_rocprof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$OUT/bench_under_rocprof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
head -8 "$OUT/kernel_stats.csv" | cut -c1-160
for W in loop_closure ouster_multiscale; do
  timeout -k 10 600 python bench.py --workload $W --no-c1 --no-c45 --seq-cache /tmp/lsm_$W.npz > "$OUT/bench_$W.log" 2>&1 || { echo "bench $W failed"; tail -30 "$OUT/bench_$W.log"; exit 1; }
  tail -1 "$OUT/bench_$W.log" | cut -c1-200
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$W" -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-c45 --seq-cache /tmp/lsm_$W.npz > "$OUT/bench_${W}_under_rocprof.log" 2>&1 || { echo "rocprof $W failed"; tail -30 "$OUT/bench_${W}_under_rocprof.log"; exit 1; }
  find "$OUT/prof_$W" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$W.csv" \;
  rm -rf "$OUT/prof_$W"
done
[ "${3:-}" = "nobalance" ] && exit 0
timeout -k 10 600 python -u tools/c4_balance.py --out "$OUT/c4_balance.json" > "$OUT/c4_balance.log" 2>&1 || { echo "c4_balance failed"; tail -30 "$OUT/c4_balance.log"; exit 1; }
tail -12 "$OUT/c4_balance.log"
