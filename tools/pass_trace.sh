#!/bin/bash
# (needs a diagnostics build: bash tools/build_ab.sh diag -DLSM_DIAG=1, run with LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/diag.so)
# Per-pass NN statistics and per-dispatch kernel durations of the bench workload.
# usage: bash tools/pass_trace.sh TAG [extra env ...]
set -u
TAG=${1:-pt}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
env "$@" LSM_DEBUG_PASSES=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-c45 --steps 1 --warmup 1 > "$OUT/bench.log" 2> "$OUT/passes.log" || { echo "bench failed"; tail -20 "$OUT/passes.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-400
tail -32 "$OUT/passes.log"
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-c45 --steps 1 --warmup 0 > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
T=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
for k in "nn_kernel<false>" "nn_kernel<true>" nn_fallback accumulate_kernel solve_kernel normals_kernel; do
  echo "== $k"; python3 tools/trace_passes.py "$T" "$k" 40
done
