#!/bin/bash
# round 5: crowded fallback blocks scanned nearest rows first (merge, then the rest pruned)
set -u
OUT=gpurun_out/r05y; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05y base:base: near:-: base2:base: near2:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05y c4base:base: c4near:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05y c5base:base: c5near:-: || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_headline.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_near.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_near.log | head -20; tail -1 $OUT/pytest_near.log
exit $rc
