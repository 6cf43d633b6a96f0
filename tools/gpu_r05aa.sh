#!/bin/bash
# round 5: fallback survivors in batches of FB_B blocks (one stream of points per batch)
set -u
OUT=gpurun_out/r05aa; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05aa base:base: b4:-: b2:b2: b8:b8: base2:base: b4b:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05aa c4base:base: c4b4:-: c4b8:b8: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05aa c5base:base: c5b4:-: || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_headline.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_b4.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_b4.log | head -20; tail -1 $OUT/pytest_b4.log
exit $rc
