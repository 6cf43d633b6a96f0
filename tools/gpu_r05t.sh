#!/bin/bash
# round 5: fallback candidates staged in LDS, FB_U chunks per round (occupancy-bit loads together)
set -u
OUT=gpurun_out/r05t; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05t base:base:LSM_FB_WAVES=20 u4:-: u2:u2: u1:u1: u4b:-: base2:base:LSM_FB_WAVES=20 || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05t c4base:base:LSM_FB_WAVES=20 c4u4:-: c4u2:u2: || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_u4.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_u4.log | head -20; tail -1 $OUT/pytest_u4.log
exit $rc
