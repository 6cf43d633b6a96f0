#!/bin/bash
# round 5: fallback occupancy (diag-only counters, 5 waves/SIMD) and lanes per query (LSM_FB_GL),
# workgroups per CU (LSM_FB_WAVES); then parity with GL 16
set -u
OUT=gpurun_out/r05s; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05s base:base: w16:-: w20:-:LSM_FB_WAVES=20 g16w16:-:LSM_FB_GL=16 g16w20:-:LSM_FB_GL=16,LSM_FB_WAVES=20 g16w40:-:LSM_FB_GL=16,LSM_FB_WAVES=40 w20b:-:LSM_FB_WAVES=20 || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05s c4base:base: c4w20:-:LSM_FB_WAVES=20 c4g16w20:-:LSM_FB_GL=16,LSM_FB_WAVES=20 || exit 1
timeout -k 10 900 env LSM_FB_GL=16 LSM_FB_WAVES=20 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_g16.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_g16.log | head -20; tail -1 $OUT/pytest_g16.log
exit $rc
