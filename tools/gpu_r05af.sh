#!/bin/bash
# round 5: fallback lanes per query chosen on the device from the queue length (nn_fallback_auto)
set -u
OUT=gpurun_out/r05af; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05af g32:-:LSM_FB_GL=32 auto:-: m100:-:LSM_FB_WIDE_MAX=100000 m200:-:LSM_FB_WIDE_MAX=200000 m800:-:LSM_FB_WIDE_MAX=800000 g32w8:-:LSM_FB_GL=32,LSM_FB_WIDE_FROM=8 auto2:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05af c4g32:-:LSM_FB_GL=32 c4auto:-: c4m100:-:LSM_FB_WIDE_MAX=100000 || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05af c5g32:-:LSM_FB_GL=32 c5auto:-: c5m100:-:LSM_FB_WIDE_MAX=100000 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_headline.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; tail -1 $OUT/pytest.log
