#!/bin/bash
# round 5: x-wider grid blocks (LSM_BLKX_SHIFT 3 / 4: 8 / 16 cells): A/B on C3 / C4 / C5, then the
# GPU suite on the widest variant
set -u
OUT=gpurun_out/r05l; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05l b4:-: b8:bx8: b16:bx16: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05l c4b4:-: c4b8:bx8: c4b16:bx16: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05l c5b4:-: c5b8:bx8: c5b16:bx16: || exit 1
timeout -k 10 1000 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/bx16.so python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/pytest_bx16.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_bx16.log | head -20; tail -1 $OUT/pytest_bx16.log
exit 0
