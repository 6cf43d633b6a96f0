#!/bin/bash
# round 5: the fallback on virtual 4x4x4-cell blocks (independent of the layout's x block width):
# A/B on C3 / C4 / C5, then the parity files on the widest variant
set -u
OUT=gpurun_out/r05o; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05o b4:-: b16:vb16: b32:vb32: b64:vb64: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05o c4b16:vb16: c4b32:vb32: c4b64:vb64: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05o c5b16:vb16: c5b32:vb32: c5b64:vb64: || exit 1
timeout -k 10 900 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/vb64.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_vb64.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_vb64.log | head -20; tail -1 $OUT/pytest_vb64.log
exit $rc
