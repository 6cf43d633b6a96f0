#!/bin/bash
# round 5: software-pipelined fallback survivors (pipe) vs the committed virtual-block fallback
# (base), 64-cell x blocks: A/B on C3 / C4 / C5, then the parity files on pipe
set -u
OUT=gpurun_out/r05p; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05p base:base: pipe:pipe: base2:base: pipe2:pipe: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05p c4base:base: c4pipe:pipe: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05p c5base:base: c5pipe:pipe: || exit 1
timeout -k 10 900 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/pipe.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_pipe.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_pipe.log | head -20; tail -1 $OUT/pytest_pipe.log
exit $rc
