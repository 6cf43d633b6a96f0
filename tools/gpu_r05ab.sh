#!/bin/bash
# round 5: NN row runs' entry search within the query's own x-cell (LSM_NN_CELLENTRY)
set -u
OUT=gpurun_out/r05ab; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05ab base:base: ce:-: base2:base: ce2:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ab c4base:base: c4ce:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ab c5base:base: c5ce:-: || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_headline.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_ce.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_ce.log | head -20; tail -1 $OUT/pytest_ce.log
exit $rc
