#!/bin/bash
# round 5: 4-ary entry search in the NN row runs (LSM_NN_BS4)
set -u
OUT=gpurun_out/r05ah; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05ah base:base: bs4:-: base2:base: bs42:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ah c4base:base: c4bs4:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ah c5base:base: c5bs4:-: || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; tail -1 $OUT/pytest.log
