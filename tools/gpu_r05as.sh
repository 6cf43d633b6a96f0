#!/bin/bash
# round 5: fallback queue split into 8 sub-queues (one append counter per XCD instead of one)
set -u
OUT=gpurun_out/r05as; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05as base:base: subq:-: base2:base: subq2:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05as c4base:base: c4subq:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05as c5base:base: c5subq:-: || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_headline.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; grep -E "FAILED|ERROR" $OUT/pytest.log | head; tail -1 $OUT/pytest.log
