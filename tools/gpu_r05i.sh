#!/bin/bash
# round 5: lanes per query in the full NN passes (LSM_NN_FULL_L 1 / 2 / 4): bit-identity tests, A/B
set -u
OUT=gpurun_out/r05i; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "variants or certified" > $OUT/pytest_sel.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_sel.log | head; tail -1 $OUT/pytest_sel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_env.sh r05i l1:-: l2:-:LSM_NN_FULL_L=2 l4:-:LSM_NN_FULL_L=4 l1b:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05i c4l1:-: c4l2:-:LSM_NN_FULL_L=2 c4l4:-:LSM_NN_FULL_L=4 || exit 1
