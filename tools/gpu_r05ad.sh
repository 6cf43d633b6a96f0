#!/bin/bash
# round 5: a whole wave per fallback query from pass LSM_FB_WIDE_FROM on
set -u
OUT=gpurun_out/r05ad; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05ad base:-: w0:-:LSM_FB_WIDE_FROM=0 w8:-:LSM_FB_WIDE_FROM=8 w12:-:LSM_FB_WIDE_FROM=12 w18:-:LSM_FB_WIDE_FROM=18 base2:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ad c4base:-: c4w0:-:LSM_FB_WIDE_FROM=0 c4w8:-:LSM_FB_WIDE_FROM=8 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "variants" > $OUT/pytest_variants.log 2>&1; tail -1 $OUT/pytest_variants.log
