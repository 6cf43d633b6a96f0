#!/bin/bash
# round 5: accumulate kernel at 8 waves/SIMD (LSM_ACC_WPE=8: 64 VGPRs, 2 spilled)
set -u
OUT=gpurun_out/r05bc; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05bc base:-: acc8:acc8: base2:-: acc82:acc8: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05bc c4base:-: c4acc8:acc8: || exit 1
