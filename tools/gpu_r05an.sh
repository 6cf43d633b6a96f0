#!/bin/bash
# round 5: certified-pass knobs on the 64-wide layout (first checked pass, split lanes)
set -u
OUT=gpurun_out/r05an; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05an base:-: cf3:-:LSM_NN_CERT_FROM=3 sp4:-:LSM_NN_SPLIT=4 sp16:-:LSM_NN_SPLIT=16 base2:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05an c4base:-: c4cf3:-:LSM_NN_CERT_FROM=3 c4sp16:-:LSM_NN_SPLIT=16 || exit 1
