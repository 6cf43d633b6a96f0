#!/bin/bash
# round 5: NN walk load groups / prefetch on the 64-wide layout (LSM_NN_G, LSM_NN_PF)
set -u
OUT=gpurun_out/r05ai; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05ai base:-: pf0:pf0: g1:g1: g1pf0:g1pf0: g4pf0:g4pf0: base2:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ai c4base:-: c4pf0:pf0: c4g1:g1: || exit 1
