#!/bin/bash
# round 5: x block width 16 / 32 / 64 cells, A/B on C3 / C4 / C5
set -u
OUT=gpurun_out/r05n; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05n b16:bx16: b32:bx32: b64:bx64: b16b:bx16: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05n c4b16:bx16: c4b32:bx32: c4b64:bx64: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05n c5b16:bx16: c5b32:bx32: c5b64:bx64: || exit 1
