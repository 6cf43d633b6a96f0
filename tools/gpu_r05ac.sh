#!/bin/bash
# round 5: entry search within the own x-cell, loaded lazily inside long runs only
set -u
OUT=gpurun_out/r05ac; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05ac base:base: ce:-: base2:base: ce2:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ac c5base:base: c5ce:-: || exit 1
