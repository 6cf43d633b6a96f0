#!/bin/bash
# round 5: device-chosen fallback lanes (queue <= 200k and max_corr >= 4 m: a wave per query)
# A/B against 32 lanes throughout, then the full measurement session
set -u
OUT=gpurun_out/r05ag; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05ag g32:-:LSM_FB_GL=32 auto:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ag c4g32:-:LSM_FB_GL=32 c4auto:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ag c5g32:-:LSM_FB_GL=32 c5auto:-: || exit 1
bash tools/gpu_measure.sh r05ag_m tests nobalance
