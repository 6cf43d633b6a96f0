#!/bin/bash
# round 5: fallback far split (a whole wave for queries whose box-search best lies beyond
# LSM_FB_FAR m) with a whole wave per query from pass 8 on
set -u
OUT=gpurun_out/r05ae; mkdir -p $OUT; export TMPDIR=/tmp
W=LSM_FB_WIDE_FROM=8
bash tools/ab_env.sh r05ae base:-: w8:-:$W f10:-:$W,LSM_FB_FAR=1.0 f15:-:$W,LSM_FB_FAR=1.5 f20:-:$W,LSM_FB_FAR=2.0 f30:-:$W,LSM_FB_FAR=3.0 f15n:-:LSM_FB_FAR=1.5 || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ae c4base:-: c4w0:-:LSM_FB_WIDE_FROM=0 c4f10:-:$W,LSM_FB_FAR=1.0 c4f15:-:$W,LSM_FB_FAR=1.5 c4f20:-:$W,LSM_FB_FAR=2.0 c4f30:-:$W,LSM_FB_FAR=3.0 || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05ae c5base:-: c5w8:-:$W c5f15:-:$W,LSM_FB_FAR=1.5 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "variants" > $OUT/pytest_variants.log 2>&1; tail -1 $OUT/pytest_variants.log
