#!/bin/bash
# round 5: box-search reach on the 64-wide layout (LSM_NN_KMAX / KCOLD / DIRECT knobs; all
# bit-identical paths): does a wider box now beat the fallback?
set -u
OUT=gpurun_out/r05v; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05v base:-: kmax5:-:LSM_NN_KMAX=5 kmax6:-:LSM_NN_KMAX=6 kc5:-:LSM_NN_KCOLD=5,LSM_NN_KMAX=5 kc3:-:LSM_NN_KCOLD=3 dir4:-:LSM_NN_DIRECT=4 dir0:-:LSM_NN_DIRECT=0 dyn:-:LSM_FB_DYN=1 base2:-: dyn2:-:LSM_FB_DYN=1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "variants" > gpurun_out/r05v/pytest_variants.log 2>&1; tail -1 gpurun_out/r05v/pytest_variants.log
