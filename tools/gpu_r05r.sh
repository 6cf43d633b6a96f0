#!/bin/bash
# fallback cost per pass on the full C3 batch (diagnostics build): max-item chunks per pass
set -u
OUT=gpurun_out/r05r; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/diag.so python tools/nn_stats.py 1999 > $OUT/nn_stats.log 2>&1 || { echo "nn_stats failed"; tail -5 $OUT/nn_stats.log; exit 1; }
grep fbstat $OUT/nn_stats.log
