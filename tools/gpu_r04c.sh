#!/bin/bash
# round 4 A/B: small-neighbourhood threshold (16 in-tree, 8, none) and the NN cold seed; headline
# parity with NSMALL = 8
set -u
OUT=gpurun_out/r04c; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r04c intree:-: ns8:ns8: ns2:ns2: noseed:-:LSM_NN_COLD_SEED=0 gd4:gd4: gd3:gd3: pfd2:pfd2: || exit 1
timeout -k 10 600 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/ns8.so python -u tools/bench_parity.py --out $OUT/parity_ns8.json > $OUT/parity_ns8.log 2>&1 || { tail -20 $OUT/parity_ns8.log; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/parity_ns8.json')); print('ns8 parity', j['within_tolerance'], j['worst_converged'], j['iterations_equal'])"
