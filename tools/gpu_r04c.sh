#!/bin/bash
# round 4 A/B: small-neighbourhood threshold (16 in-tree, 8, none), the NN cold seed, dense-half
# load groups; headline parity with NSMALL = 8; the normals tests on the in-tree build first
set -u
OUT=gpurun_out/r04c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "normals or headline_full or lazy or fpfh" > $OUT/pytest_sel.log 2>&1
rc=$?; tail -3 $OUT/pytest_sel.log; grep -E "FAILED|ERROR" $OUT/pytest_sel.log | head; [ $rc -gt 1 ] && exit $rc
bash tools/ab_env.sh r04c intree:-: ns8:ns8: ns2:ns2: noseed:-:LSM_NN_COLD_SEED=0 gd4:gd4: gd3:gd3: pfd2:pfd2: || exit 1
timeout -k 10 600 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/ns8.so python -u tools/bench_parity.py --out $OUT/parity_ns8.json > $OUT/parity_ns8.log 2>&1 || { tail -20 $OUT/parity_ns8.log; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/parity_ns8.json')); print('ns8 parity', j['within_tolerance'], j['worst_converged'], j['iterations_equal'])"
