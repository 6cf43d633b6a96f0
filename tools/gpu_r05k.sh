#!/bin/bash
# round 5: top_add / top2_add as selects -- the C3 batch bit-identical to the previous build
# (every pair's transform, fitness, rmse, iterations), the search-path tests, the A/B
set -u
OUT=gpurun_out/r05k; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/prev.so python tools/bench_parity.py --save-gpu $OUT/prev.npz --out $OUT/parity_prev.json > $OUT/parity_prev.log 2>&1 || { tail -5 $OUT/parity_prev.log; exit 1; }
timeout -k 10 600 python tools/bench_parity.py --save-gpu $OUT/new.npz --out $OUT/parity_new.json > $OUT/parity_new.log 2>&1 || { tail -5 $OUT/parity_new.log; exit 1; }
python3 - $OUT <<'PY'
import numpy as np, sys
a = np.load(sys.argv[1] + "/prev.npz"); b = np.load(sys.argv[1] + "/new.npz")
print("bit-identical to the previous build:", all(np.array_equal(a[k], b[k]) for k in a.files if k != "sha256"))
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "variants or certified" > $OUT/pytest_sel.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_sel.log | head; tail -1 $OUT/pytest_sel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_env.sh r05k new:-: prev:prev: new2:-: prev2:prev: || exit 1
