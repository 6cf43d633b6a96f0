#!/bin/bash
# round 5: the strict 32-pair headline test; sparse-half occupancy A/B (8 / 7 / 6 waves per SIMD)
set -u
OUT=gpurun_out/r05j; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -v -s --timeout 600 --timeout-method thread -k "both_oracles or iterations_close" > $OUT/pytest_headline.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_headline.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_env.sh r05j w8:-: w7:nsp7: w6:nsp6: w8b:-: || exit 1
