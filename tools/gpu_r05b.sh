#!/bin/bash
# round 5: LDS tiles for the full NN passes -- bit-identity tests, A/B against the global path,
# rocprof kernel stats of the tiled run
set -u
OUT=gpurun_out/r05b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "variants or certified" > $OUT/pytest_sel.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_sel.log | head; tail -1 $OUT/pytest_sel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_env.sh r05b tile1:-: tile0:-:LSM_NN_TILE=0 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
head -12 $OUT/kernel_stats.csv | cut -d, -f1-5 | cut -c1-150
