#!/bin/bash
# Round-3 measurement, part 1: GPU parity suite + smoke, the default bench line (CPU baseline
# and C1 included), its rocprof kernel stats. usage: bash tools/gpu_full_r03.sh TAG
set -u
TAG=${1:-r03}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_tests.sh $TAG || exit $?
timeout -k 10 900 python bench.py --seq-cache /tmp/lsm_seq.npz > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --seq-cache /tmp/lsm_seq.npz > $OUT/bench_under_rocprof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/bench_under_rocprof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
head -8 $OUT/kernel_stats.csv | cut -c1-160
