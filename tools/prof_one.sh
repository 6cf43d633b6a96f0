#!/bin/bash
# kernel statistics of one workload's bench (no CPU baseline): bash tools/prof_one.sh TAG WORKLOAD
# -> gpurun_out/TAG/kernel_stats.csv (a plain run fills the data cache first: generation forks)
set -u
TAG=$1; W=$2; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --workload $W --no-cpu-baseline --no-c1 --no-c45 --steps 3 --warmup 1 --seq-cache /tmp/lsm_$W.npz > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-c1 --no-c45 --steps 3 --warmup 1 --seq-cache /tmp/lsm_$W.npz > $OUT/bench_under_rocprof.log 2>&1 || { tail -30 $OUT/bench_under_rocprof.log; exit 1; }
cp $(find $OUT/prof -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
gzip -c $(find $OUT/prof -name "*kernel_trace.csv" | head -1) > $OUT/kernel_trace.csv.gz
rm -rf $OUT/prof
