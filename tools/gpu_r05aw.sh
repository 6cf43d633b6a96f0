#!/bin/bash
# round 5: kernel trace of two C3 steps for the idle-gap analysis (tools/gap_timeline.py)
set -u
OUT=gpurun_out/r05aw; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz --steps 2 --warmup 1 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
T=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
gzip -c "$T" > $OUT/kernel_trace.csv.gz; rm -rf $OUT/prof
python3 tools/gap_timeline.py $OUT/kernel_trace.csv.gz grid_keys 1 | tail -30
