#!/bin/bash
# round 5: independent contexts (streams) per GPU on the 64-wide layout
set -u
OUT=gpurun_out/r05al; mkdir -p $OUT; export TMPDIR=/tmp
for s in 1 2 3; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz --steps 5 --warmup 2 --streams $s > $OUT/bench_s$s.log 2>&1 || { tail -20 $OUT/bench_s$s.log; exit 1; }
  tail -1 $OUT/bench_s$s.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$s', j['value'], j['ms_per_step'], j['roofline']['frac'], j['breakdown_ms_per_step'])"
done
