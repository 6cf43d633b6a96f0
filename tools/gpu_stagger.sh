#!/bin/bash
# Multi-stream pipelining of the C3 step: S contexts, staggered or not.
set -u
OUT=gpurun_out/${1:-r03_st}; mkdir -p $OUT; export TMPDIR=/tmp
A="--no-cpu-baseline --seq-cache /tmp/lsm_seq.npz --steps 3 --warmup 1"
summ() { tail -1 "$1" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$2', j['value'], j['ms_per_step'], j['roofline']['frac'], j['breakdown_ms_per_step'])"; }
timeout -k 10 600 python bench.py $A > $OUT/s1.log 2>&1 || exit 1; summ $OUT/s1.log s1
for S in 2 3 4 8; do
  timeout -k 10 600 python bench.py $A --streams $S --stagger > $OUT/s${S}st.log 2>&1 || { tail -20 $OUT/s${S}st.log; exit 1; }
  summ $OUT/s${S}st.log s${S}stagger
done
timeout -k 10 600 python bench.py $A --streams 2 > $OUT/s2.log 2>&1 || exit 1; summ $OUT/s2.log s2
