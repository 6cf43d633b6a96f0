#!/bin/bash
# round 5: the default bench line with 20 timed steps (a stable final figure)
set -u
OUT=gpurun_out/r05ao; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_normals']['frac'], j['c4']['value'], j['c5']['value'])"
