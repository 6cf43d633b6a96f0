#!/bin/bash
# A/B bench lines: the in-tree library and each lidar_slam_arvc_amd/_lib/ab/NAME.so given.
# usage: bash tools/ab_bench.sh OUTTAG NAME... (bench args via BENCH_ARGS)
set -u
OUT=gpurun_out/$1; shift; mkdir -p $OUT; export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --seq-cache /tmp/lsm_seq.npz --steps 3 --warmup 1"}
summ() { tail -1 "$1" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); b=j['breakdown_ms_per_step']; print('$2', j['value'], j['ms_per_step'], {k: b[k] for k in b if k in ('normals','nn','nn_fallback','accumulate','grid','normals_lazy')})"; }
timeout -k 10 600 python bench.py $ARGS > $OUT/bench_intree.log 2>&1 || { tail -20 $OUT/bench_intree.log; exit 1; }
summ $OUT/bench_intree.log intree
for n in "$@"; do
  timeout -k 10 600 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/$n.so python bench.py $ARGS > $OUT/bench_$n.log 2>&1 || { tail -20 $OUT/bench_$n.log; exit 1; }
  summ $OUT/bench_$n.log $n
done
