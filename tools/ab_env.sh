#!/bin/bash
# A/B bench lines over (library, environment) variants.
# usage: bash tools/ab_env.sh OUTTAG SPEC...   SPEC = tag[:lib][:VAR=val,VAR=val]
#   lib: a lidar_slam_arvc_amd/_lib/ab/<lib>.so name, or '-' for the in-tree library
# bench args via BENCH_ARGS
set -u
OUT=gpurun_out/$1; shift; mkdir -p $OUT; export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz --steps 3 --warmup 1"}
summ() { tail -1 "$1" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); b=j['breakdown_ms_per_step']; print('$2', j['value'], j['ms_per_step'], {k: b[k] for k in b if k in ('normals','nn','nn_fallback','accumulate','grid','normals_lazy')})"; }
for spec in "$@"; do
  IFS=: read -r tag lib envs <<< "$spec"
  E=()
  [ -n "${lib:-}" ] && [ "$lib" != "-" ] && E+=("LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/$lib.so")
  if [ -n "${envs:-}" ]; then IFS=, read -ra kv <<< "$envs"; E+=("${kv[@]}"); fi
  timeout -k 10 600 env "${E[@]}" python bench.py $ARGS > $OUT/bench_$tag.log 2>&1 || { tail -20 $OUT/bench_$tag.log; exit 1; }
  summ $OUT/bench_$tag.log $tag
done
