#!/bin/bash
# A/B of environment variants on the bench workload: value and per-kernel ms per step.
# usage: bash tools/ab_env.sh "VAR=a" "VAR=b" ...   (use "X=0" for the default)
set -u
mkdir -p gpurun_out/ab
for v in "$@"; do
  echo "== $v"
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --seq-cache /tmp/lsm_seq.npz ${AB_ARGS:-} 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], round(d['roofline']['frac'],4), d['breakdown_ms_per_step'])" || exit 1
done
