#!/bin/bash
# A/B of NN search-box caps on the bench workload (per-kernel times per step).
set -u
mkdir -p gpurun_out/nnv
for v in "LSM_NN_KMAX=4" "LSM_NN_KMAX=3" "LSM_NN_KMAX=2" "LSM_NN_KMAX=2 LSM_NN_KCOLD=1" "LSM_NN_KMAX=1 LSM_NN_KCOLD=1"; do
  echo "== $v"
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --pairs-per-gpu 128 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_ms'], d['breakdown_ms_per_step'])"
done
