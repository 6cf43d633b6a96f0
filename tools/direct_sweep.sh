#!/bin/bash
# Step breakdown of the default bench workload at several LSM_NN_DIRECT values (cells; 0 = off).
set -u
mkdir -p gpurun_out/sweep
for d in "$@"; do
  LSM_NN_DIRECT=$d timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --seq-cache /tmp/seq_cache.npz > gpurun_out/sweep/d$d.log 2>&1 || { tail -20 gpurun_out/sweep/d$d.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sweep/d$d.log').read().strip().splitlines()[-1]); print('direct $d', d['value'], d['breakdown_ms_per_step'], d['nn_fallback_fraction'])"
done
