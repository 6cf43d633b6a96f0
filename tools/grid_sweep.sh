#!/bin/bash
# Step breakdown (normals / nn / grid ms per step) of the default bench workload at several grid cells.
# usage: bash tools/grid_sweep.sh 0.2 0.25 ...
set -u
mkdir -p gpurun_out/sweep
for c in "$@"; do
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --grid-cell $c --seq-cache /tmp/seq_cache.npz > gpurun_out/sweep/g$c.log 2>&1 || { tail -20 gpurun_out/sweep/g$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/g$c.log').read().strip().splitlines()[-1]); print('cell $c', d['value'], d['breakdown_ms_per_step'])"
done
