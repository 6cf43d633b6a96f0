#!/bin/bash
# Rehearsal of the driver's N-GPU launch of the DEFAULT bench line (C3 main line + c4 / c5
# blocks) on a one-GPU box: torch.distributed.run with 2 and 3 ranks sharing device 0
# (bench.py --share-gpu: gloo collectives on host tensors). Not a scaling measurement.
set -u
OUT=gpurun_out/${1:-r05_mr}; mkdir -p $OUT; export TMPDIR=/tmp
port=29711
for n in 2 3; do
  port=$((port+1))
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus $n --share-gpu --steps 2 --warmup 1 > $OUT/mr_${n}_default.log 2>&1 || { echo "ranks $n failed"; tail -30 $OUT/mr_${n}_default.log; exit 1; }
  grep '^{' $OUT/mr_${n}_default.log | python3 -c "
import json, sys
j = json.loads(sys.stdin.read())
print($n, j['n_gpus'], j['value'], j['config']['global_pairs'], j['config']['parallelism'],
      'c4', j['c4']['value'], j['c4']['config']['global_pairs'], 'c5', j['c5']['value'], j['c5']['config']['global_pairs'])"
done
