#!/bin/bash
# Rehearsal of the driver's N-GPU bench launch on a one-GPU box: torch.distributed.run with 2 and
# 3 ranks sharing device 0 (bench.py --share-gpu: gloo collectives), every workload.
set -u
OUT=gpurun_out/${1:-r03_mr}; mkdir -p $OUT; export TMPDIR=/tmp
port=29611
for n in 2 3; do
  for w in hdl64_seq loop_closure ouster_multiscale; do
    port=$((port+1))
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port \
      bench.py --gpus $n --share-gpu --workload $w --pairs-per-gpu 64 --steps 2 --warmup 1 --no-cpu-baseline --no-c45 > $OUT/mr_${n}_$w.log 2>&1 || { echo "ranks $n $w failed"; tail -30 $OUT/mr_${n}_$w.log; exit 1; }
    grep '^{' $OUT/mr_${n}_$w.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print($n, '$w', j['n_gpus'], j['value'], j['config']['global_pairs'], j['config']['parallelism'])"
  done
done
