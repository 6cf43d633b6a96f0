#!/bin/bash
# BASELINE.json configs[3] at its stated size on a one-GPU box: 8 ranks x 512 revisit pairs
# (torch.distributed.run, --share-gpu: every rank on device 0, gloo collectives on host tensors),
# the 4096 results gathered by gather_pair_results; then one context registers all 4096 pairs in
# one batch and tools/c4_gather_check.py compares bit for bit. Not a scaling measurement.
# usage: bash tools/gpu_c4_8rank.sh TAG [ranks]
set -u
TAG=${1:-c4_8rank}; N=${2:-8}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29811 \
  bench.py --gpus $N --share-gpu --workload loop_closure --steps 2 --warmup 1 --no-cpu-baseline --no-c45 \
  --save-gathered $OUT/gathered.npz > $OUT/mr${N}_c4.log 2>&1 || { echo "ranks $N failed"; tail -30 $OUT/mr${N}_c4.log; exit 1; }
grep '^{' $OUT/mr${N}_c4.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print($N, j['n_gpus'], j['value'], j['config']['global_pairs'], j['config']['parallelism'])"
timeout -k 10 900 python -u tools/c4_gather_check.py $OUT/gathered.npz --out $OUT/c4_gather_check.json > $OUT/c4_gather_check.log 2>&1
rc=$?; tail -14 $OUT/c4_gather_check.log; exit $rc
