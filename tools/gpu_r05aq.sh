#!/bin/bash
# round 5: occupied-cell count moved from grid_scatter into grid_fill
set -u
OUT=gpurun_out/r05aq; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05aq base:base: fill:-: base2:base: fill2:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05aq c5base:base: c5fill:-: || exit 1
for v in base fill; do tail -1 $OUT/bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$v', j['roofline']['algo_bytes_per_launch'])"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "grid_layout or icp_parity or batch_equals" > $OUT/pytest.log 2>&1; tail -1 $OUT/pytest.log
