#!/bin/bash
# quick check of a change: selected GPU tests, then the C3 / C4 / C5 bench lines without the CPU
# baselines. usage: bash tools/gpu_quick.sh TAG "pytest -k expression" [workloads]
set -u
TAG=${1:-quick}; K=${2:-"normals or headline_full or lazy"}; WS=${3:-"hdl64_seq loop_closure ouster_multiscale"}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest_sel.log 2>&1
  rc=$?; tail -2 $OUT/pytest_sel.log; grep -E "FAILED|ERROR" $OUT/pytest_sel.log | head; [ $rc -gt 1 ] && exit $rc
fi
for W in $WS; do
  timeout -k 10 600 python bench.py --workload $W --no-cpu-baseline --no-c45 --seq-cache /tmp/lsm_$W.npz > $OUT/bench_$W.log 2>&1 || { tail -20 $OUT/bench_$W.log; exit 1; }
  tail -1 $OUT/bench_$W.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$W', j['value'], j['ms_per_step'], j['breakdown_ms_per_step'])"
done
