#!/bin/bash
# lazy-normals / normals tests, then the C4 and C5 lines. usage: bash tools/gpu_c45.sh TAG [pytest -k]
set -u
TAG=${1:-run}
K=${2:-lazy or normals}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > "$OUT/pytest_sel.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_sel.log"; exit 1; }
tail -1 "$OUT/pytest_sel.log"
for W in loop_closure ouster_multiscale; do
  timeout -k 10 600 python bench.py --workload $W --no-c1 --no-cpu-baseline > "$OUT/bench_$W.log" 2>&1 || { echo "bench $W failed"; tail -30 "$OUT/bench_$W.log"; exit 1; }
  tail -1 "$OUT/bench_$W.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$W', j['value'], j['ms_per_step'], j['breakdown_ms_per_step'])"
done
