#!/bin/bash
# Lazy-normals checks: the lazy GPU tests, then lazy vs eager benches on C3 / C4 / C5.
set -u
OUT=gpurun_out/r03_v4; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "lazy" > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -2 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
summ() { tail -1 "$1" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['config']['workload'], j['config']['normals'], j['value'], j['ms_per_step'], j['breakdown_ms_per_step'])"; }
for w in hdl64_seq loop_closure ouster_multiscale; do
  for m in lazy eager; do
    timeout -k 10 600 python bench.py --no-cpu-baseline --workload $w --normals $m --steps 3 --warmup 1 > $OUT/bench_${w}_$m.log 2>&1 || { tail -20 $OUT/bench_${w}_$m.log; exit 1; }
    summ $OUT/bench_${w}_$m.log
  done
done
