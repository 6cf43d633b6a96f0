#!/bin/bash
# round 5, first GPU call: the whole GPU suite on HEAD (with the C4 / C5 full-batch parity tests),
# the C4 / C5 parity summaries, then the default bench line (c4 / c5 blocks included).
set -u
OUT=gpurun_out/r05a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -1 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
for W in loop_closure ouster_multiscale; do
  timeout -k 10 600 python tools/bench_parity.py --workload $W --out $OUT/bench_parity_$W.json > $OUT/bench_parity_$W.log 2>&1 || { echo "parity $W failed"; tail -20 $OUT/bench_parity_$W.log; exit 1; }
  python - $OUT/bench_parity_$W.json <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
print(j["workload"], "within", j["within_tolerance"], "of", j["pairs"], "iters equal", j["iterations_equal"], "outside conv", j["outside_tolerance_converged"], "nonconv", j["nonconverged"]["count"])
PY
done
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
python - $OUT/bench.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("C3", j["value"], j["ms_per_step"], j["roofline"]["frac"])
for c in ("c4", "c5"):
    b = j[c]
    print(c, b["value"], b["ms_per_step"], b["roofline"]["frac"], (b["roofline_normals"] or {}).get("ms_per_step"), b["cpu_baseline"]["value"])
PY
