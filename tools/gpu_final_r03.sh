#!/bin/bash
# Round-3 final measurement: GPU suite + smoke, headline parity over all 1999 pairs, the default
# bench line (CPU baseline included) with its rocprof kernel stats, and the C4 / C5 lines.
# usage: bash tools/gpu_final_r03.sh TAG
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh $TAG; rc=$?
[ $rc -ne 0 ] && { echo "gpu tests rc $rc"; exit $rc; }
timeout -k 10 600 python -u tools/bench_parity.py --out "$OUT/bench_parity.json" > "$OUT/bench_parity.log" 2>&1 || { echo "bench_parity failed"; tail -30 "$OUT/bench_parity.log"; exit 1; }
python3 - "$OUT/bench_parity.json" <<'PY'
import json,sys; j=json.load(open(sys.argv[1]))
print({k: j[k] for k in ("pairs","within_tolerance","converged_both","converged_within_tolerance","worst_converged","iterations_equal")})
PY
timeout -k 10 900 python bench.py --seq-cache /tmp/lsm_seq.npz > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --seq-cache /tmp/lsm_seq.npz > "$OUT/bench_under_rocprof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$OUT/bench_under_rocprof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
head -8 "$OUT/kernel_stats.csv" | cut -c1-160
for W in loop_closure ouster_multiscale; do
  timeout -k 10 900 python bench.py --workload $W --no-c1 > "$OUT/bench_$W.log" 2>&1 || { echo "bench $W failed"; tail -30 "$OUT/bench_$W.log"; exit 1; }
  tail -1 "$OUT/bench_$W.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$W', j['value'], j['ms_per_step'], j['breakdown_ms_per_step'], j['cpu_baseline']['value'])"
done
