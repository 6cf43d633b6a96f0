#!/bin/bash
# Headline parity over all 1999 pairs, the default bench line, its rocprof kernel stats, and the
# normals PMC pass. usage: bash tools/gpu_bench_r03.sh TAG
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_parity.py --out "$OUT/bench_parity.json" > "$OUT/bench_parity.log" 2>&1 || { echo "bench_parity failed"; tail -30 "$OUT/bench_parity.log"; exit 1; }
python - "$OUT/bench_parity.json" <<'PY'
import json,sys; j=json.load(open(sys.argv[1]))
print({k: j[k] for k in ("pairs","within_tolerance","converged_both","converged_within_tolerance","worst_converged","iterations_equal")})
print("nonconverged", j["nonconverged"]["count"], "within", j["nonconverged"]["within_tolerance"], "outside conv", j["outside_tolerance_converged"])
PY
timeout -k 10 900 python bench.py --seq-cache /tmp/lsm_seq.npz > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-3000
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --seq-cache /tmp/lsm_seq.npz > "$OUT/bench_prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
head -12 "$OUT/kernel_stats.csv" | cut -c1-200
bash tools/pmc_normals_bench.sh > "$OUT/pmc_normals.log" 2>&1 || { echo "pmc normals failed"; tail -20 "$OUT/pmc_normals.log"; exit 1; }
cp gpurun_out/pmc_normals_bench/summary.json "$OUT/normals_valu.json"
cat "$OUT/normals_valu.json"
