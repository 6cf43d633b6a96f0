#!/bin/bash
# The round's measurement session on one GPU box: PMC traffic of the correspondence pass (into
# profiles/nn_traffic.json, which the bench reads), parity tests, smoke, the headline bench and
# its rocprof kernel stats, the C4 / C5 workloads and the per-pass ICP timeline.
# usage: bash tools/gpu_final.sh TAG      (results under gpurun_out/TAG, small enough to copy back)
set -u
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/pmc_nn.sh > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; tail -8 "$OUT/pmc.log"; exit 1; }
cp gpurun_out/pmc_nn/summary.json profiles/nn_traffic.json
cp gpurun_out/pmc_nn/summary.json "$OUT/nn_traffic.json"
for c in FETCH_SIZE WRITE_SIZE; do
  f=$(find gpurun_out/pmc_nn/$c -name '*counter_collection.csv' | head -1)
  cp "$f" "$OUT/pmc_${c}.csv"
done
rm -rf gpurun_out/pmc_nn
bash tools/gpu_round.sh "$TAG" || exit 1
for w in loop_closure ouster_multiscale; do
  timeout -k 10 600 python bench.py --workload $w --no-cpu-baseline > "$OUT/bench_$w.log" 2>&1 || { echo "$w failed"; tail -8 "$OUT/bench_$w.log"; exit 1; }
  tail -1 "$OUT/bench_$w.log" | cut -c1-300
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --seq-cache /tmp/lsm_seq.npz > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -8 "$OUT/trace.log"; exit 1; }
T=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 tools/trace_timeline.py "$T" > "$OUT/icp_pass_timeline.txt"
rm -rf "$OUT/trace"
tail -3 "$OUT/icp_pass_timeline.txt"
