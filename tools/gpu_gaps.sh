#!/bin/bash
# idle gaps between kernels (host-side stalls) of the C5 and C4 steps, from rocprofv3 kernel
# traces. usage: bash tools/gpu_gaps.sh TAG [WORKLOAD ...] (default: ouster_multiscale loop_closure)
set -u
TAG=${1:-run}
shift
WL=("$@"); [ ${#WL[@]} -eq 0 ] && WL=(ouster_multiscale loop_closure)
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for W in "${WL[@]}"; do
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pt_$W" -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-c1 --steps 2 --warmup 1 --seq-cache /tmp/lsm_seq.npz > "$OUT/bench_${W}_trace.log" 2>&1 || { echo "trace $W failed"; tail -30 "$OUT/bench_${W}_trace.log"; exit 1; }
  grep '"metric"' "$OUT/bench_${W}_trace.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$W', j['value'], j['ms_per_step'])"
  T=$(find "$OUT/pt_$W" -name '*kernel_trace.csv' | head -1)
  MS=$(grep '"metric"' "$OUT/bench_${W}_trace.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
  PER=1; [ $W = ouster_multiscale ] && PER=3
  python3 tools/gap_timeline.py "$T" filter_count $PER > "$OUT/gaps_$W.txt" 2>&1
  gzip -c "$T" > "$OUT/trace_$W.csv.gz"
  rm -rf "$OUT/pt_$W"
  cat "$OUT/gaps_$W.txt"
done
