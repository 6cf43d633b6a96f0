#!/bin/bash
# Round-3 (continued): full GPU suite + smoke, C3 bench line, C4 / C5 lines, C5 rocprof stats.
# usage: bash tools/gpu_r03d.sh TAG
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh $TAG; rc=$?
[ $rc -ne 0 ] && { echo "gpu tests rc $rc"; exit $rc; }
timeout -k 10 900 python bench.py --seq-cache /tmp/lsm_seq.npz > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-600
for W in ouster_multiscale loop_closure; do
  timeout -k 10 600 python bench.py --workload $W --no-c1 > "$OUT/bench_$W.log" 2>&1 || { echo "bench $W failed"; tail -30 "$OUT/bench_$W.log"; exit 1; }
  tail -1 "$OUT/bench_$W.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$W', j['value'], j['ms_per_step'], j['breakdown_ms_per_step'], j['cpu_baseline']['value'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5" -o run -- python3 bench.py --workload ouster_multiscale --no-cpu-baseline --no-c1 --steps 3 --warmup 1 > "$OUT/bench_c5_prof.log" 2>&1 || { echo "rocprof c5 failed"; tail -30 "$OUT/bench_c5_prof.log"; exit 1; }
find "$OUT/prof5" -name '*kernel_stats.csv' -exec cp {} "$OUT/c5_kernel_stats.csv" \;
rm -rf "$OUT/prof5"
cut -c1-140 "$OUT/c5_kernel_stats.csv" | head -24
