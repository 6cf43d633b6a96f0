#!/bin/bash
# HBM traffic of the correspondence pass (nn_kernel + nn_fallback) of one bench workload:
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (MI355X_MICROARCH.md: TCC counters, one
# block's slots per pass). The synthetic data is generated once by a plain run (data generation
# forks; it must not run under the profiler) and loaded from its cache by both passes. The
# summary is merged, keyed by workload, into gpurun_out/nn_traffic.json (a copy of profiles/').
#   tools/pmc_nn.sh [hdl64_seq|loop_closure|ouster_multiscale] [more bench.py args]
set -u
W=${1:-hdl64_seq}; shift || true
OUT=gpurun_out/pmc_nn_$W; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-c45 --seq-cache /tmp/lsm_$W.npz $*"
timeout -k 10 300 python bench.py $ARGS > $OUT/plain.log 2>&1 || { echo "plain run failed"; tail -5 $OUT/plain.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "nn_kernel|nn_fallback" \
    --output-format csv -d $OUT/$c -o run -- python3 bench.py $ARGS \
    > $OUT/$c.log 2>&1 || { echo "$c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python3 tools/nn_traffic.py $OUT $W > $OUT/summary.json || exit 1
[ -f gpurun_out/nn_traffic.json ] || cp profiles/nn_traffic.json gpurun_out/nn_traffic.json
python3 tools/pmc_merge.py $OUT/summary.json gpurun_out/nn_traffic.json && cat $OUT/summary.json
