#!/bin/bash
# HBM traffic of the correspondence pass (nn_kernel + nn_fallback): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes (MI355X_MICROARCH.md: TCC counters, one block's slots per pass), on
# the default bench workload. The synthetic sequence is generated once by a plain run (data
# generation forks; it must not run under the profiler) and loaded from its cache by both passes.
set -u
OUT=gpurun_out/pmc_nn; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --seq-cache /tmp/lsm_seq.npz $*"
timeout -k 10 300 python bench.py $ARGS > $OUT/plain.log 2>&1 || { echo "plain run failed"; tail -5 $OUT/plain.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "nn_kernel|nn_fallback" \
    --output-format csv -d $OUT/$c -o run -- python3 bench.py $ARGS \
    > $OUT/$c.log 2>&1 || { echo "$c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python3 tools/nn_traffic.py $OUT > $OUT/summary.json && cat $OUT/summary.json
