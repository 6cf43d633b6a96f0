#!/bin/bash
# round 5: the MB-sized workgroup tables uploaded through pinned staging
set -u
OUT=gpurun_out/r05bb; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05bb base:base: pin:-: base2:base: pin2:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05bb c5base:base: c5pin:-: c5base2:base: c5pin2:-: || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; grep -E "FAILED|ERROR" $OUT/pytest.log | head; tail -1 $OUT/pytest.log
