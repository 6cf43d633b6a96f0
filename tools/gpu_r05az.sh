#!/bin/bash
# round 5: workgroup tables built in the context's grow-only host storage (no fresh multi-MB
# vectors per call)
set -u
OUT=gpurun_out/r05az; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05az base:base: tab:-: base2:base: tab2:-: || exit 1
BENCH_ARGS="--workload loop_closure --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_loop_closure.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05az c4base:base: c4tab:-: || exit 1
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_ouster_multiscale.npz --steps 3 --warmup 1" bash tools/ab_env.sh r05az c5base:base: c5tab:-: || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; grep -E "FAILED|ERROR" $OUT/pytest.log | head; tail -1 $OUT/pytest.log
