#!/bin/bash
# voxel path check: its GPU parity tests, then the C5 bench line (no CPU baseline)
set -u
TAG=${1:-vcheck}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests -k "voxel or multiscale or build_map or fpfh" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
BENCH_ARGS="--workload ouster_multiscale --no-cpu-baseline --no-c1 --seq-cache /tmp/lsm_ouster.npz --steps 3 --warmup 1" bash tools/ab_env.sh $TAG new:- || exit 1
tail -1 $OUT/bench_new.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['breakdown_ms_per_step'])"
