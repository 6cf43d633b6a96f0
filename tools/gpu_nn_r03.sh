#!/bin/bash
# NN search-path exactness tests, normals phase statistics, and a bench line.
set -u
OUT=gpurun_out/${1:-r03_nn}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "variants or certified or icp_parity or correspondences or headline or sharded" > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -2 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/normals_phases.py 64 > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
grep -v amdgpu.ids $OUT/phases.log
timeout -k 10 600 python bench.py --no-cpu-baseline --seq-cache /tmp/lsm_seq.npz > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['breakdown_ms_per_step'], j['roofline']['frac'])"
