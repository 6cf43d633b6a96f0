#!/bin/bash
# round 5: side-stream refine without its own timing bracket; normals roofline without it
set -u
OUT=gpurun_out/r05av; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05av side:-: side0:-:LSM_NORMALS_SIDE=0 side2:-: || exit 1
for v in side side0; do tail -1 $OUT/bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); n=j['roofline_normals']; print('$v', n['ms_per_step'], n['frac'], n['valu_instructions_per_step'])"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "split_launch or lazy" > $OUT/pytest.log 2>&1; tail -1 $OUT/pytest.log
