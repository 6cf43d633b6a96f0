#!/bin/bash
# round 5: LDS tile capacity A/B (2048 / 3072 / 4096 points: 4 / 3 / 2 workgroups per CU) vs the
# global path; the C5 workload test with the per-pair magnitudes
set -u
OUT=gpurun_out/r05d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py -v -s --timeout 600 --timeout-method thread -k ouster > $OUT/pytest_c5.log 2>&1
rc=$?; grep -E "FAILED|ERROR|within the bar" $OUT/pytest_c5.log | cut -c1-600 | head -20; tail -1 $OUT/pytest_c5.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_env.sh r05d t4096:-: t2048:tcap2048: t3072:tcap3072: t0:-:LSM_NN_TILE=0 || exit 1
