#!/bin/bash
# round 5: the GPU suite on the final tree (all knob variants included)
set -u
OUT=gpurun_out/r05am; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head; tail -1 $OUT/pytest_gpu.log; exit $rc
