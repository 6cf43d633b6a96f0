#!/bin/bash
# A/B of normals kernel variants on one bench-sized batch (65 HDL-64 scans): normals ms per batch.
# usage: bash tools/ab_normals.sh "ENV=1 ..." "LIDARSM_LIB=ab/x.so" ...   ("X=0": the default)
# AB_TESTS="pattern": afterwards run the GPU tests matching it under the LAST variant.
set -u
mkdir -p gpurun_out/ab
last=""
for v in "$@"; do
  echo "== $v"; env $v timeout -k 10 300 python tools/prep_only.py 65 3 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  last=$v
done
if [ -n "${AB_TESTS:-}" ]; then
  env $last timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$AB_TESTS" > gpurun_out/ab/pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/ab/pytest.log; exit $rc
fi
