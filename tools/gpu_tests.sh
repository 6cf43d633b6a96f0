#!/bin/bash
# GPU parity suite + smoke on the box (all tests run; failures are listed, not fatal to the rest).
# usage: bash tools/gpu_tests.sh TAG [pytest -k expression]
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
K=${2:-}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${KARG[@]}" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" "$OUT/pytest_gpu.log" | grep -v PASSED | head -40
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
exit $rc
