#!/bin/bash
# round 4, first GPU call: small-neighbourhood normals check, headline parity, GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python -u tools/normals_small_check.py --out $O/small.json > $O/small.log 2>&1 || exit 11
timeout -k 10 600 python -u tools/bench_parity.py --out $O/parity.json --save-gpu $O/gpu_res.npz > $O/parity.log 2>&1 || exit 12
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 13
