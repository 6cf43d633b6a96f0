set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "split_launch or preclass or normals" > gpurun_out/r03_walk_tests.log 2>&1 || { tail -30 gpurun_out/r03_walk_tests.log; exit 1; }
tail -2 gpurun_out/r03_walk_tests.log
bash tools/ab_env.sh r03_walk buf:- pfd2:pfd2 nobuf:nobuf buf2:-
