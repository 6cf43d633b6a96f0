set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "split_launch" > gpurun_out/r03_coop_tests.log 2>&1 || { tail -30 gpurun_out/r03_coop_tests.log; exit 1; }
tail -2 gpurun_out/r03_coop_tests.log
bash tools/ab_env.sh r03_coop split:- coop:-:LSM_NORMALS_COOP=1
