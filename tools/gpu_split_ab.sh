set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "split_launch or preclassification" > gpurun_out/r03_sp1_tests.log 2>&1 || { tail -30 gpurun_out/r03_sp1_tests.log; exit 1; }
tail -2 gpurun_out/r03_sp1_tests.log
bash tools/ab_env.sh r03_sp1 mono:-:LSM_NORMALS_SPLIT=0 split:- s32w5:s32w5 s32w5sp7:s32w5sp7 w5mono:s32w5:LSM_NORMALS_SPLIT=0
