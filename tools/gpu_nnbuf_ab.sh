set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r03_nnbuf_tests.log 2>&1 || { tail -30 gpurun_out/r03_nnbuf_tests.log; exit 1; }
tail -2 gpurun_out/r03_nnbuf_tests.log
bash tools/ab_env.sh r03_nnbuf nbuf:- nbw7:nbw7 nbw8:nbw8 nbpf2w7:nbpf2w7 nobufnn:nobufnn
