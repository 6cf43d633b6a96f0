set -e
export TMPDIR=/tmp

mkdir -p gpurun_out/r03_sp2/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_sp2/prof -o run -- python bench.py --no-cpu-baseline --no-c1 --seq-cache /tmp/lsm_seq.npz --steps 2 --warmup 1 > gpurun_out/r03_sp2/prof.log 2>&1
f=$(find gpurun_out/r03_sp2/prof -name '*kernel_stats.csv' | head -1); head -12 "$f" | cut -c1-200
