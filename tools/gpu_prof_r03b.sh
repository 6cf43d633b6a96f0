set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03_pb; mkdir -p $OUT/prof
timeout -k 10 300 python tools/nn_stats.py 256 > $OUT/nn_stats.log 2>&1 || { tail -20 $OUT/nn_stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-c1 --seq-cache /tmp/lsm_seq.npz --steps 2 --warmup 1 > $OUT/prof.log 2>&1
tail -1 $OUT/prof.log | cut -c1-200
