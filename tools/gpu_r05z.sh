#!/bin/bash
# round 5: fallback timing probes (diagnostics builds with wrong results): per-dispatch durations
# of nn_fallback_g in the first passes for the product build, item setup only (probe1), and no
# survivor scans (probe2)
set -u
OUT=gpurun_out/r05z; mkdir -p $OUT; export TMPDIR=/tmp
for v in prod probe1 probe2; do
  if [ $v = prod ]; then unset LIDARSM_LIB; else export LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- python3 bench.py --no-cpu-baseline --no-c45 --no-c1 --steps 1 --warmup 0 --seq-cache /tmp/lsm_hdl64_seq.npz > $OUT/prof_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 $OUT/prof_$v.log; exit 1; }
  T=$(find $OUT/prof_$v -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python3 tools/trace_passes.py "$T" nn_fallback 12
  cp "$T" $OUT/trace_$v.csv; rm -rf $OUT/prof_$v
done
