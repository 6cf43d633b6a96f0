#!/bin/bash
# round 4: two-phase scan 1 (near rows first) -- normals bit-identical to the previous build for
# every NEAR_BINS, then the A/B timing
set -u
OUT=gpurun_out/r04i; mkdir -p $OUT; export TMPDIR=/tmp
for v in prev nb128 nb64 nb84 nb96 intree; do
  if [ $v = intree ]; then E=(); else E=("LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/$v.so"); fi
  timeout -k 10 300 env "${E[@]}" python tools/normals_dump.py $OUT/n_$v.npz > $OUT/dump_$v.log 2>&1 || { cat $OUT/dump_$v.log; exit 1; }
done
for v in nb128 nb64 nb84 nb96 intree; do echo -n "$v vs prev: "; python tools/normals_dump.py --compare $OUT/n_prev.npz $OUT/n_$v.npz; done
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "normals or lazy" > $OUT/pytest_sel.log 2>&1; tail -1 $OUT/pytest_sel.log
bash tools/ab_env.sh r04i intree:-: prev:prev: nb64:nb64: nb84:nb84: nb96:nb96: nb128:nb128:
