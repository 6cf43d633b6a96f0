#!/bin/bash
# round 5: capped LDS tile search + untiled workgroups through nn_kernel; f64 centroids in the
# small-neighbourhood normals of voxelised clouds. Selected GPU tests, A/B, rocprof stats.
set -u
OUT=gpurun_out/r05c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -k "variants or certified or multiscale or voxel or fpfh or workloads or normals or lazy" > $OUT/pytest_sel.log 2>&1
rc=$?; grep -E "FAILED|ERROR|within the bar" $OUT/pytest_sel.log | head -20; tail -1 $OUT/pytest_sel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_env.sh r05c tile1:-: tile0:-:LSM_NN_TILE=0 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 - $OUT/kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.reader(open(sys.argv[1])))
for r in rows[1:12]:
    print(r[0][:50].ljust(50), r[1], round(float(r[2]) / 1e6, 2), "ms total", round(float(r[3]) / 1e3, 1), "us avg")
PY
