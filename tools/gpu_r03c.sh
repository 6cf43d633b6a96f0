#!/bin/bash
# Round-3 (continued) GPU session: grid A/B (radix vs counting sort), the counting-sort kernels'
# rocprof stats, and the C5 (Ouster multi-scale) timeline gaps (host-side idle).
# (the normals diagnostics at the end expect lidar_slam_arvc_amd/_lib/ab/ndiag{1,2,3}.so built by
#  tools/build_ab.sh NAME -DLSM_NDIAG=N; the grid A/B needs a build with LSM_GRID_RADIX, since removed)
# usage: bash tools/gpu_r03c.sh TAG
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grid or voxel or multiscale or fpfh" > "$OUT/pytest_sel.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_sel.log"; exit 1; }
tail -1 "$OUT/pytest_sel.log"
bash tools/ab_env.sh $TAG radix:-:LSM_GRID_RADIX=1 csort:-: || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-c1 --seq-cache /tmp/lsm_seq.npz --steps 2 --warmup 1 > "$OUT/bench_prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
cut -c1-160 "$OUT/kernel_stats.csv" | head -24
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof5" -o run -- python3 bench.py --workload ouster_multiscale --no-cpu-baseline --no-c1 --steps 2 --warmup 1 > "$OUT/bench_c5_prof.log" 2>&1 || { echo "rocprof c5 failed"; tail -30 "$OUT/bench_c5_prof.log"; exit 1; }
tail -1 "$OUT/bench_c5_prof.log" | cut -c1-300
T=$(find "$OUT/prof5" -name '*kernel_trace.csv' | head -1)
python3 tools/gap_timeline.py "$T" 90 > "$OUT/c5_gaps.txt" 2>&1
rm -rf "$OUT/prof5"
cat "$OUT/c5_gaps.txt"
for v in in-tree ndiag1 ndiag2 ndiag3; do
  if [ $v = in-tree ]; then E=(); else E=("LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/$v.so"); fi
  timeout -k 10 300 env "${E[@]}" python3 tools/normals_ab.py 3 >> "$OUT/normals_ab.txt" 2>&1 || { echo "normals_ab $v failed"; tail -20 "$OUT/normals_ab.txt"; exit 1; }
done
cat "$OUT/normals_ab.txt"
