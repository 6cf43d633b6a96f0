#!/bin/bash
# Build an A/B variant of liblidarsm.so with extra compiler defines into lidar_slam_arvc_amd/_lib/ab/NAME.so
# usage: bash tools/build_ab.sh NAME -DFOO=1 ...   (run with LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/NAME.so)
set -eu
NAME=$1; shift
D=$(mktemp -d); mkdir -p lidar_slam_arvc_amd/_lib/ab
cd lidar_slam_arvc_amd/csrc
PIDS=""
for f in api.cpp se3_host.cpp prep.hip icp.hip loop.hip plane.hip; do
  X=""; [ "${f##*.}" = cpp ] && X="-x hip"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" $X -c $f -o $D/$f.o &
  PIDS="$PIDS $!"
done
for p in $PIDS; do wait $p || { echo "compile failed"; rm -rf $D; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $D/*.o -o ../_lib/ab/$NAME.so
rm -rf $D
echo "built lidar_slam_arvc_amd/_lib/ab/$NAME.so"
