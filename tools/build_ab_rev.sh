#!/bin/bash
# Build liblidarsm.so from the csrc of a git revision (plus extra defines) into
# lidar_slam_arvc_amd/_lib/ab/NAME.so -- the "before" side of an A/B.
# usage: bash tools/build_ab_rev.sh NAME REV [-DFOO=1 ...]
set -eu
NAME=$1; REV=$2; shift 2
ROOT=$(git rev-parse --show-toplevel)
D=$(mktemp -d); C="$D/lidar_slam_arvc_amd/csrc"; mkdir -p "$C" "$D/include" "$ROOT/lidar_slam_arvc_amd/_lib/ab"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" lidar_slam_arvc_amd/csrc/); do
  git -C "$ROOT" show "$REV:$f" > "$C/$(basename $f)"
done
git -C "$ROOT" show "$REV:include/lidarsm.h" > "$D/include/lidarsm.h"
cd "$C"
PIDS=""
for f in api.cpp se3_host.cpp prep.hip icp.hip loop.hip plane.hip; do
  X=""; [ "${f##*.}" = cpp ] && X="-x hip"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" $X -c $f -o $f.o &
  PIDS="$PIDS $!"
done
for p in $PIDS; do wait $p || { echo "compile failed"; rm -rf $D; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC *.o -o "$ROOT/lidar_slam_arvc_amd/_lib/ab/$NAME.so"
rm -rf "$D"
echo "built lidar_slam_arvc_amd/_lib/ab/$NAME.so from $REV"
