#!/bin/bash
# A/B of the normals paths on one bench-sized keyframe batch (65 HDL-64 scans).
set -u
mkdir -p gpurun_out/nv
run() { echo "== $1"; env $2 timeout -k 10 300 python tools/prep_only.py 65 3 2>&1 | grep -v amdgpu.ids | tail -1; }
run legacy "LSM_NORMALS_LEGACY=1"
run queue128 "LSM_NORMALS_DENSE_T=128"
run queue300 "LSM_NORMALS_DENSE_T=300"
run queue64 "LSM_NORMALS_DENSE_T=64"
run wave300 "LSM_NORMALS_WAVE=1 LSM_NORMALS_DENSE_T=300"
