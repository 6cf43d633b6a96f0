#!/bin/bash
# Occupancy sensitivity of the normals and correspondence kernels: extra dynamic LDS per
# workgroup (LSM_NORMALS_XLDS / LSM_NN_XLDS) lowers the resident workgroups per CU.
set -u
OUT=gpurun_out/${1:-r03_occ}; mkdir -p $OUT; export TMPDIR=/tmp
A="--no-cpu-baseline --no-c1 --seq-cache /tmp/lsm_seq.npz --steps 3 --warmup 1"
summ() { tail -1 "$1" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); b=j['breakdown_ms_per_step']; print('$2', j['value'], 'normals', b['normals'], 'nn', b['nn'])"; }
run() { tag=$1; shift; env "$@" timeout -k 10 600 python bench.py $A > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }; summ $OUT/$tag.log $tag; }
run base LSM_X=0
run n3wg LSM_NORMALS_XLDS=7200
run n2wg LSM_NORMALS_XLDS=21000
run nn5wg LSM_NN_XLDS=28000
run nn4wg LSM_NN_XLDS=33000
run nn3wg LSM_NN_XLDS=41000
