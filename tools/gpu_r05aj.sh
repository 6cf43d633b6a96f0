#!/bin/bash
# round 5: normals walk parameters re-checked on the 64-wide layout (load groups of the sparse /
# dense halves, entry-search thresholds)
set -u
OUT=gpurun_out/r05aj; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_env.sh r05aj base:-: gd2:gd2: gd3:gd3: gs1:gs1: gs4:gs4: bs8:bs8: bs32:bs32: sl4:sl4: base2:-: || exit 1
