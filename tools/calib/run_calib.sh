#!/bin/bash
# SQ counter calibration on the box: known VALU counts per wave (tools/calib/valu_calib.hip)
set -u
OUT=gpurun_out/calib; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 60 tools/calib/valu_calib > $OUT/plain.log 2>&1 || { cat $OUT/plain.log; exit 1; }
cat $OUT/plain.log
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU \
  --output-format csv -d $OUT/p1 -o run -- tools/calib/valu_calib > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:12]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: f"{x:.6g}" for c, x in sorted(v.items())})
PY
