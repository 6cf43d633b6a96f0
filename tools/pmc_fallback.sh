#!/bin/bash
# The correspondence fallback (nn_fallback_g) on the C3 bench workload: per-launch durations and
# SQ / TA counters (separate --pmc passes), then the diagnostics build's per-pass fbstat lines.
# usage: bash tools/pmc_fallback.sh   (expects lidar_slam_arvc_amd/_lib/ab/diag.so for the stats)
set -u
OUT=gpurun_out/pmc_fb; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--workload hdl64_seq --steps 1 --warmup 1 --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz"
[ -f /tmp/lsm_hdl64_seq.npz ] || timeout -k 10 300 python bench.py $ARGS > $OUT/plain.log 2>&1 || { echo "plain run failed"; exit 1; }
RX="nn_fallback"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "$RX" \
    --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
agg = collections.defaultdict(float)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
durs = []
for f in glob.glob(out + "/p1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "nn_fallback" in r["Kernel_Name"]:
            durs.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
durs = [d for _, d in sorted(durs)]
res = {"counters_per_step_2": dict(agg), "launch_us": durs}
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print({c: f"{x:.4g}" for c, x in sorted(agg.items())})
print("launches", len(durs), "us:", [round(d) for d in durs])
PY
if [ -f lidar_slam_arvc_amd/_lib/ab/diag.so ]; then
  timeout -k 10 300 env LIDARSM_LIB=lidar_slam_arvc_amd/_lib/ab/diag.so python tools/nn_stats.py 512 > $OUT/nn_stats.log 2>&1 || { echo "nn_stats failed"; tail -5 $OUT/nn_stats.log; exit 1; }
  grep fbstat $OUT/nn_stats.log | head -12
fi
