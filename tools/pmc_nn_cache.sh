#!/bin/bash
# Cache behaviour of the correspondence search (diagnostics): L1 (TCP) and L2 (TCC) request and
# hit counters of nn_kernel over the C3 bench workload, in separate rocprofv3 --pmc passes
# (kernel-trace only). Output: gpurun_out/pmc_nn_cache/*.
set -u
OUT=gpurun_out/pmc_nn_cache; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--workload hdl64_seq --steps 1 --warmup 1 --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz"
[ -f /tmp/lsm_hdl64_seq.npz ] || timeout -k 10 300 python bench.py $ARGS > $OUT/plain.log 2>&1 || { echo "plain run failed"; exit 1; }
i=0
for set in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
           "TCC_REQ_sum TCC_READ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "nn_kernel" \
    --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "nn_kernel<true>" if "ILb1E" in r["Kernel_Name"] or "<true" in r["Kernel_Name"] else "nn_kernel<false>"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})
PY
