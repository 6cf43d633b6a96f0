#!/bin/bash
# Address / L1 pipeline counters of the walk kernels (nn_kernel, normals halves) on the C3 bench
# workload: is the vector-memory front end (TA / TCP) what bounds them? Separate --pmc passes.
set -u
OUT=gpurun_out/pmc_ta; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--workload hdl64_seq --steps 1 --warmup 1 --no-cpu-baseline --no-c1 --no-c45 --seq-cache /tmp/lsm_hdl64_seq.npz"
[ -f /tmp/lsm_hdl64_seq.npz ] || timeout -k 10 300 python bench.py $ARGS > $OUT/plain.log 2>&1 || { echo "plain run failed"; exit 1; }
RX="nn_kernel|normals_dense_kernel|normals_sparse_kernel"
i=0
for set in "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCP_TOTAL_ACCESSES_sum" \
           "TA_BUFFER_READ_WAVEFRONTS_sum TA_TOTAL_WAVEFRONTS_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "$RX" \
    --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = ("nn_kernel<true>" if "<true" in n else "nn_kernel<false>") if "nn_kernel" in n else \
            ("normals_dense" if "dense" in n else "normals_sparse")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
res = {k: dict(v) for k, v in agg.items()}
json.dump(res, open(out + "/summary.json", "w"), indent=1)
for k, v in res.items():
    print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})
PY
