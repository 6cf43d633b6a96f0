#!/bin/bash
# round 5: the default bench line with the recounted PMC (complete rooflines for C3 / C4 / C5),
# the N-rank rehearsal of the default line (2 and 3 ranks sharing the GPU), NN cache counters
set -u
OUT=gpurun_out/r05g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
python3 - $OUT/bench.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for name, b in (("C3", j), ("c4", j["c4"]), ("c5", j["c5"])):
    r, n = b["roofline"], b["roofline_normals"]
    print(name, b["value"], b["ms_per_step"], "frac", r["frac"], "traffic", r["traffic"], r["traffic_over_algorithmic"], "valu frac", n["frac"], "cpu", b["cpu_baseline"]["value"])
PY
bash tools/gpu_multirank_default.sh r05g_mr || exit 1
bash tools/pmc_nn_cache.sh || exit 1
