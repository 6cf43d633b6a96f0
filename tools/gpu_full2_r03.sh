#!/bin/bash
# Round-3 measurement, part 2: PMC passes (normals VALU, NN traffic), C4 / C5 bench lines with
# their CPU baselines, headline parity with the three-way analysis. usage: bash tools/gpu_full2_r03.sh TAG
set -u
TAG=${1:-r03}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/pmc_normals_bench.sh > $OUT/pmc_normals.log 2>&1 || { echo "pmc normals failed"; tail -20 $OUT/pmc_normals.log; exit 1; }
cp gpurun_out/pmc_normals_bench/summary.json $OUT/normals_valu.json; grep -E "valu_per_step|normals_mode" $OUT/normals_valu.json
bash tools/pmc_nn.sh > $OUT/pmc_nn.log 2>&1 || { echo "pmc nn failed"; tail -20 $OUT/pmc_nn.log; exit 1; }
cp gpurun_out/pmc_nn/summary.json $OUT/nn_traffic.json; grep -E "hbm_bytes|traffic_over" $OUT/nn_traffic.json
for w in loop_closure ouster_multiscale; do
  timeout -k 10 900 python bench.py --workload $w > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-400
done
timeout -k 10 800 python -u tools/bench_parity.py --explain --out $OUT/bench_parity.json > $OUT/bench_parity.log 2>&1 || { echo "parity failed"; tail -20 $OUT/bench_parity.log; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/bench_parity.json')); print({k: j[k] for k in ('within_tolerance','converged_both','converged_within_tolerance','worst_converged')})"
