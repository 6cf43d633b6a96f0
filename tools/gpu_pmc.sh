#!/bin/bash
# PMC passes of the bench workloads: HBM traffic of the correspondence pass (tools/pmc_nn.sh) and
# the normals' SQ instruction counts (tools/pmc_normals_bench.sh); merged per workload into
# gpurun_out/nn_traffic.json and gpurun_out/normals_valu.json (copy to profiles/ afterwards).
# usage: bash tools/gpu_pmc.sh "hdl64_seq loop_closure" [nn|normals|both]
set -u
WS=${1:-"hdl64_seq loop_closure ouster_multiscale"}
WHAT=${2:-both}
for W in $WS; do
  if [ "$WHAT" != normals ]; then bash tools/pmc_nn.sh $W > /dev/null || { echo "pmc_nn $W failed"; exit 1; }; echo "nn $W done"; fi
  if [ "$WHAT" != nn ]; then bash tools/pmc_normals_bench.sh $W > /dev/null || { echo "pmc_normals $W failed"; exit 1; }; echo "normals $W done"; fi
done
python3 - <<'PY'
import json
for f in ("gpurun_out/nn_traffic.json", "gpurun_out/normals_valu.json"):
    try:
        d = json.load(open(f))
    except OSError:
        continue
    for w, e in d.items():
        print(f, w, e.get("traffic_over_algorithmic") or e.get("valu_per_step"))
PY
