set -u
# usage: bash tools/ab_direct.sh "LSM_NN_DIRECT=0" "LSM_NN_DIRECT_K=1" ...  (C3 and C4 nn + fallback ms per step)
for v in "$@"; do
  echo "== $v"
  for w in hdl64_seq loop_closure; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --seq-cache /tmp/lsm_seq.npz --workload $w 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown_ms_per_step']; print('$w', d['value'], 'nn+fb', round(b['nn']+b['nn_fallback'],2), b['nn'], b['nn_fallback'])" || exit 1
  done
done
