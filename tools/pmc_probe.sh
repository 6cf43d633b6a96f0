#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc run per counter group) over the ICP and normals
# kernels of a bench-shaped run. usage: bash tools/pmc_probe.sh TAG [bench args]
set -u
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps 1 --warmup 0 --seq-cache /tmp/lsm_seq.npz $*"
# the sequence cache is written by a plain run first (no profiler: data generation may fork)
timeout -k 10 300 python bench.py $ARGS > $OUT/plain.log 2>&1 || { echo "plain run failed"; tail -5 $OUT/plain.log; exit 1; }
tail -1 $OUT/plain.log | cut -c1-300
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex "nn_kernel|nn_fallback|normals_kernel|accumulate" \
    --output-format csv -d $OUT/$name -o run -- python3 bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
  echo "pass $name ok"
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
pass sq2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC
pass mem TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
python3 tools/pmc_summary.py $OUT
