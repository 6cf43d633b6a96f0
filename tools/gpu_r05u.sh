#!/bin/bash
# round 5: per-dispatch durations of the correspondence pass kernels (C3, one step), then the
# fallback's SQ / TA counters and the diagnostics build's per-pass statistics
set -u
bash tools/pass_trace.sh r05u_pt || exit 1
bash tools/pmc_fallback.sh
bash tools/gpu_r05v.sh
