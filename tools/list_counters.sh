#!/bin/bash
# the PMC counters rocprofv3 offers on this box's gfx950 (names only)
mkdir -p gpurun_out/counters
timeout -s KILL 120 rocprofv3 --list-avail > gpurun_out/counters/list.txt 2>&1
grep -oE "^\s*(TA|TD|TCP|TCC|SQ|SQC|GRBM)[A-Z0-9_]*" gpurun_out/counters/list.txt | sort -u > gpurun_out/counters/names.txt
wc -l gpurun_out/counters/names.txt
