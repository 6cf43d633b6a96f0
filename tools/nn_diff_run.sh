#!/bin/bash
# Find the pair and pass where two builds' NOCERT searches disagree (debug). usage: bash tools/nn_diff_run.sh ab/base.so
set -eu
B=$1
export LSM_NN_NOCERT=1
LIDARSM_LIB=$B timeout -k 10 300 python tools/split_check.py /tmp/a.npz 64 > /dev/null
timeout -k 10 300 python tools/split_check.py /tmp/b.npz 64 > /dev/null
P=$(python3 -c "
import numpy as np
a=np.load('/tmp/a.npz'); b=np.load('/tmp/b.npz')
d=np.abs(a['T']-b['T']).max(axis=(1,2)); print(','.join(str(i) for i in np.nonzero(d>0)[0]))")
echo "pairs differing: $P"
[ -z "$P" ] && exit 0
LIDARSM_LIB=$B timeout -k 10 600 python tools/nn_diff.py /tmp/da.npz 64 $P > /dev/null
timeout -k 10 600 python tools/nn_diff.py /tmp/db.npz 64 $P > /dev/null
python3 - <<PY
import numpy as np
a=np.load('/tmp/da.npz'); b=np.load('/tmp/db.npz')
for p in "$P".split(','):
    for k in range(31):
        kc=f'c_{p}_{k}'
        if kc not in a.files: break
        ca, cb = a[kc], b[kc]
        if not np.array_equal(ca, cb):
            idx=np.nonzero(ca!=cb)[0]
            print(f"pair {p} pass {k}: {len(idx)} queries differ, first src {idx[:5]} base {ca[idx[:5]]} new {cb[idx[:5]]}")
            np.savez('gpurun_out/nn_diff.npz', pair=int(p), k=k, T=a[f'T_{p}_{k}'], Tprev=a[f'T_{p}_{k-1}'] if k>0 else np.eye(4), idx=idx, ca=ca[idx], cb=cb[idx])
            break
PY
