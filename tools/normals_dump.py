"""Dump the device normals of a few bench scans (and their FPFH lists' normals path) to an .npz,
for bit-for-bit comparisons between two builds (LIDARSM_LIB selects the library):

    LIDARSM_LIB=... python tools/normals_dump.py OUT.npz
    python tools/normals_dump.py --compare A.npz B.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
        print("identical" if not bad else f"DIFFER: {bad}", f"({len(a.files)} arrays)")
        sys.exit(1 if bad else 0)
    from lidar_slam_arvc_amd import _lib, synthetic
    seq = synthetic.make_sequence(12, seed=3, model=synthetic.HDL64, first_index=600)
    ous = synthetic.make_sequence(2, seed=5, model=synthetic.OUSTER128)
    dev = _lib.device(0)
    out = {}
    for tag, scans, prm in (("hdl64", seq.scans, _lib.prep_params()),
                            ("hdl64_nn30", seq.scans[:3], _lib.prep_params(max_nn=30)),
                            ("ouster_v01", ous.scans, _lib.prep_params(voxel_size=0.1))):
        ids = [dev.upload(s) for s in scans]
        dev.preprocess(ids, prm)
        for k, h in enumerate(ids):
            out[f"{tag}_{k}"] = dev.download(h, normals=True)[1]
            dev.release(h)
    np.savez_compressed(sys.argv[1], **out)
    print(f"{len(out)} normal arrays -> {sys.argv[1]}")


if __name__ == "__main__":
    main()
