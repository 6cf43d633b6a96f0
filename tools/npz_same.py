"""Bit-for-bit comparison of two npz files: python tools/npz_same.py A.npz B.npz"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
bad = [k for k in a.files if k not in b.files or not np.array_equal(a[k], b[k])]
print("identical" if not bad else f"DIFFER in {bad}")
sys.exit(1 if bad else 0)
