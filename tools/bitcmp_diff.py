"""Compares two tools/bitcmp.py outputs bit for bit (dev tool).  usage: python tools/bitcmp_diff.py A.npz B.npz"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in a.files:
    x, y = a[k], b[k]
    same = np.array_equal(x.view(np.uint64) if x.dtype == np.float64 else x, y.view(np.uint64) if y.dtype == np.float64 else y)
    diff = "" if same else f"  differing elements {np.count_nonzero(x != y)}, max |d| {np.max(np.abs(x - y)):.3e}"
    print(f"{k:20s} {'bit-identical' if same else 'DIFFERENT'}{diff}")
