"""Compare two frame_pnp_dump.py outputs bitwise: python frame_pnp_cmp.py A.npz B.npz"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
same = True
for k in a.files:
    eq = np.array_equal(a[k], b[k])
    same &= eq
    d = 0.0 if eq or a[k].dtype.kind not in "fc" else float(np.max(np.abs(a[k] - b[k])))
    print(f"{k}: {'identical' if eq else f'DIFFERS (max |d| {d:.3e})'}")
print("ALL IDENTICAL" if same else "SOME DIFFER")
