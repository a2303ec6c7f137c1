"""Compares gpurun_out/<ref>_codes.npz with gpurun_out/<tag>_codes.npz (tools/lib_codes.py) bitwise; exit 1 on any
difference."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ref = np.load(os.path.join(ROOT, "gpurun_out", f"{sys.argv[1]}_codes.npz"))
bad = 0
for tag in sys.argv[2:]:
    got = np.load(os.path.join(ROOT, "gpurun_out", f"{tag}_codes.npz"))
    for k in ref.files:
        if k not in got.files:
            print(tag, k, "MISSING")
            bad += 1
            continue
        a, b = ref[k], got[k]
        same = a.shape == b.shape and np.array_equal(a.view(np.uint32) if a.dtype == np.float32 else a,
                                                    b.view(np.uint32) if b.dtype == np.float32 else b)
        if a.dtype.kind == "U":  # (a tap's sha-256)
            print(tag, k, "bitwise equal" if same else "DIFFERS")
            bad += not same
            continue
        bad += not same
        print(tag, k, "bitwise equal" if same else f"DIFFERS in {int((a != b).sum()) if a.shape == b.shape else 'shape'} values")
sys.exit(1 if bad else 0)
