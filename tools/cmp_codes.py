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
        same = np.array_equal(ref[k], got[k])
        bad += not same
        print(tag, k, "bitwise equal" if same else f"DIFFERS in {int((ref[k] != got[k]).sum())} codes")
sys.exit(1 if bad else 0)
