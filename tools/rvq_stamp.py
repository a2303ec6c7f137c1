"""Per-phase cycle stamps of the persistent RVQ (build with -DRVQC_STAMP=1 into tools/bin/libmimi_hip_stamp.so):
    MIMI_HIP_LIB=tools/bin/libmimi_hip_stamp.so python tools/rvq_stamp.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tokenize-audio_amd"), ROOT]
from mimi_hip import synthetic  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402

m = MimiHipModel(synthetic.make_state_dict(seed=0), device="cuda:0")
m.set_option("rvq_chain", 1)
emb = torch.from_numpy(np.load(os.path.join(ROOT, "tests/golden/golden.npz"))["emb_speech10s"])[None].cuda()
for _ in range(3):
    m.quantize(emb, 32)
torch.cuda.synchronize()
