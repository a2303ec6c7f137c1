"""Runs B = 32 x 10 s f16x3 encodes with the in-kernel phase-stamp build of the fused stage-0 kernel
(MIMI_HIP_LIB=tools/bin/libmimi_hip_st.so, built with -DS0F_STAMP=1); the kernel prints per-wave cycle sums."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tokenize-audio_amd")
from mimi_hip import synthetic  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402

m = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=8), device="cuda:0")
m.set_graphs(False)
if len(sys.argv) > 1:
    m.set_option("stage0_fused", int(sys.argv[1]))
x = torch.from_numpy(np.stack([synthetic.speech_like(240000, 1, i) for i in range(32)])).cuda()
for _ in range(2):
    m.encode_int32(x, 8)
torch.cuda.synchronize()
