"""Codes of fixed synthetic batches from the engine library named by MIMI_HIP_LIB (A/B builds): writes
gpurun_out/<tag>_codes.npz with B = 32 x 10 s (K = 32), a ragged 17-item batch and a batch-1 clip, so builds that must
give the same bits can be compared file to file (tools/cmp_codes.py)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))
from mimi_hip import synthetic  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402

tag = sys.argv[1]
m = MimiHipModel(synthetic.make_state_dict(seed=0), device="cuda:0")
out = {}
x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=501)).cuda()
out["b32"] = m.encode_int32(x, 32).cpu().numpy()
rng = np.random.default_rng(502)
lengths = [int(v) for v in rng.integers(1, 300000, 17)]
clips = [synthetic.speech_like(L, 503, i) for i, L in enumerate(lengths)]
xr = np.zeros((len(clips), max(lengths)), np.float32)
for i, c in enumerate(clips):
    xr[i, :len(c)] = c
out["ragged"] = m.encode_ragged(torch.from_numpy(xr).cuda(), lengths, 32).cpu().numpy()
out["b1"] = m.encode_int32(torch.from_numpy(synthetic.clip_batch(1, 240000, seed=504)).cuda(), 32).cpu().numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"{tag}_codes.npz"), **out)
print(tag, {k: v.shape for k, v in out.items()})
