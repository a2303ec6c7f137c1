"""Codes of fixed synthetic batches from the engine library named by MIMI_HIP_LIB (A/B builds): writes
gpurun_out/<tag>_codes.npz with B = 32 x 10 s (K = 32), a ragged 17-item batch and a batch-1 clip, and every stage tap
(sha-256 of the fp32 values, planes reconstructed) of a B = 32 x 1 s batch (the fused q/k/v + attention path) and a B = 2 x 3 s batch
(the two-kernel path), so builds that must give the same bits can be compared file to file (tools/cmp_codes.py)."""
import hashlib
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
TAPS = (["conv0", "encoder", "ds_gemm", "downsample", "proj"] + [f"res{i}_elu" for i in range(4)] +
        [f"down{i}" for i in range(3)] + ["down3_elu"] +
        [f"{n}{l}" for l in range(8) for n in ("qkv", "att", "oproj", "ff", "xfmr")])
for name, (B, L, seed) in {"tb32": (32, 24000, 505), "tb2": (2, 72000, 506)}.items():
    m.set_taps(True)
    out[name] = m.encode_int32(torch.from_numpy(synthetic.clip_batch(B, L, seed=seed)).cuda(), 32).cpu().numpy()
    for t in TAPS:
        try:
            a = np.ascontiguousarray(m.get_tap(t))
            out[f"{name}_{t}"] = np.array([hashlib.sha256(a.tobytes()).hexdigest() + f" {a.shape}"])
        except Exception:  # (a tap the path does not produce, e.g. q/k/v under the fused attention)
            pass
    m.set_taps(False)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"{tag}_codes.npz"), **out)
print(tag, {k: v.shape for k, v in out.items()})
