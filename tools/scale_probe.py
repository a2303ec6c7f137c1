"""f16x3 per-tensor maxima read back after each encode: eager vs hipGraph replays (diagnostic)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tokenize-audio_amd")
from mimi_hip import synthetic
from mimi_hip.model import MimiHipModel
m = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=32), device="cuda:0")
L = 96000
loud = np.clip(synthetic.speech_like(L, 9, 0) / np.float32(0.9) * np.float32(1.5), -1, 1).astype(np.float32)
quiet = {g: (synthetic.speech_like(L, 9, 1) * np.float32(g)).astype(np.float32) for g in (0.01, 0.001)}
seq = [("batch", np.stack([loud, quiet[0.01], quiet[0.001]]))] + [("loud4", np.stack([loud] * 4))] * 5 + \
      [("q0.01", quiet[0.01][None])] * 3
prev = None
for name, x in seq:
    xd = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    m.encode_int32(xd, 32)
    sc = m.act_scales()
    cur = {k: v[1] for k, v in sc.items()}
    print(name, "replays", m.graph_replays, "reruns", m.f16_reruns, flush=True)
    if prev is not None and name == "loud4" and cur != prev:
        print("   changed:", {k: (prev[k], cur[k]) for k in cur if cur[k] != prev[k]}, flush=True)
        print("   all:", cur, flush=True)
    prev = cur
