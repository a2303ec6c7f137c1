"""Determinism probe: the same batch encoded repeatedly must give identical codes (graphs off, then on)."""
import json
import sys
import numpy as np
import torch
sys.path.insert(0, "tokenize-audio_amd")
from mimi_hip import synthetic
from mimi_hip.encoder import MimiEncoder
from mimi_hip.model import MimiHipModel
m = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=32), device="cuda:0")
meta = json.load(open("tests/golden/golden_batch_meta.json"))
audio = [synthetic.speech_like(L, meta["audio_seed"], meta["audio_index0"] + i) *
         np.float32(meta["quiet_gain"].get(str(i), 1.0)) for i, L in enumerate(meta["lengths"])]
enc = MimiEncoder(device="cuda:0", model=m)
lmax = max(len(a) for a in audio)
x = np.zeros((len(audio), lmax), np.float32)
for i, a in enumerate(audio):
    x[i, :len(a)] = a
xd = torch.from_numpy(x).cuda()
for graphs in (False, True):
    m.set_graphs(graphs)
    ref = m.encode_int32(xd, 32).cpu()
    d_lean = [int((m.encode_int32(xd, 32).cpu() != ref).sum()) for _ in range(4)]
    d_async = [int((m.encode_async(xd, 32).wait().cpu() != ref).sum()) for _ in range(4)]
    wr = [np.concatenate([o.ravel() for o in enc.encode_audio_batch(audio, 24000)]) for _ in range(4)]
    d_wrap = [int((w != wr[0]).sum()) for w in wr]
    print("graphs", graphs, "lean", d_lean, "async", d_async, "wrapper", d_wrap, "reruns", m.f16_reruns,
          "replays", m.graph_replays, flush=True)
