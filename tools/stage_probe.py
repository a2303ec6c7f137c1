"""Host staging cost of one ragged batch of 32 U[10, 20] s utterances (the MLS-style path): the copy into pinned
memory, its H2D, the encode enqueue, and the collect, timed separately on the host."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))
from mimi_hip import synthetic  # noqa: E402
from mimi_hip.encoder import MimiEncoder, _Pipeline  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402

m = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=32), device="cuda:0")
lens = synthetic.random_lengths(32 * 6, 10.0, 20.0, seed=77)
clips = [synthetic.speech_like(n, 77, i) for i, n in enumerate(lens)]
pipe = _Pipeline(m, 32)
for rep in range(6):
    b = clips[32 * rep:32 * rep + 32]
    L = max(len(a) for a in b)
    t0 = time.perf_counter()
    pin = pipe._buf(pipe.slots[rep % 2], "pin", 32 * L, torch.float32, True)[:32 * L].view(32, L)
    pn = pin.numpy()
    for i, a in enumerate(b):
        pn[i, :len(a)] = a
    t1 = time.perf_counter()
    pipe.n = rep
    h = pipe.submit(b, [len(a) for a in b], [1] * 32)
    t2 = time.perf_counter()
    out = pipe.collect(h)
    t3 = time.perf_counter()
    print(f"rep {rep}: manual staging copy {1e3 * (t1 - t0):.2f} ms; submit (staging + H2D enqueue + encode enqueue) "
          f"{1e3 * (t2 - t1):.2f} ms; collect (wait + D2H + slicing) {1e3 * (t3 - t2):.2f} ms", flush=True)
