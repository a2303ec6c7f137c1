"""Diagnose MimiEncoder concurrency=2 vs 1 on encode_audio_chunks (tests/test_gpu_parity.py
test_pipeline_engines_alternate_same_codes): items whose codes differ from their batch-1 encode, per setting of the
persistent RVQ chain, over several repetitions."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tokenize-audio_amd"), os.path.join(ROOT, "tests")]
from mimi_hip import synthetic  # noqa: E402
from mimi_hip.encoder import MimiEncoder  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402

m = MimiHipModel(synthetic.make_state_dict(seed=0), device="cuda:0")
rng = np.random.default_rng(17)
lens = [int(x) for x in rng.integers(1, 24000 * 16, size=14)]
audio = [synthetic.speech_like(L, 41, i) for i, L in enumerate(lens)]
one = MimiEncoder(device="cuda:0", model=m, concurrency=1, chunk_batch=3)
two = MimiEncoder(device="cuda:0", model=m, concurrency=2, chunk_batch=3)
alone = [one.encode_audio_chunk(a, 24000) for a in audio]
two.encode_audio_chunks(audio, 24000)  # (creates the second engine)
for setting in sys.argv[1:] or ["chain1", "chain0", "chain1"]:
    for e in two._engines:
        e.set_option("rvq_chain", 1 if setting == "chain1" else 0)
    bad_total = 0
    for rep in range(int(os.environ.get("REPS", "8"))):
        got = two.encode_audio_chunks(audio, 24000)
        bad = [i for i, (g, a) in enumerate(zip(got, alone)) if not np.array_equal(g, a)]
        bad_total += len(bad)
        if bad:
            i = bad[0]
            d = np.argwhere(got[i] != alone[i])
            print(f"  {setting} rep {rep}: items {bad}; item {i} first diffs {d[:3].tolist()}", flush=True)
    print(setting, "mismatching items over reps:", bad_total, "chain reruns", [e.rvq_chain_reruns for e in two._engines],
          flush=True)
