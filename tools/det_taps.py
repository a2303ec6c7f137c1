"""Determinism bisect: encode the padded B=32 golden batch twice with taps on; report the first tap that differs."""
import json
import sys
import numpy as np
import torch
sys.path.insert(0, "tokenize-audio_amd")
from mimi_hip import synthetic
from mimi_hip.model import MimiHipModel
m = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=32), device="cuda:0")
meta = json.load(open("tests/golden/golden_batch_meta.json"))
audio = [synthetic.speech_like(L, meta["audio_seed"], meta["audio_index0"] + i) *
         np.float32(meta["quiet_gain"].get(str(i), 1.0)) for i, L in enumerate(meta["lengths"])]
lmax = max(len(a) for a in audio)
x = np.zeros((len(audio), lmax), np.float32)
for i, a in enumerate(audio):
    x[i, :len(a)] = a
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
xd = torch.from_numpy(x[:B]).cuda()
names = ["conv0", "res0_elu", "down0", "res1_elu", "down1", "res2_elu", "down2", "res3_elu", "down3_elu", "encoder",
         "qkv0", "att0", "oproj0", "ff0"] + [f"xfmr{i}" for i in range(8)] + ["downsample", "proj"]
m.set_taps(True)
runs = []
for r in range(3):
    c = m.encode_int32(xd, 32).cpu()
    runs.append(({n: m.get_tap(n).copy() for n in names}, c))
runs[0][0]["qkv0"].astype(np.float32).tofile("gpurun_out/qkv0.bin")
print("qkv0", runs[0][0]["qkv0"].shape, flush=True)
for r in (1, 2):
    first = None
    for n in names:
        a, b = runs[0][0][n], runs[r][0][n]
        d = np.argwhere(a != b)
        if len(d):
            print(f"run {r}: tap {n} differs at {len(d)} elements, first {d[:3].tolist()}, max|d| {np.abs(a-b).max():.3e}", flush=True)
            if first is None:
                first = n
    print(f"run {r}: first differing tap {first}; codes differ {(runs[0][1] != runs[r][1]).sum().item()}", flush=True)
