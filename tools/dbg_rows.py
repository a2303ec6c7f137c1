"""Debug: where the row-slab fc1 output differs from the planes kernel's (taps ff0)."""
import numpy as np
import torch
from mimi_hip import synthetic
from mimi_hip.model import MimiHipModel
from mimi_hip.synthetic import make_state_dict

m = MimiHipModel(make_state_dict(seed=0), device="cuda:0")
x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=401)).cuda()
out = {}
for mask in (0, 1, 0, 1):
    m.set_option("gemm_rows", mask)
    m.set_taps(True)
    c = m.encode_int32(x, 32).cpu().numpy()
    t = {k: m.get_tap(k).copy() for k in ("ff0", "xfmr0", "encoder")}
    m.set_taps(False)
    out.setdefault(mask, []).append((c, t))
a, b = out[0][0][1]["ff0"], out[1][0][1]["ff0"]
print("run-to-run mask0 equal:", np.array_equal(out[0][0][1]["ff0"], out[0][1][1]["ff0"]),
      "mask1 equal:", np.array_equal(out[1][0][1]["ff0"], out[1][1][1]["ff0"]))
print("shape", a.shape)
a2 = a.reshape(-1, a.shape[-1]); b2 = b.reshape(-1, b.shape[-1])
d = a2 != b2
rows = np.nonzero(d.any(1))[0]; cols = np.nonzero(d.any(0))[0]
print("mismatch", d.sum(), "rows", len(rows), rows[:20], rows[-20:], "cols", len(cols), cols[:20])
print("rows mod 256 hist", np.bincount(rows % 256, minlength=256).nonzero()[0][:40])
print("cols mod 128", np.bincount(cols % 128, minlength=128).nonzero()[0][:40])
i = np.argwhere(d)[:10]
for r, cc in i:
    print(r, cc, a2[r, cc], b2[r, cc])
print("max rel", np.abs(a2 - b2).max() / np.abs(a2).max())
