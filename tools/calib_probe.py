"""Do explicit (mimi_calibrate) and implicit (first encode) f16x3 calibrations give the same activation scales?"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))
from mimi_hip import synthetic  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402

sd = synthetic.make_state_dict(seed=0)
a = MimiHipModel(sd, device="cuda:0")
x = torch.from_numpy(synthetic.clip_batch(2, 48000, seed=5)).cuda()
ca = a.encode_int32(x, 32).cpu().numpy()
b = a.clone()
b.calibrate()
c = a.clone()
cc = c.encode_int32(x, 32).cpu().numpy()
cb = b.encode_int32(x, 32).cpu().numpy()
sa, sb, sc = a.act_scales(), b.act_scales(), c.act_scales()
print("slots", len(sa), len(sb), len(sc))
print("explicit vs implicit scale diffs:", [(k, sa[k][0], sb.get(k, (None,))[0]) for k in sa if sb.get(k, (None,))[0] != sa[k][0]][:10])
print("implicit clone diffs:", [(k, sa[k][0], sc.get(k, (None,))[0]) for k in sa if sc.get(k, (None,))[0] != sa[k][0]][:10])
print("codes equal a/b/c:", np.array_equal(ca, cb), np.array_equal(ca, cc))
