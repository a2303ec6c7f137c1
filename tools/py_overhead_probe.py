import sys, time, ctypes
sys.path.insert(0, "tokenize-audio_amd")
import numpy as np, torch
from mimi_hip import synthetic
from mimi_hip.model import MimiHipModel
from mimi_hip.config import encoded_length
m = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=32), device="cuda:0")
a = synthetic.speech_like(372000, 1, 0)
def t(name, f, n=2000):
    t0 = time.perf_counter()
    for _ in range(n): f()
    print(f"{name}: {1e6*(time.perf_counter()-t0)/n:.2f} us", flush=True)
t("check_k", lambda: m._check_k(32))
t("ascontig", lambda: np.ascontiguousarray(a[None], dtype=np.float32))
t("encoded_length", lambda: encoded_length(372000, m.config))
t("np.empty", lambda: np.empty((1, 32, 388), dtype=np.int32))
t("_stream", lambda: m._stream())
t("current_stream", lambda: torch.cuda.current_stream(m.device))
t("astype", lambda: np.empty((32, 388), np.int32).astype(np.int64))
t("no_grad", lambda: torch.no_grad().__enter__())
t("mimi_encoded_length_cfg", lambda: m._lib.mimi_encoded_length_cfg(ctypes.byref(m._cfg_c), 372000))
x = a[None]
for _ in range(3): m.encode_host(x, 32)
t("encode_host", lambda: m.encode_host(x, 32), n=50)
