"""Generate tests/golden/resample.npz: scipy.signal.resample_poly (scipy 1.15.3, the algorithm behind librosa's
res_type='polyphase') on seeded float32 clips, for the host-ingest resampler (mimi_hip.ingest, HIP kernel
resample_poly_kernel) and its oracle restatement (oracle/resample_ref.py).  librosa itself is absent, so its
fix_length step is applied as restated there (ceil(n * target / orig) samples, zero-padded / truncated).

    python tests/golden/make_resample_golden.py
"""
import math
import os

import numpy as np
from scipy.signal import resample_poly

HERE = os.path.dirname(os.path.abspath(__file__))
RATES = [16000, 8000, 22050, 44100, 48000]
LENGTHS = [1, 2, 3, 37, 1001, 16001]
TARGET = 24000


def clip(rate, n):
    return np.random.default_rng(rate * 100003 + n).normal(0.0, 0.3, n).astype(np.float32)


def main():
    out = {}
    for r in RATES:
        g = math.gcd(r, TARGET)
        for n in LENGTHS:
            y = resample_poly(clip(r, n), TARGET // g, r // g)
            m = int(math.ceil(n * (float(TARGET) / r)))  # librosa: ratio first
            y = y[:m] if len(y) >= m else np.concatenate([y, np.zeros(m - len(y), np.float32)])
            assert y.dtype == np.float32
            out[f"r{r}_n{n}"] = y
    np.savez_compressed(os.path.join(HERE, "resample.npz"), **out)
    print(f"wrote resample.npz ({len(out)} clips)")


if __name__ == "__main__":
    main()
