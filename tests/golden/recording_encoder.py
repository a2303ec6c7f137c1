"""A recording stand-in for ``MimiEncoder`` used to pin the YODAS2 segmenter / batch scheduler.

It returns deterministic, content-dependent int64 codes of the reference wrapper's shapes ([K, ceil(L/1920)]
per array) and logs every call with its lengths, so the golden fixture captures the reference scheduler's
exact slicing, batching and long-chunk splitting (``yodas2-mimi/process_shard.py:373-533``).  Test
infrastructure only.
"""
import math

import numpy as np

K = 8


def fake_codes(a: np.ndarray) -> np.ndarray:
    L = len(a)
    T = int(math.ceil(L / 1920))
    t = np.arange(T)
    x = np.abs(a[np.minimum(t * 1920, L - 1)].astype(np.float64))
    base = np.round(x * 1e6).astype(np.int64) + 7 * t + L
    return np.stack([(base + 131 * k) % 2048 for k in range(K)]).astype(np.int64)


class RecordingEncoder:
    def __init__(self):
        self.calls = []

    def encode_audio_chunk(self, audio_array, sample_rate=24000):
        self.calls.append(["chunk", [int(len(audio_array))]])
        return fake_codes(np.asarray(audio_array))

    def encode_audio_batch(self, audio_arrays, sample_rate=24000):
        self.calls.append(["batch", [int(len(a)) for a in audio_arrays]])
        return [fake_codes(np.asarray(a)) for a in audio_arrays]
