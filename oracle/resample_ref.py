"""ORACLE — test infrastructure only, never shipped, never on the product path.

CPU restatement of the host-ingest resampler on the shard scripts' load path: ``librosa.load(path, sr=24000)``
(``librispeech-mimi/utils.py:84-87``, ``emilia-mimi/process_shard.py:479-482``, ``yodas2-mimi/process_shard.py:389``)
resamples with ``librosa.resample``.  librosa is third-party and NOT installed here, so the
default ``res_type='soxr_hq'`` (libsoxr) cannot be pinned: parity with it is UNPINNED.  What is pinned is
librosa's ``res_type='polyphase'`` mode, which (librosa 0.10 ``core/audio.py`` ``resample``) is
``scipy.signal.resample_poly(y, target_sr // g, orig_sr // g, axis=-1)`` followed by ``fix_length`` to
``ceil(n * target_sr / orig_sr)`` samples (no scaling by default); scipy 1.15.3 is installed, so the fixtures
and the tests check against scipy itself.

``resample_poly_ref`` restates scipy 1.15.3 ``signal/_signaltools.py`` ``resample_poly`` (padtype
'constant', cval 0, the default Kaiser(5.0) window) with the accumulation order of its ``upfirdn`` inner
loop (``signal/_upfirdn_apply.pyx`` ``_apply_impl``): for output m at up-sampled position p = m * down, the
products ``x[j] * h[p - j * up]`` (each rounded to float32) are added to a 0-initialised float32 accumulator
in ASCENDING input index j.  It is a pure-numpy loop over taps, vectorised over outputs, and is bit-exact
with scipy on float32 input (tests/test_resample.py).
"""
import math

import numpy as np
from scipy.signal import firwin


def design_filter(up: int, down: int, dtype=np.float32):
    """(h, n_pre_pad, half_len) exactly as resample_poly builds it: firwin(2*half_len+1, 1/max_rate,
    window=('kaiser', 5.0)) cast to x's dtype, times up, with n_pre_pad zeros in front."""
    max_rate = max(up, down)
    half_len = 10 * max_rate
    h = firwin(2 * half_len + 1, 1.0 / max_rate, window=("kaiser", 5.0)).astype(dtype)
    h *= up
    n_pre_pad = down - half_len % down
    return h, n_pre_pad, half_len


def resample_poly_ref(x: np.ndarray, up: int, down: int) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32)
    g = math.gcd(up, down)
    up //= g
    down //= g
    if up == down == 1:
        return x.copy()
    n_in = len(x)
    n_out = -(-n_in * up // down)
    h, n_pre_pad, half_len = design_filter(up, down)
    hp = np.concatenate([np.zeros(n_pre_pad, np.float32), h])  # post-padding zeros contribute nothing
    n_pre_remove = (half_len + n_pre_pad) // down
    m = np.arange(n_pre_remove, n_pre_remove + n_out, dtype=np.int64)
    p = m * down
    j_hi = np.minimum(p // up, n_in - 1)                       # largest j with p - j*up >= 0
    j_lo = np.maximum(-((len(hp) - 1 - p) // up), 0)          # smallest j with p - j*up < len(hp)
    acc = np.zeros(n_out, np.float32)
    span = int((j_hi - j_lo).max()) + 1 if n_out else 0
    for t in range(span):
        j = j_lo + t
        ok = j <= j_hi
        jj = np.where(ok, j, 0)
        term = (x[jj] * hp[np.where(ok, p - jj * up, 0)]).astype(np.float32)
        acc = np.where(ok, (acc + term).astype(np.float32), acc)
    return acc


def librosa_polyphase_ref(y: np.ndarray, orig_sr: int, target_sr: int) -> np.ndarray:
    """librosa.resample(y, orig_sr=, target_sr=, res_type='polyphase') on float32 mono (restated)."""
    y = np.asarray(y, dtype=np.float32)
    if orig_sr == target_sr:
        return y
    g = math.gcd(orig_sr, target_sr)
    out = resample_poly_ref(y, target_sr // g, orig_sr // g)
    n = int(math.ceil(len(y) * float(target_sr) / orig_sr))
    if len(out) > n:
        out = out[:n]
    elif len(out) < n:
        out = np.concatenate([out, np.zeros(n - len(out), np.float32)])
    return out
