"""The LayerNorm output bound the engine uses to skip the f16x3 range check of a LayerNorm output
(engine.cpp DevXfmr::ln*_bound): |LN(x)_c| <= |gamma_c| sqrt(D - 1) + |beta_c| for every input row, because a
normalised value (x_c - mean) / sqrt(var + eps) never exceeds sqrt(D - 1) in magnitude (equality for a one-hot row,
eps = 0).  Checked here in float32 with torch's layer_norm (the reference's op, TF/modeling_mimi.py:737-738) on the
rows that come closest to the bound: one-hot rows of every scale, the same with a constant offset, rows with two
outliers, and random rows -- the engine's 1.001 margin must cover the rounding."""
import numpy as np
import torch

D = 512


def bound(g, b):
    return np.max(np.abs(g.astype(np.float64)) * np.sqrt(D - 1) * 1.001 + np.abs(b.astype(np.float64)))


def test_layernorm_output_bound_holds_on_extreme_rows():
    rng = np.random.default_rng(0)
    g = rng.normal(0, 1.5, D).astype(np.float32)
    b = rng.normal(0, 0.5, D).astype(np.float32)
    rows = []
    for scale in (1e-3, 1.0, 1e3, 1e6):
        for c in (0, 7, 511):
            r = np.zeros(D, np.float32)
            r[c] = scale
            rows += [r, r + 3.0 * scale, -r]
        two = np.zeros(D, np.float32)
        two[[1, 2]] = scale
        rows.append(two)
    rows += list(rng.standard_t(1.5, (256, D)).astype(np.float32))
    x = torch.from_numpy(np.stack(rows))
    y = torch.nn.functional.layer_norm(x, (D,), torch.from_numpy(g), torch.from_numpy(b), eps=1e-5).numpy()
    assert np.all(np.isfinite(y))
    assert float(np.abs(y).max()) <= bound(g, b)
    # the one-hot rows come within 1 % of it: the bound is not loose where it matters
    per_c = np.abs(g) * np.sqrt(D - 1) + np.abs(b)
    assert float(np.max(np.abs(y) / per_c[None, :])) > 0.99


def test_bound_skips_the_check_only_below_half_the_plane_limit():
    # the engine skips when bound * scale < 2^14 (half of the 2^15 at which an fp16 plane value can overflow)
    g = np.ones(D, np.float32)
    b = np.zeros(D, np.float32)
    bd = bound(g, b)
    assert 22.6 < bd < 22.7
    assert bd * 2.0 ** 9 < 2 ** 14 <= bd * 2.0 ** 10
