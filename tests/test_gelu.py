"""fc1's f16x3 GELU epilogue (gemm_kernel.h gelu_fast: x erfc(-x / sqrt 2) / 2 with one branch-free erfc, the
Chebyshev erfcc fit) against float64 GELU and against torch-CPU's GELU(approximate='none'), the reference's
activation (TF/modeling_mimi.py:602-615 MimiMLP, config hidden_act "gelu").

CPU: a float32 restatement of the device formula (each operation rounded to float32 as the device rounds it; the
device's rcp / exp2 are within an ulp of these) is within the bounds below.  GPU: the device function itself, through
the diagnostic entry mimi_gelu_check, within the same bounds and within a few ulps of the restatement."""
import ctypes

import numpy as np
import pytest
import torch
from scipy import special

L2E = np.float32(1.4426950408889634)
COEF = (0.17087277, -0.82215223, 1.48851587, -1.13520398, 0.27886807, -0.18628806, 0.09678418, 0.37409196,
        1.00002368)


def gelu_fast_f32(x):
    """float32 restatement of gemm_kernel.h gelu_fast (fma as float64 product + add rounded once)."""
    f = np.float32
    x = np.asarray(x, np.float32)
    a = (np.abs(x) * f(0.70710678118654752440)).astype(np.float32)
    t = (f(1) / (f(0.5) * a.astype(np.float64) + 1.0).astype(np.float32)).astype(np.float32)
    p = np.full_like(t, f(f(COEF[0]) * L2E))
    for c in COEF[1:]:
        p = (p.astype(np.float64) * t + np.float64(f(f(c) * L2E))).astype(np.float32)
    inner = ((-a * L2E).astype(np.float32).astype(np.float64) * a + np.float64(f(f(-1.26551223) * L2E))).astype(np.float32)
    y = (t.astype(np.float64) * p + inner).astype(np.float32)
    h = (f(0.5) * (t * np.exp2(y.astype(np.float64)).astype(np.float32))).astype(np.float32)
    return (x * np.where(x > 0, f(1) - h, h)).astype(np.float32)


def _exact(x):
    x = np.asarray(x, np.float64)
    return x * 0.5 * special.erfc(-x / np.sqrt(2.0))


def _inputs():
    rng = np.random.default_rng(3)
    v = np.concatenate([np.linspace(-10, 10, 200001), rng.standard_normal(100000) * 2.0,
                        [0.0, -0.0, 1e-30, -1e-30, 1e-7, -1e-7, 5.0, -5.0, 30.0, -30.0, 1e4, -1e4]])
    return v.astype(np.float32)


def _check_bounds(x, g):
    ex = _exact(x)
    tg = torch.nn.functional.gelu(torch.from_numpy(x)).numpy().astype(np.float64)
    err = np.abs(g.astype(np.float64) - ex)
    rel = err / np.maximum(np.abs(ex), 1e-300)
    nz = ex != 0
    assert rel[(np.abs(x) < 2) & nz].max() < 1e-6  # measured ~4e-7
    assert rel[(x >= 2) & nz].max() < 3e-7  # (1 - Phi(-x) / ... : measured ~1e-7)
    assert err[x <= -2].max() < 1e-7  # tiny values: Phi(-|x|) keeps full relative precision (~1e-5 at x = -10)
    # over the whole range no larger than torch's own absolute error (its (1 + erf) form cancels for x < 0)
    assert err.max() <= np.abs(tg - ex).max()
    assert np.all(np.isfinite(g))


def test_gelu_fast_restatement_bounds():
    x = _inputs()
    _check_bounds(x, gelu_fast_f32(x))


@pytest.mark.gpu
def test_gelu_device_matches_bounds_and_restatement():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip import _lib
    lib = _lib.load()
    x = _inputs()
    xin = torch.from_numpy(x).cuda()
    out = torch.empty_like(xin)
    torch.cuda.synchronize()
    _lib.check(lib.mimi_gelu_check(ctypes.c_void_p(xin.data_ptr()), xin.numel(), ctypes.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    g = out.cpu().numpy()
    _check_bounds(x, g)
    # the same formula: the device's v_rcp / v_exp are within an ulp of the restatement's correctly rounded ones; an ulp
    # of the exp2 argument y (|y| up to ~75 at x = -10) moves Phi(-|x|) by up to 2^-17 relative, hence the 3e-5 term
    r = gelu_fast_f32(x).astype(np.float64)
    d = np.abs(g.astype(np.float64) - r)
    tol = 3e-5 * np.abs(r) + 4 * np.spacing(np.abs(r).astype(np.float32)).astype(np.float64) + 1e-37
    assert np.all(d <= tol), x[np.argmax(d / tol)]
