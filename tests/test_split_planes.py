"""GPU: the fp16 plane split every planes epilogue, the LayerNorm and conv0 use (kernels.h split2_f16s) is the exact
arithmetic definition hi = RN16(v s), lo = RN16(v s - hi) (operations exact, one rounding each), checked against
float64 numpy on edge values: zeros of both signs, fp32 and fp16 subnormals, fp16 rounding ties (both parities), the
fp16 overflow edge, and random values over the magnitudes the engine's scales produce; and the conversion form it
replaced (mul, cvt, cvt back, sub, cvt) agrees with it wherever v s is an fp32 number other than a zero."""
import ctypes

import numpy as np
import pytest
import torch


def _edge_values():
    f16 = np.finfo(np.float16)
    v = [0.0, -0.0, 1.0, -1.0, 1e-45, -1e-45, 1e-40, -1e-38, 2.0 ** -126, 2.0 ** -24, 2.0 ** -25, -2.0 ** -25,
         3 * 2.0 ** -26, 2.0 ** -14, 2.0 ** -15, float(f16.max), 65504.0 + 15.99, 65520.0, -65520.0, 1e30]
    # fp16 rounding ties: the midpoint between consecutive fp16 values, even and odd neighbours
    h = np.arange(0x3C00, 0x3C40, dtype=np.uint16).view(np.float16).astype(np.float32)
    v += list(((h[:-1] + h[1:]) / 2).astype(np.float32))
    v += list(-((h[:-1] + h[1:]) / 2).astype(np.float32))
    rng = np.random.default_rng(7)
    for e in range(-40, 17, 3):
        v += list((rng.standard_normal(512) * 2.0 ** e).astype(np.float32))
    v = np.asarray(v, np.float32)
    return v if len(v) % 2 == 0 else np.append(v, np.float32(0.5))


def _exact(v, scale):
    x = v.astype(np.float64) * scale  # exact: a float32 times a power of two
    with np.errstate(over="ignore", invalid="ignore"):
        hi = x.astype(np.float16)
        lo = (x - hi.astype(np.float64)).astype(np.float16)
    return hi.view(np.uint16), lo.view(np.uint16), np.isfinite(hi)


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [2.0 ** -14, 2.0 ** -8, 1.0, 2.0 ** 7, 2.0 ** 14])
def test_plane_split_is_exact_arithmetic(scale):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip import _lib
    lib = _lib.load()
    vals = _edge_values()
    v = torch.from_numpy(vals).cuda()
    n = v.numel() // 2
    out = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _lib.check(lib.mimi_split_check(ctypes.c_void_p(v.data_ptr()), n, scale, ctypes.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    w = out.cpu().numpy().view(np.uint32).reshape(n, 4)
    halves = lambda col: w[:, col].copy().view(np.uint16)  # noqa: E731  (pair i: values 2i, 2i + 1)
    hi, lo, fin = _exact(vals, scale)
    # the kernels' split == exact arithmetic (finite hi; past fp16's range hi is inf and lo NaN in both)
    assert np.array_equal(halves(0)[fin], hi[fin]), np.nonzero(halves(0) != hi)[0][:8]
    assert np.array_equal(halves(1)[fin], lo[fin]), [(float(vals[i]), hex(halves(1)[i]), hex(lo[i]))
                                                    for i in np.nonzero((halves(1) != lo) & fin)[0][:8]]
    # the conversion form agrees wherever v s is a nonzero fp32 number (both are exact there)
    t = (vals * np.float32(scale)).astype(np.float32)
    same = fin & (t != 0)
    assert np.array_equal(halves(2)[same], hi[same]) and np.array_equal(halves(3)[same], lo[same])
