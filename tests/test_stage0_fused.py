"""Stage 0 fused with down conv 0 (resblock.hip stage0_fused_h16_kernel): bit-identical to the two-kernel path.

The fused kernel keeps y (the stage-0 block's output) on chip and runs down conv 0 (TF/modeling_mimi.py:269-279,
k = 8, s = 4) from it; every y plane value and every down-conv MFMA is the one the unfused pair computes, so the
fp32 output x1 (tap "down0"), y itself (tap "res0_elu", stored only when taps are on) and all 32 codebooks must be
equal BITWISE across the two settings of the "stage0_fused" option (0: two kernels, 1: fused) -- uniform batches whose lengths are not multiples of the 32-step block or the stride, ragged
batches (edge lengths 1 / 961 / 1921 ...), and long items whose per-wave ranges start mid-item (the halo
recompute).  The graph-replayed encode (taps off) must give the same codes.
"""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.config import encoded_length

pytestmark = pytest.mark.gpu
VARIANTS = (0, 1)


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("stage0_fused", 1)


def run(engine, variant, fn):
    engine.set_option("stage0_fused", variant)
    engine.set_taps(True)
    try:
        codes = fn()
        return codes, engine.get_tap("down0").copy(), engine.get_tap("res0_elu").copy()
    finally:
        engine.set_taps(False)


def check_identical(results, lengths=None):
    c0, x0, y0 = results[0]
    for v, (c, x, y) in zip(VARIANTS[1:], results[1:]):
        if lengths is None:
            assert np.array_equal(x, x0), (v, int((x != x0).sum()), x.size)
            assert np.array_equal(y, y0), (v, int((y != y0).sum()))
            assert np.array_equal(c, c0), (v, int((c != c0).sum()))
        else:  # ragged: compare each item's valid rows
            for i, L in enumerate(lengths):
                T0, T1, F = L, (L + 3) // 4, encoded_length(L)
                assert np.array_equal(x[i, :T1], x0[i, :T1]), (v, i, L, int((x[i, :T1] != x0[i, :T1]).sum()))
                assert np.array_equal(y[i, :T0], y0[i, :T0]), (v, i, L)
                assert np.array_equal(c[i, :, :F], c0[i, :, :F]), (v, i, L)


@pytest.mark.parametrize("B,L", [(3, 24000 * 3 + 7), (1, 1), (2, 1921), (2, 24000 * 60 + 13)])
def test_fused_stage0_uniform_bitwise(engine, B, L):
    x = np.stack([synthetic.speech_like(L, 61, i) for i in range(B)])[:, None]
    xt = torch.from_numpy(x).cuda()
    res = [run(engine, v, lambda: engine.encode_int32(xt[:, 0], 32).cpu().numpy()) for v in VARIANTS]
    assert res[0][1].shape == (B, (L + 3) // 4, 128)
    check_identical(res)


def test_fused_stage0_ragged_bitwise(engine):
    lengths = [1, 960, 961, 1919, 1921, 33333, 240000, 24000 * 20 + 5]
    clips = [synthetic.speech_like(L, 62, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    res = [run(engine, v, lambda: engine.encode_ragged(xt, lengths, 32).cpu().numpy()) for v in VARIANTS]
    check_identical(res, lengths)


def test_fused_stage0_graph_replay_same_codes(engine):
    """Taps off (the product path, graph-captured on the 2nd encode of a shape, replayed on the 3rd): the same
    codes as the taps-on two-kernel encode."""
    x = torch.from_numpy(np.stack([synthetic.speech_like(48000, 63, i) for i in range(4)])).cuda()
    ref, _, _ = run(engine, 0, lambda: engine.encode_int32(x, 32).cpu().numpy())
    engine.set_option("stage0_fused", 1)
    before = engine.graph_replays
    outs = [engine.encode_int32(x, 32).cpu().numpy() for _ in range(3)]
    assert engine.graph_replays > before
    for o in outs:
        assert np.array_equal(o, ref)


def test_set_option_rejects_unknown(engine):
    from mimi_hip._lib import MimiHipError
    with pytest.raises(MimiHipError):
        engine.set_option("stage0_fused", 2)
    with pytest.raises(MimiHipError):
        engine.set_option("no_such_option", 1)
