"""Banded attention for items over 256 frames (clips over 10.24 s; ops.hip attention_band_h16_kernel): every chunk's
contribution is formed on its own and folded in ascending chunk order, so the two decompositions -- 128-query
workgroups sharing each chunk image (large grids) and one 32-query tile per workgroup with the chunks spread over its
4 waves (small grids: a batch-1 utterance) -- give the same values bit for bit.  The engine picks one by grid size
(option "attn_band_split": 0 never, 1 auto, 2 always); the attention output planes ("att0".."att7") and all 32
codebooks must not depend on it, nor an utterance's codes on its batch (TF/modeling_mimi.py:687-726 MimiAttention with
the window-250 causal mask of masking_utils.py:76-101; long-clip parity against the oracle is test_gpu_parity.py's)."""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.config import encoded_length

pytestmark = pytest.mark.gpu
TAPS = ["att%d" % i for i in range(8)]


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("attn_band_split", 1)


def run(engine, split, x, K=32):
    engine.set_option("attn_band_split", split)
    engine.set_taps(True)
    try:
        c = engine.encode_int32(x, K).cpu().numpy()
        return c, {t: engine.get_tap(t).copy() for t in TAPS}
    finally:
        engine.set_taps(False)
        engine.set_option("attn_band_split", 1)


@pytest.mark.parametrize("B,L", [(1, 24000 * 15 + 500), (2, 24000 * 20 + 7), (1, 24000 * 30), (3, 245761)])
def test_band_decompositions_bitwise(engine, B, L):
    x = torch.from_numpy(np.stack([synthetic.speech_like(L, 601, i) for i in range(B)])).cuda()
    ref = run(engine, 0, x)
    for split in (1, 2):
        got = run(engine, split, x)
        for t in TAPS:
            assert np.array_equal(ref[1][t].view(np.uint32), got[1][t].view(np.uint32)), (split, t)
        assert np.array_equal(ref[0], got[0]), (split, int((ref[0] != got[0]).sum()))
    assert ref[0].shape == (B, 32, encoded_length(L))


def test_band_item_alone_equals_item_in_batch(engine):
    """A ragged batch of 32 items, some over 10.24 s (the 128-query form: 32 x 8 x 4 workgroups), against each
    long item encoded alone (the one-tile form) and the whole batch with the one-tile form forced."""
    rng = np.random.default_rng(602)
    lengths = [int(v) for v in rng.integers(24000, 24000 * 20, 32)]
    lengths[0], lengths[1] = 24000 * 20, 245761
    clips = [synthetic.speech_like(L, 603, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    got = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    engine.set_option("attn_band_split", 2)
    try:
        forced = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    finally:
        engine.set_option("attn_band_split", 1)
    for i, L in enumerate(lengths):
        F = encoded_length(L)
        assert np.array_equal(got[i, :, :F], forced[i, :, :F]), i
    for i in [i for i, L in enumerate(lengths) if L > 245760][:4] + [1]:
        one = engine.encode_int32(torch.from_numpy(clips[i][None]).cuda(), 32).cpu().numpy()
        F = encoded_length(lengths[i])
        assert np.array_equal(one[0], got[i, :, :F]), (i, lengths[i])


def test_band_split_option_rejects_bad_value(engine):
    from mimi_hip._lib import MimiHipError
    with pytest.raises(MimiHipError):
        engine.set_option("attn_band_split", 3)
