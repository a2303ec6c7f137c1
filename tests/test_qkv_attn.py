"""Fused q/k/v projection + RoPE + attention (qkv_attn.hip): bit-identical to the q/k/v GEMM + attention kernel pair.

For batches of items up to 256 frames (10.24 s) with at least 256 (item, head) pairs the engine runs one kernel per
layer that computes a head's q/k/v columns (TF/modeling_mimi.py:657-726 q_proj / k_proj / v_proj + apply_rotary_pos_emb)
and its causal sliding-window attention (MimiAttention.forward) without the fp32 q/k/v tensor leaving the CU.  Every
fp32 q/k/v value is formed with the q/k/v GEMM's instruction sequence and the attention with
attention_t256_h16_kernel's, so the q/k/v taps ("qkv0".."qkv7", written only when taps are on), the attention output
planes ("att0".."att7"), the transformer output and all 32 codebooks must be equal BITWISE across the "qkv_attn"
option (0: two kernels; 1: fused for large batches; 2: fused whenever the items fit) and "qkv_attn_xcd" -- on the
uniform B = 32 x 10 s headline batch, on small forced batches with partial 32-query tiles and a 1-frame item, on
ragged batches, and through graph replays.  An item alone (batch 1: never fused) equals the same item inside a fused
batch (test_full_size_batch_properties covers B = 1 vs B = 32; here a ragged case).
"""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.config import encoded_length

pytestmark = pytest.mark.gpu
TAPS = ["qkv%d" % i for i in range(8)] + ["att%d" % i for i in range(8)] + ["xfmr7"]


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("qkv_attn", 1)
    m.set_option("qkv_attn_xcd", 1)


def run(engine, variant, x, K=32, taps=True, xcd=1):
    engine.set_option("qkv_attn", variant)
    engine.set_option("qkv_attn_xcd", xcd)
    engine.set_taps(taps)
    try:
        codes = engine.encode_int32(x, K).cpu().numpy()
        return codes, ({t: engine.get_tap(t).copy() for t in TAPS} if taps else {})
    finally:
        engine.set_taps(False)
        engine.set_option("qkv_attn", 1)
        engine.set_option("qkv_attn_xcd", 1)


def same(a, b, what):
    c0, t0 = a
    c1, t1 = b
    for name in t0:
        assert np.array_equal(t0[name], t1[name]), (what, name, int((t0[name] != t1[name]).sum()), t0[name].size)
    assert np.array_equal(c0, c1), (what, int((c0 != c1).sum()))


def test_fused_headline_batch_bitwise(engine):
    x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=301)).cuda()
    ref = run(engine, 0, x)
    same(ref, run(engine, 1, x), "auto")
    same(ref, run(engine, 1, x, xcd=0), "xcd 0")
    assert ref[0].shape == (32, 32, 125)


@pytest.mark.parametrize("B,L", [(2, 240000), (3, 24000 * 7 + 11), (2, 1), (5, 245760)])
def test_fused_forced_small_batches_bitwise(engine, B, L):
    """qkv_attn = 2 fuses batches of any size: partial 32-query tiles (T = 88), one frame, T = 256 exactly."""
    x = torch.from_numpy(np.stack([synthetic.speech_like(L, 302, i) for i in range(B)])).cuda()
    ref = run(engine, 0, x)
    got = run(engine, 2, x)
    same(ref, got, (B, L))
    assert got[0].shape == (B, 32, encoded_length(L))


def test_fused_ragged_bitwise_and_equals_single(engine):
    """A ragged batch of 32 items <= 10.24 s (packed rows, per-item lengths) through the fused kernel equals the
    two-kernel path bitwise, and each item equals its own batch-1 encode."""
    rng = np.random.default_rng(303)
    lengths = [int(v) for v in rng.integers(1, 245760, 32)]
    lengths[0], lengths[1] = 245760, 1
    clips = [synthetic.speech_like(L, 304, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    engine.set_option("qkv_attn", 0)
    ref = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    engine.set_option("qkv_attn", 1)
    got = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    assert np.array_equal(ref, got), int((ref != got).sum())
    for i in (0, 1, 7, 20):
        one = engine.encode_int32(torch.from_numpy(clips[i][None]).cuda(), 32).cpu().numpy()
        F = encoded_length(lengths[i])
        assert np.array_equal(one[0], got[i, :, :F]), (i, lengths[i])


def test_fused_ragged_with_long_item_unfused(engine):
    """An item over 256 frames sends the whole ragged batch through the two-kernel path (banded attention for it):
    the codes are those of qkv_attn = 0."""
    lengths = [24000 * 10] * 31 + [24000 * 13 + 5]
    clips = [synthetic.speech_like(L, 305, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    engine.set_option("qkv_attn", 0)
    ref = engine.encode_ragged(xt, lengths, 8).cpu().numpy()
    engine.set_option("qkv_attn", 1)
    got = engine.encode_ragged(xt, lengths, 8).cpu().numpy()
    assert np.array_equal(ref, got)


def test_fused_graph_replay(engine):
    x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=306)).cuda()
    ref, _ = run(engine, 0, x, taps=False)
    before = engine.graph_replays
    outs = [engine.encode_int32(x, 32).cpu().numpy() for _ in range(3)]
    assert engine.graph_replays > before
    for o in outs:
        assert np.array_equal(o, ref)


def test_qkv_attn_option_rejects_bad_value(engine):
    from mimi_hip._lib import MimiHipError
    with pytest.raises(MimiHipError):
        engine.set_option("qkv_attn", 3)
    with pytest.raises(MimiHipError):
        engine.set_option("qkv_attn_xcd", 2)
