"""o_proj + layer scale + residual and the post-attention LayerNorm in one kernel (oproj_ln.hip): bit-identical to the
o_proj planes GEMM + LayerNorm launch it replaces on large batches.

MimiTransformerLayer.forward (TF/modeling_mimi.py:851-869): the residual stream after `self_attn_layer_scale(o_proj(
attn))` ("oproj0".."oproj7"), the fc1 output that reads the post_attention_layernorm planes ("ff0".."ff7"), the
transformer output and all 32 codebooks must be equal BITWISE across the "oproj_ln" option, on the B = 32 x 10 s
headline batch, on a ragged batch (packed rows, a row count that ends inside a 32-row slab) with each item equal to
its own batch-1 encode, and through graph replays.  Opt-in (default 0): slower than the two kernels
(profiles/r4v_ab_oproj_ln.txt).
"""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.config import encoded_length

pytestmark = pytest.mark.gpu
TAPS = ["oproj%d" % i for i in range(8)] + ["ff%d" % i for i in range(8)] + ["xfmr7"]


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("oproj_ln", 0)


def run(engine, v, x, K=32):
    engine.set_option("oproj_ln", v)
    engine.set_taps(True)
    try:
        codes = engine.encode_int32(x, K).cpu().numpy()
        return codes, {t: engine.get_tap(t).copy() for t in TAPS}
    finally:
        engine.set_taps(False)
        engine.set_option("oproj_ln", 0)


def test_oproj_ln_headline_batch_bitwise(engine):
    x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=601)).cuda()
    c0, t0 = run(engine, 0, x)
    c1, t1 = run(engine, 1, x)
    for name in TAPS:
        assert np.array_equal(t0[name], t1[name]), (name, int((t0[name] != t1[name]).sum()))
    assert np.array_equal(c0, c1), int((c0 != c1).sum())
    one = engine.encode_int32(x[5:6], 32).cpu().numpy()  # (batch 1: the two kernels)
    assert np.array_equal(one[0], c1[5])


def test_oproj_ln_ragged_bitwise(engine):
    rng = np.random.default_rng(602)
    lengths = [int(v) for v in rng.integers(1, 24000 * 14, 40)]
    lengths[0], lengths[1] = 24000 * 14, 3
    clips = [synthetic.speech_like(L, 603, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    engine.set_option("oproj_ln", 0)
    ref = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    engine.set_option("oproj_ln", 1)
    got = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    engine.set_option("oproj_ln", 0)
    assert np.array_equal(ref, got), int((ref != got).sum())
    for i in (0, 1, 17):
        one = engine.encode_int32(torch.from_numpy(clips[i][None]).cuda(), 32).cpu().numpy()
        F = encoded_length(lengths[i])
        assert np.array_equal(one[0], got[i, :, :F]), (i, lengths[i])


def test_oproj_ln_graph_replay(engine):
    x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=604)).cuda()
    engine.set_option("oproj_ln", 0)
    ref = engine.encode_int32(x, 8).cpu().numpy()
    engine.set_option("oproj_ln", 1)
    try:
        before = engine.graph_replays
        outs = [engine.encode_int32(x, 8).cpu().numpy() for _ in range(3)]
        assert engine.graph_replays > before
    finally:
        engine.set_option("oproj_ln", 0)
    for o in outs:
        assert np.array_equal(o, ref)
