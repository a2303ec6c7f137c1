"""LayerNorm prologue of the small-batch q/k/v and fc1 GEMMs (gemm_planes.h FL_LNA): bit-identical to the LayerNorm
kernel + GEMM pair it replaces.

On small grids (batch 1-4 of 10 s) every q/k/v and fc1 tile computes LayerNorm (TF/modeling_mimi.py:737-738,
`input_layernorm` / `post_attention_layernorm` in MimiTransformerLayer.forward :851-869) of its own rows with the
LayerNorm kernel's arithmetic (kernels.h ln_row_coeffs) and feeds its fp16 planes to the MFMAs from LDS.  The
q/k/v outputs of every layer (taps "qkv0".."qkv7", fp32 after RoPE), the transformer output and all 32 codebooks
must be equal BITWISE across the "ln_fused" option (0: LayerNorm launches, 1: fc1 prologue, 2 / 3 / 4: fc1 and q/k/v
prologues, q/k/v on 16x64 / 32x64 / 16x128 tiles), for every small-grid tile
(16-, 32- and 64-row tiles: B = 1, 2, 4 at 10 s, a 1-sample clip, a length that leaves a partial tile), and the
graph-replayed encode must give the same codes.  The ragged batch (LayerNorm kernel on packed rows, large grid)
must equal per-utterance encodes (which take the prologue) -- the batch-invariance contract of
test_ragged.py, here with both settings.
"""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.config import encoded_length

pytestmark = pytest.mark.gpu
TAPS = ["qkv%d" % i for i in range(8)] + ["xfmr7"]


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("ln_fused", 1)


def run(engine, variant, xt, K=32):
    engine.set_option("ln_fused", variant)
    engine.set_taps(True)
    try:
        codes = engine.encode_int32(xt, K).cpu().numpy()
        return codes, {t: engine.get_tap(t).copy() for t in TAPS}
    finally:
        engine.set_taps(False)


@pytest.mark.parametrize("B,L", [(1, 240000), (2, 240000), (4, 240000), (1, 1), (3, 24000 * 7 + 11)])
def test_ln_prologue_bitwise(engine, B, L):
    x = torch.from_numpy(np.stack([synthetic.speech_like(L, 71, i) for i in range(B)])).cuda()
    c0, t0 = run(engine, 0, x)
    for v in (1, 2, 3, 4):
        c1, t1 = run(engine, v, x)
        for name in TAPS:
            assert np.array_equal(t0[name], t1[name]), (v, name, int((t0[name] != t1[name]).sum()), t0[name].size)
        assert np.array_equal(c0, c1), (v, int((c0 != c1).sum()))
        assert c1.shape == (B, 32, encoded_length(L))


def test_ln_prologue_graph_replay(engine):
    x = torch.from_numpy(np.stack([synthetic.speech_like(240000, 72, 0)])).cuda()
    ref, _ = run(engine, 0, x)
    engine.set_option("ln_fused", 2)
    before = engine.graph_replays
    outs = [engine.encode_int32(x, 32).cpu().numpy() for _ in range(3)]
    assert engine.graph_replays > before
    for o in outs:
        assert np.array_equal(o, ref)


def test_ln_prologue_ragged_equals_single(engine):
    """Per-utterance encodes with the prologue equal the same clips in one ragged batch through the LayerNorm kernel."""
    lengths = [24000 * 10, 24000 * 4 + 333, 961, 24000 * 13 + 5]
    clips = [synthetic.speech_like(L, 73, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    engine.set_option("ln_fused", 0)
    rag = engine.encode_ragged(torch.from_numpy(x).cuda(), lengths, 32).cpu().numpy()
    engine.set_option("ln_fused", 2)
    for i, c in enumerate(clips):
        one = engine.encode_int32(torch.from_numpy(c[None]).cuda(), 32).cpu().numpy()
        F = encoded_length(len(c))
        assert np.array_equal(one[0], rag[i, :, :F]), (i, len(c))


def test_ln_option_rejects_bad_value(engine):
    from mimi_hip._lib import MimiHipError
    with pytest.raises(MimiHipError):
        engine.set_option("ln_fused", 5)
