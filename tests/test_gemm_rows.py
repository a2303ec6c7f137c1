"""Row-slab GEMM for the large-batch transformer linears (gemm_rows.h): bit-identical to the planes kernel it
replaces.

fc1 + GELU (TF/modeling_mimi.py MimiMLP.fc1 / activation_fn), fc2 and o_proj with the layer scale and residual
(MimiTransformerLayer.forward :851-869, MimiLayerScale) run, on large grids, as row slabs whose waves own 16 rows x
all the tile's columns, the A fragments loaded straight into registers and only the weight planes staged in LDS.
Every output element is formed with the planes kernel's instruction sequence, so the fc1 output planes ("ff0".."ff7"),
the residual stream after o_proj and fc2 ("oproj0".., "xfmr0"..), and all 32 codebooks must be equal BITWISE for
every setting of the "gemm_rows" option (bit 0 fc1, bit 1 fc2, bit 2 o_proj; default 0: slower than the planes kernel
on these shapes, profiles/r4p_ab_gemm_rows.txt), on the B = 32 x 10 s headline batch, a
ragged batch (packed rows, M not a multiple of the slab) and through graph replays; batch 1 (small-grid tiles) equals
the same item inside the batch.
"""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.config import encoded_length

pytestmark = pytest.mark.gpu
TAPS = ["ff%d" % i for i in range(8)] + ["oproj%d" % i for i in range(8)] + ["xfmr%d" % i for i in range(8)]


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("gemm_rows", 0)


def run(engine, mask, x, K=32):
    engine.set_option("gemm_rows", mask)
    engine.set_taps(True)
    try:
        codes = engine.encode_int32(x, K).cpu().numpy()
        return codes, {t: engine.get_tap(t).copy() for t in TAPS}
    finally:
        engine.set_taps(False)
        engine.set_option("gemm_rows", 0)


def same(a, b, what):
    for name in a[1]:
        assert np.array_equal(a[1][name], b[1][name]), (what, name, int((a[1][name] != b[1][name]).sum()))
    assert np.array_equal(a[0], b[0]), (what, int((a[0] != b[0]).sum()))


def test_rows_headline_batch_bitwise(engine):
    x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=401)).cuda()
    ref = run(engine, 0, x)
    for mask in (1, 2, 4, 7):
        same(ref, run(engine, mask, x), mask)


def test_rows_ragged_bitwise_and_single(engine):
    rng = np.random.default_rng(402)
    lengths = [int(v) for v in rng.integers(1, 24000 * 14, 24)]
    clips = [synthetic.speech_like(L, 403, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    engine.set_option("gemm_rows", 0)
    ref = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    engine.set_option("gemm_rows", 7)
    got = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    assert np.array_equal(ref, got), int((ref != got).sum())
    engine.set_option("gemm_rows", 0)
    for i in (0, 5, 11):
        one = engine.encode_int32(torch.from_numpy(clips[i][None]).cuda(), 32).cpu().numpy()
        F = encoded_length(lengths[i])
        assert np.array_equal(one[0], got[i, :, :F]), (i, lengths[i])


def test_rows_graph_replay(engine):
    x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=404)).cuda()
    engine.set_option("gemm_rows", 0)
    ref = engine.encode_int32(x, 8).cpu().numpy()
    engine.set_option("gemm_rows", 7)
    try:
        before = engine.graph_replays
        outs = [engine.encode_int32(x, 8).cpu().numpy() for _ in range(3)]
        assert engine.graph_replays > before
    finally:
        engine.set_option("gemm_rows", 0)
    for o in outs:
        assert np.array_equal(o, ref)
