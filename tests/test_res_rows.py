"""Stage-2 residual block in one kernel (resblock_rows.hip): bit-identical to the down conv ELU(x) planes + k3 planes
GEMM + k1 planes GEMM it replaces on large grids.

MimiResnetBlock.forward (TF/modeling_mimi.py:299-312) of the third encoder stage (256 channels, 128 hidden) runs, for
batches with >= 256 tiles of 128 frames, as one kernel that builds the k3 conv's fp16 operand planes from the fp32
down-conv output in registers, keeps the hidden activations in LDS and writes only the block output planes.  The
block output ("res2_elu"), the next down conv's output ("down2"), the transformer output and all 32 codebooks must be
equal BITWISE across the "res_rows" option, on the B = 32 x 10 s headline batch, ragged batches (per-item frame
counts, items ending inside a tile) and graph replays, and batch 1 (never fused: 94 tiles) equals the item in the
batch.  The option is off by default: slower than the two planes GEMMs (profiles/r4q_ab_res_rows.txt).
"""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.config import encoded_length

pytestmark = pytest.mark.gpu
TAPS = ["res2_elu", "down2", "xfmr7"]


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("res_rows", 0)


def run(engine, v, x, K=32):
    engine.set_option("res_rows", v)
    engine.set_taps(True)
    try:
        codes = engine.encode_int32(x, K).cpu().numpy()
        return codes, {t: engine.get_tap(t).copy() for t in TAPS}
    finally:
        engine.set_taps(False)
        engine.set_option("res_rows", 0)


def test_res_rows_headline_batch_bitwise(engine):
    x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=501)).cuda()
    c0, t0 = run(engine, 0, x)
    c1, t1 = run(engine, 1, x)
    for name in TAPS:
        assert np.array_equal(t0[name], t1[name]), (name, int((t0[name] != t1[name]).sum()))
    assert np.array_equal(c0, c1), int((c0 != c1).sum())
    one = engine.encode_int32(x[7:8], 32).cpu().numpy()  # (batch 1: the two planes GEMMs)
    assert np.array_equal(one[0], c1[7])


def test_res_rows_ragged_bitwise(engine):
    rng = np.random.default_rng(502)
    lengths = [int(v) for v in rng.integers(1, 24000 * 16, 24)]
    lengths[0], lengths[1] = 24000 * 16, 7
    clips = [synthetic.speech_like(L, 503, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    engine.set_option("res_rows", 0)
    ref = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    engine.set_option("res_rows", 1)
    got = engine.encode_ragged(xt, lengths, 32).cpu().numpy()
    engine.set_option("res_rows", 0)
    assert np.array_equal(ref, got), int((ref != got).sum())
    for i in (0, 1, 9):
        one = engine.encode_int32(torch.from_numpy(clips[i][None]).cuda(), 32).cpu().numpy()
        F = encoded_length(lengths[i])
        assert np.array_equal(one[0], got[i, :, :F]), (i, lengths[i])


def test_res_rows_graph_replay(engine):
    x = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=504)).cuda()
    engine.set_option("res_rows", 0)
    ref = engine.encode_int32(x, 8).cpu().numpy()
    engine.set_option("res_rows", 1)
    try:
        before = engine.graph_replays
        outs = [engine.encode_int32(x, 8).cpu().numpy() for _ in range(3)]
        assert engine.graph_replays > before
    finally:
        engine.set_option("res_rows", 0)
    for o in outs:
        assert np.array_equal(o, ref)
