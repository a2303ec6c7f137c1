"""Stage-1 residual block forms (resblock.hip resblock128_h16_kernel, engine option "res1_form"): one 8-wave workgroup
per CU (0) or two 4-wave workgroups per CU (1, the default: each wave both 16-step tiles of its M tile).  Only the assignment of
tiles to waves differs, so the codes must be equal BITWISE -- uniform batches with partial 32-step blocks, a 1-sample
item, ragged batches (per-item lengths, packed block ranges) and graph replays (TF/modeling_mimi.py:408-447
MimiResnetBlock on the 6 kHz stage)."""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("res1_form", 1)


def codes(engine, form, x, K=32):
    engine.set_option("res1_form", form)
    try:
        return engine.encode_int32(x, K).cpu().numpy()
    finally:
        engine.set_option("res1_form", 1)


@pytest.mark.parametrize("B,L", [(32, 240000), (3, 24000 * 7 + 11), (2, 1), (5, 1920 * 33 + 7)])
def test_res1_form_uniform_bitwise(engine, B, L):
    x = torch.from_numpy(np.stack([synthetic.speech_like(L, 401, i) for i in range(B)])).cuda()
    assert np.array_equal(codes(engine, 0, x), codes(engine, 1, x)), (B, L)


def test_res1_form_ragged_bitwise(engine):
    rng = np.random.default_rng(402)
    lengths = [int(v) for v in rng.integers(1, 300000, 17)]
    lengths[0], lengths[1] = 1, 300000
    clips = [synthetic.speech_like(L, 403, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    got = []
    for form in (0, 1):
        engine.set_option("res1_form", form)
        try:
            got.append(engine.encode_ragged(xt, lengths, 32).cpu().numpy())
        finally:
            engine.set_option("res1_form", 1)
    assert np.array_equal(got[0], got[1]), int((got[0] != got[1]).sum())


def test_res1_form_graph_replay(engine):
    x = torch.from_numpy(synthetic.clip_batch(8, 240000, seed=404)).cuda()
    ref = codes(engine, 0, x)
    engine.set_option("res1_form", 1)
    try:
        before = engine.graph_replays
        outs = [engine.encode_int32(x, 32).cpu().numpy() for _ in range(3)]
        assert engine.graph_replays > before
    finally:
        engine.set_option("res1_form", 1)
    for o in outs:
        assert np.array_equal(o, ref)
