"""The k = 1 residual conv + skip + ELU of stages 2 and 3 as the streaming kernel (res1_stream.hip, engine option
"res1_stream": 1 stage 2 (default), 2 stages 2 and 3, 0 the planes GEMM) against the planes GEMM it replaces (ROLE_RES1P): the
same fragments, K order, product order and epilogue expressions, so the stage-2 and stage-3 block outputs (taps
"res2_elu" / "res3_elu": the y planes the down convs read) and all 32 codebooks must be equal BITWISE -- uniform
batches whose row count is not a multiple of the 16-step tile, a 1-sample item, ragged batches (per-item valid steps;
stage 3 keeps the GEMM there) and graph replays (TF/modeling_mimi.py:433-447 MimiResnetBlock, the 1 kHz and 200 Hz
stages)."""
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
    m.set_option("res1_stream", 1)


def run(engine, on, x, taps=True, K=32):
    engine.set_option("res1_stream", on)
    engine.set_taps(taps)
    try:
        c = engine.encode_int32(x, K).cpu().numpy()
        return c, ((engine.get_tap("res2_elu").copy(), engine.get_tap("res3_elu").copy()) if taps else None)
    finally:
        engine.set_taps(False)
        engine.set_option("res1_stream", 1)


FORMS = [1, 2]  # res1_stream on for stage 2 (default), for stages 2 and 3


@pytest.mark.parametrize("B,L", [(8, 240000), (3, 24000 * 7 + 11), (2, 1), (5, 1920 * 33 + 7)])
def test_res1_stream_uniform_bitwise(engine, B, L):
    x = torch.from_numpy(np.stack([synthetic.speech_like(L, 411, i) for i in range(B)])).cuda()
    c0, y0 = run(engine, 0, x)
    for f in FORMS:
        c1, y1 = run(engine, f, x)
        for st, a, b in zip((2, 3), y0, y1):
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (f, st, int((a != b).sum()))
        assert np.array_equal(c0, c1), (f, B, L)


def test_res1_stream_ragged_bitwise(engine):
    rng = np.random.default_rng(412)
    lengths = [int(v) for v in rng.integers(1, 300000, 17)]
    lengths[0], lengths[1] = 1, 300000
    clips = [synthetic.speech_like(L, 413, i) for i, L in enumerate(lengths)]
    x = np.zeros((len(clips), max(lengths)), np.float32)
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    xt = torch.from_numpy(x).cuda()
    got = []
    for on in [0] + FORMS:
        engine.set_option("res1_stream", on)
        try:
            got.append(engine.encode_ragged(xt, lengths, 32).cpu().numpy())
        finally:
            engine.set_option("res1_stream", 1)
    for g in got[1:]:
        assert np.array_equal(got[0], g), int((got[0] != g).sum())


def test_res1_stream_graph_replay(engine):
    x = torch.from_numpy(synthetic.clip_batch(8, 240000, seed=414)).cuda()
    ref, _ = run(engine, 0, x, taps=False)
    engine.set_option("res1_stream", 1)
    before = engine.graph_replays
    outs = [engine.encode_int32(x, 32).cpu().numpy() for _ in range(3)]
    assert engine.graph_replays > before
    for o in outs:
        assert np.array_equal(o, ref)
