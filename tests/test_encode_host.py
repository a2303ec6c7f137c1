"""mimi_encode_host (host samples in, host codes out in one engine call): the per-utterance path of
MimiEncoder.encode_audio_chunk (librispeech-mimi/process_librispeech_dev-test.py:136-141,
mls-en-mimi-pretrain/process_shard.py:302-307).  Its codes must be those of mimi_encode on a device copy, bit for bit,
including when the encode is re-run inside the wait (persistent RVQ chain give-up) -- the codes copied back are the
re-run's -- and from several threads at once."""
import threading

import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.config import encoded_length

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine(state_dict):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    m = MimiHipModel(state_dict, device="cuda:0")
    yield m
    m.set_option("rvq_chain_fault", 0)
    m.set_option("rvq_chain", 1)


@pytest.mark.parametrize("B,L", [(1, 1), (1, 1919), (1, 1921), (1, 240000), (1, 24000 * 13 + 5), (2, 48000)])
def test_encode_host_equals_device_encode(engine, B, L):
    x = np.stack([synthetic.speech_like(L, 501, i) for i in range(B)])
    for K in (8, 32):
        ref = engine.encode_int32(torch.from_numpy(x).cuda(), K).cpu().numpy()
        got = engine.encode_host(x, K)
        assert got.dtype == np.int32 and got.shape == (B, K, encoded_length(L))
        assert np.array_equal(got, ref), (B, L, K, int((got != ref).sum()))


def test_encoder_chunk_equals_padded_path(engine):
    from mimi_hip.encoder import MimiEncoder
    enc = MimiEncoder(device="cuda:0", model=engine)
    for i, L in enumerate([1, 30001, 240000, 400007]):
        a = synthetic.speech_like(L, 502, i)
        got = enc.encode_audio_chunk(a, 24000)
        ref = enc._encode_padded([a])[0].astype(np.int64)
        assert got.dtype == np.int64 and got.shape == (32, encoded_length(L))
        assert np.array_equal(got, ref), L
    with pytest.raises(ValueError):
        enc.encode_audio_chunk(np.zeros(0, np.float32), 24000)
    with pytest.raises(ValueError):
        engine.encode_host(np.zeros((1, 100), np.float32), 33)


def test_encode_host_copies_back_rerun_codes(engine):
    """rvq_chain_fault = 2: every chain sweep gives up, the wait re-runs the encode without the chain, and the host
    codes must be the re-run's (the per-level path's), not the abandoned first pass's."""
    x = synthetic.speech_like(200000, 503, 0)[None]
    engine.set_option("rvq_chain", 0)
    try:
        ref = engine.encode_host(x, 32)
        engine.set_option("rvq_chain", 1)
        engine.set_option("rvq_chain_fault", 2)
        r0 = engine.rvq_chain_reruns
        for _ in range(3):
            assert np.array_equal(engine.encode_host(x, 32), ref)
        assert engine.rvq_chain_reruns - r0 == 3
    finally:
        engine.set_option("rvq_chain_fault", 0)
        engine.set_option("rvq_chain", 1)
    assert np.array_equal(engine.encode_host(x, 32), ref)


def test_encode_host_threads(engine):
    clips = [synthetic.speech_like(int(n), 504, i)[None]
             for i, n in enumerate(np.random.default_rng(504).integers(24000, 300000, 12))]
    ref = [engine.encode_host(c, 32) for c in clips]
    out = [None] * len(clips)
    errs = []

    def work(t):
        try:
            for i in range(t, len(clips), 4):
                out[i] = engine.encode_host(clips[i], 32)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    ths = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    for i, (o, r) in enumerate(zip(out, ref)):
        assert np.array_equal(o, r), i
