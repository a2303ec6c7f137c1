"""Ragged batches (``mimi_encode_ragged``): each item encoded exactly as alone at its own length, in one pass.

The per-utterance callers (MLS ``mls-en-mimi-pretrain/process_shard.py:302-307``, LibriSpeech
``process_librispeech_dev-test.py:136-141``) encode one utterance at a time (batch-1 semantics: each conv's extra
padding at the utterance's own end, ``TF/modeling_mimi.py:269-279``; the downsample's replicate edge at its own
last frame, ``:1196-1206``; attention over its own frames).  A ragged batch must give every item those codes bit
for bit -- so every kernel must read only its item's rows (the rest as zero) and pick the kernel the item would get
alone (T <= 256 frames: the one-workgroup-per-head attention; longer: the banded one).

The pad-to-longest callers (Emilia / YODAS2 / LibriTTS-R) get their padded batch's kept frames from a ragged
encode at E_i = min(Lmax, 1920 ceil(L_i / 1920)) (mimi_hip/encoder.py); those are checked against the reference
wrapper's own outputs in tests/test_gpu_parity.py::test_padded_batch_b32_vs_reference_wrapper.
"""
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
    return MimiHipModel(state_dict, device="cuda:0")


def ragged_batch(lengths, seed):
    clips = [synthetic.speech_like(L, seed, i) for i, L in enumerate(lengths)]
    L = max(lengths)
    x = np.full((len(clips), L), np.nan, np.float32)  # past its length an item's row is never read: NaN proves it
    for i, c in enumerate(clips):
        x[i, :len(c)] = c
    return clips, x


def alone(engine, clip, K):
    return engine.encode_int32(torch.from_numpy(clip)[None].cuda(), K)[0].cpu().numpy()


def check_equal_alone(engine, lengths, K, seed):
    clips, x = ragged_batch(lengths, seed)
    got = engine.encode_ragged(torch.from_numpy(x).cuda(), lengths, K).cpu().numpy()
    assert got.shape == (len(lengths), K, encoded_length(max(lengths)))
    for i, c in enumerate(clips):
        T = encoded_length(lengths[i])
        ref = alone(engine, c, K)
        assert ref.shape == (K, T)
        assert np.array_equal(got[i, :, :T], ref), (i, lengths[i], int((got[i, :, :T] != ref).sum()))
    return got


def test_ragged_mls_batch_equals_per_utterance(engine):
    """32 utterances U[10, 20] s (T > 256 frames for most: the banded attention; some at <= 10.24 s: the T <= 256
    kernel) in one ragged encode == each encoded alone, bitwise, at K = 8; run twice (determinism)."""
    lengths = synthetic.random_lengths(32, 10.0, 20.0, seed=41)
    a = check_equal_alone(engine, lengths, 8, 41)
    b = engine.encode_ragged(torch.from_numpy(ragged_batch(lengths, 41)[1]).cuda(), lengths, 8).cpu().numpy()
    for i, L in enumerate(lengths):
        T = encoded_length(L)
        assert np.array_equal(a[i, :, :T], b[i, :, :T])


def test_ragged_edge_lengths_k32(engine):
    """Edge lengths in one batch -- 1 sample (T = 1: both replicate edges on one row), 960 / 961 (25 Hz frame
    boundaries), 1919 / 1920 / 1921 (12.5 Hz boundaries), odd and even 25 Hz counts, a 10.24 s / 10.28 s pair around
    the attention kernel switch, 60 s -- at K = 32, each == alone."""
    lengths = [1, 960, 961, 1919, 1920, 1921, 24000 * 3 + 7, 245760, 246720, 240000, 1440000, 5000]
    check_equal_alone(engine, lengths, 32, 43)


def test_ragged_overflow_fallback_per_item(engine):
    """An item 3e4 x louder than the calibration overflows the fixed fp16 scales: the ragged encode's fallback
    re-encodes each item alone at its own length -- its codes equal the alone encodes (which take the same
    fallback), and the quiet items are unaffected."""
    lengths = [48000, 30000, 70001]
    clips, x = ragged_batch(lengths, 44)
    x[1, :lengths[1]] *= np.float32(3e4)
    clips[1] = clips[1] * np.float32(3e4)
    before = engine.f16_reruns
    got = engine.encode_ragged(torch.from_numpy(x).cuda(), lengths, 8).cpu().numpy()
    assert engine.f16_reruns > before
    for i, c in enumerate(clips):
        T = encoded_length(lengths[i])
        assert np.array_equal(got[i, :, :T], alone(engine, c, 8)), i


def test_ragged_other_precision_item_by_item(engine):
    """Outside f16x3 the ragged call runs item by item (same definition): == alone in f32 mode."""
    prev = engine.precision
    engine.set_precision("f32")
    try:
        check_equal_alone(engine, [24000, 7000, 33333], 8, 45)
    finally:
        engine.set_precision(prev)


def test_encoder_chunks_and_batches(engine):
    """MimiEncoder: encode_audio_chunks (ragged, grouped by length, pipelined) == encode_audio_chunk per item;
    encode_batches (pipelined) == encode_audio_batch per batch; ragged pad-to-longest keeps the literal padded
    encode's codes up to near-ties (the reference comparison is in test_gpu_parity)."""
    from mimi_hip.encoder import MimiEncoder
    enc = MimiEncoder(device="cuda:0", model=engine, num_quantizers=8, chunk_batch=5)
    lens = synthetic.random_lengths(13, 0.05, 21.0, seed=46) + [1, 1921]
    clips = [synthetic.speech_like(L, 46, i) for i, L in enumerate(lens)]
    got = enc.encode_audio_chunks(clips, 24000)
    for i, c in enumerate(clips):
        assert np.array_equal(got[i], enc.encode_audio_chunk(c, 24000)), i
    batches = [clips[0:4], clips[4:5], clips[5:11], [], clips[11:15]]
    streamed = list(enc.encode_batches(iter(batches), 24000))
    assert len(streamed) == len(batches)
    for b, s in zip(batches, streamed):
        want = enc.encode_audio_batch(b, 24000)
        assert len(s) == len(want) and all(np.array_equal(x, y) for x, y in zip(s, want))
    literal = MimiEncoder(device="cuda:0", model=engine, num_quantizers=8, ragged=False)
    a = np.concatenate([x.ravel() for x in enc.encode_audio_batch(clips[5:11], 24000)])
    b = np.concatenate([x.ravel() for x in literal.encode_audio_batch(clips[5:11], 24000)])
    assert a.shape == b.shape and (a == b).mean() > 0.99


def test_encoder_empty_item_in_batch(engine):
    """An empty item among non-empty ones: the reference pads it and trims it to 0 frames
    (emilia-mimi/process_shard.py:113-139), so it comes back as (K, 0); the other items are unchanged."""
    from mimi_hip.encoder import MimiEncoder
    enc = MimiEncoder(device="cuda:0", model=engine, num_quantizers=8)
    clips = [synthetic.speech_like(L, 47, i) for i, L in enumerate((30000, 5000))]
    empty = np.zeros(0, np.float32)
    got = enc.encode_audio_batch([clips[0], empty, clips[1]], 24000)
    want = enc.encode_audio_batch(clips, 24000)
    assert got[1].shape == (8, 0) and got[1].dtype == np.int64
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[2], want[1])
    literal = MimiEncoder(device="cuda:0", model=engine, num_quantizers=8, ragged=False)
    assert literal.encode_audio_batch([clips[0], empty], 24000)[1].shape == (8, 0)
    with pytest.raises(ValueError):
        enc.encode_audio_batch([empty, empty], 24000)


def test_encoder_threads_share_one_encoder(engine):
    """Several threads calling encode_audio_batch / encode_audio_chunks on ONE MimiEncoder (the YODAS2
    ThreadPoolExecutor, yodas2-mimi/process_shard.py:691-717) get exactly the serial results: every thread stages
    through its own pipeline buffers."""
    from concurrent.futures import ThreadPoolExecutor
    from mimi_hip.encoder import MimiEncoder
    enc = MimiEncoder(device="cuda:0", model=engine, num_quantizers=8)
    jobs = []
    for j in range(12):
        lens = synthetic.random_lengths(3 + j % 4, 0.5, 12.0, seed=300 + j)
        jobs.append([synthetic.speech_like(L, 300 + j, i) for i, L in enumerate(lens)])
    serial = [enc.encode_audio_batch(b, 24000) if j % 3 else enc.encode_audio_chunks(b, 24000)
              for j, b in enumerate(jobs)]

    def run(j):
        b = jobs[j]
        return enc.encode_audio_batch(b, 24000) if j % 3 else enc.encode_audio_chunks(b, 24000)

    for _ in range(2):
        with ThreadPoolExecutor(max_workers=4) as ex:
            par = list(ex.map(run, range(len(jobs))))
        for j, (s, p) in enumerate(zip(serial, par)):
            assert len(s) == len(p) and all(np.array_equal(x, y) for x, y in zip(s, p)), j
