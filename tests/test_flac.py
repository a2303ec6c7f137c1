"""FLAC ingest (mimi_flac_decode, csrc/flac.cpp; mimi_hip.ingest.load_flac): CPU tests, no GPU.

Parity: libFLAC / libsndfile are absent, so the decoder is pinned to the format, not to libFLAC -- FLAC is
lossless, and every stream the spec-written test encoder (tests/flac_writer.py) produces must decode to exactly
the PCM it encoded.  The float conversion is libsndfile's (PCM / 2^(bits-1)), the channel mix librosa's
``to_mono``, the same code path as WAV (ingest.load_wav).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import flac_writer as fw  # noqa: E402

from mimi_hip import _lib, ingest  # noqa: E402


def _signal(rng, C, n, bps, kind):
    hi = 2 ** (bps - 1)
    if kind == "noise":
        return rng.integers(-hi, hi, size=(C, n))
    t = np.arange(n)
    x = np.stack([0.6 * np.sin(2 * np.pi * (180 + 70 * c) * t / 16000) + 0.02 * rng.standard_normal(n)
                  for c in range(C)])
    return np.clip(np.round(x * (hi - 1)), -hi, hi - 1).astype(np.int64)


CASES = [
    # (channels, bps, n, block sizes, variable, id3, total_known, kind, wasted)
    (1, 16, 16000, [4096], False, False, True, "tone", 0),         # LibriSpeech-like mono 16-bit
    (1, 16, 4097, [4096], False, False, True, "noise", 0),         # 1-sample last frame
    (2, 16, 9000, [1152, 576], False, False, True, "tone", 0),     # stereo decorrelations
    (2, 24, 5000, [1024], True, False, True, "tone", 0),           # variable-blocksize stream, 24-bit
    (2, 8, 3000, [192, 17, 300], False, True, True, "noise", 0),   # ID3 tag, 8-/16-bit header block sizes
    (3, 12, 2500, [256], False, False, False, "tone", 2),          # 3 channels, wasted bits, unknown length
    (6, 20, 2049, [512, 1000], False, False, True, "tone", 0),     # 6 channels, 20-bit
    (1, 24, 7000, [4608], False, False, True, "noise", 4),         # wasted bits on noise
    (2, 16, 1, [4096], False, False, True, "tone", 0),             # one sample
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_flac_round_trip(case):
    C, bps, n, bsz, variable, id3, known, kind, wasted = CASES[case]
    rng = np.random.default_rng(100 + case)
    pcm = _signal(rng, C, n, bps, kind)
    if wasted:
        pcm = (pcm >> wasted) << wasted
    data = fw.encode(pcm, 16000, bps, block_sizes=bsz, seed=case, variable=variable, id3=id3, total_known=known)
    out, sr, b = ingest.decode_flac(data)
    assert (sr, b) == (16000, bps)
    assert out.shape == pcm.shape
    np.testing.assert_array_equal(out, pcm)


def test_flac_random_streams():
    """60 random streams: every subframe kind, LPC orders 1-32, Rice / Rice2 / escapes, every channel mode."""
    rng = np.random.default_rng(7)
    for trial in range(60):
        C = int(rng.choice([1, 2, 2, 2, 4]))
        bps = int(rng.choice([8, 12, 16, 16, 20, 24]))
        n = int(rng.integers(1, 6000))
        pcm = _signal(rng, C, n, bps, "tone" if trial % 3 else "noise")
        bsz = [int(rng.choice([192, 576, 1152, 256, 4096, 1000, 17, 300, 33]))]
        rate = int(rng.choice([8000, 16000, 22050, 24000, 44100, 48000, 12345, 96000, 50000]))
        data = fw.encode(pcm, rate, bps, block_sizes=bsz, seed=trial, variable=bool(trial % 4 == 0))
        out, sr, b = ingest.decode_flac(data)
        assert sr == rate and b == bps
        np.testing.assert_array_equal(out, pcm, err_msg=f"trial {trial}")


def test_flac_corruption_is_an_error():
    rng = np.random.default_rng(3)
    pcm = _signal(rng, 1, 5000, 16, "tone")
    data = bytearray(fw.encode(pcm, 16000, 16, block_sizes=[1024], seed=1))
    first = bytes(data).index(b"\xff\xf8")  # first frame (fixed-blocksize sync)
    for pos, what in ((first + 2, "header CRC-8"), (first + 40, "CRC-16 / malformed"), (len(data) - 1, "CRC-16")):
        bad = bytearray(data)
        bad[pos] ^= 0x10
        with pytest.raises(_lib.MimiHipError) as ei:
            ingest.decode_flac(bytes(bad))
        assert ei.value.status == 6, what
    with pytest.raises(_lib.MimiHipError):
        ingest.decode_flac(bytes(data[:len(data) // 2]))  # truncated
    with pytest.raises(_lib.MimiHipError):
        ingest.decode_flac(b"RIFF....WAVEfmt ")
    with pytest.raises(ValueError):
        ingest.decode_flac(b"")


def test_load_flac_matches_libsndfile_float_and_librosa_mono(tmp_path):
    rng = np.random.default_rng(11)
    for C, bps in ((1, 16), (2, 16), (2, 24), (3, 8)):
        pcm = _signal(rng, C, 3001, bps, "tone")
        p = tmp_path / f"x{C}_{bps}.flac"
        p.write_bytes(fw.encode(pcm, 16000, bps, block_sizes=[1024], seed=C))
        y, sr = ingest.load_flac(str(p))
        f = (pcm / float(2 ** (bps - 1))).astype(np.float32)   # libsndfile: PCM / 2^(bits-1)
        want = np.mean(f, axis=0, dtype=np.float32) if C > 1 else f[0]  # librosa.to_mono
        assert sr == 16000 and y.dtype == np.float32
        np.testing.assert_array_equal(y, want)
        assert ingest._is_flac(str(p))
