"""Host-ingest resampler: the HIP kernel (mimi_hip.ingest.resample -> mimi_resample_poly) bit-exact with
scipy.signal.resample_poly (librosa's res_type='polyphase'), pinned by tests/golden/resample.npz; the oracle
restatement (oracle/resample_ref.py) checked against scipy and the fixtures; WAV loading semantics."""
import math
import os
import wave

import numpy as np
import pytest
import torch

from mimi_hip import ingest
from oracle.resample_ref import design_filter, librosa_polyphase_ref, resample_poly_ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RATES = [16000, 8000, 22050, 44100, 48000]
LENGTHS = [1, 2, 3, 37, 1001, 16001]


def _clip(rate, n):  # as tests/golden/make_resample_golden.py
    return np.random.default_rng(rate * 100003 + n).normal(0.0, 0.3, n).astype(np.float32)


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLDEN, "resample.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def bits_equal(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("rate", RATES)
def test_oracle_matches_golden(gold, rate):
    for n in LENGTHS:
        assert bits_equal(librosa_polyphase_ref(_clip(rate, n), rate, 24000), gold[f"r{rate}_n{n}"]), (rate, n)


def test_oracle_matches_scipy_live():
    from scipy.signal import resample_poly
    rng = np.random.default_rng(1)
    for up, down in [(3, 2), (1, 2), (160, 147), (3, 1), (2, 3)]:
        for n in [5, 999, 4097]:
            x = rng.normal(0, 1, n).astype(np.float32)
            assert bits_equal(resample_poly_ref(x, up, down), resample_poly(x, up, down)), (up, down, n)


def test_plan_matches_scipy_design():
    for r in RATES:
        up, down, hp, pre = ingest.resample_plan(r, 24000)
        g = math.gcd(r, 24000)
        assert (up, down) == (24000 // g, r // g)
        h, n_pre_pad, half_len = design_filter(up, down)
        assert bits_equal(hp, np.concatenate([np.zeros(n_pre_pad, np.float32), h]))
        assert pre == (half_len + n_pre_pad) // down
    with pytest.raises(ValueError):
        ingest.resample_plan(16000.5, 24000)


def test_resample_refuses_cpu_device():
    with pytest.raises(ValueError, match="HIP device only"):
        ingest.resample([np.zeros(10, np.float32)], 16000, 24000, device="cpu")


def _write_wav(path, data, sr, sampwidth):
    with wave.open(path, "wb") as w:
        w.setnchannels(1 if data.ndim == 1 else data.shape[1])
        w.setsampwidth(sampwidth)
        w.setframerate(sr)
        w.writeframes(data.tobytes())


def test_load_wav_formats(tmp_path):
    rng = np.random.default_rng(3)
    pcm16 = rng.integers(-32768, 32767, (500, 2), dtype=np.int16)
    p = str(tmp_path / "s16.wav")
    _write_wav(p, pcm16, 16000, 2)
    y, sr = ingest.load_wav(p)
    assert sr == 16000 and y.dtype == np.float32 and y.shape == (500,)
    f = pcm16.astype(np.float32) / 32768.0
    assert bits_equal(y, (f[:, 0] + f[:, 1]) / np.float32(2))       # librosa.to_mono: channel mean
    u8 = rng.integers(0, 255, 300, dtype=np.uint8)
    p = str(tmp_path / "u8.wav")
    _write_wav(p, u8, 8000, 1)
    y, sr = ingest.load_wav(p)
    assert sr == 8000 and bits_equal(y, (u8.astype(np.float32) - 128) / 128)
    from scipy.io import wavfile
    fl = rng.normal(0, 0.2, 700).astype(np.float32)
    p = str(tmp_path / "f32.wav")
    wavfile.write(p, 24000, fl)
    y, sr = ingest.load_wav(p)
    assert sr == 24000 and bits_equal(y, fl)


@pytest.mark.gpu
def test_resample_kernel_bit_exact(gold):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    for rate in RATES:
        clips = [_clip(rate, n) for n in LENGTHS]
        outs = ingest.resample(clips, rate, 24000, device="cuda:0")   # ragged batch: one launch
        for n, o in zip(LENGTHS, outs):
            assert o.is_cuda and o.dtype == torch.float32
            assert bits_equal(o.cpu().numpy(), gold[f"r{rate}_n{n}"]), (rate, n)


@pytest.mark.gpu
def test_resample_kernel_full_size_vs_scipy():
    """A 60 s LibriSpeech-rate clip (the YODAS2 maximum chunk) and an empty clip in one batch; scipy live."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from scipy.signal import resample_poly
    x = np.random.default_rng(11).normal(0, 0.1, 16000 * 60).astype(np.float32)
    outs = ingest.resample([x, np.zeros(0, np.float32), x[:7]], 16000, 24000, device="cuda:0")
    assert outs[1].numel() == 0
    assert bits_equal(outs[0].cpu().numpy(), resample_poly(x, 3, 2))
    assert bits_equal(outs[2].cpu().numpy(), resample_poly(x[:7], 3, 2))


@pytest.mark.gpu
def test_load_then_encode(tmp_path, state_dict):
    """WAV at 16 kHz -> GPU resample -> the same samples librosa's polyphase mode gives (restated) -> the
    drop-in MimiEncoder on the HIP engine -> the oracle's codes for those samples."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.encoder import MimiEncoder
    from mimi_hip.model import MimiHipModel
    from oracle import mimi_ref
    t = np.arange(16000) / 16000.0
    pcm = (8000 * np.sin(2 * np.pi * 180 * t) * (0.6 + 0.4 * np.sin(2 * np.pi * 3 * t))
           + np.random.default_rng(5).normal(0, 300, t.size)).astype(np.int16)
    p = str(tmp_path / "a.wav")
    _write_wav(p, pcm, 16000, 2)
    y, sr = ingest.load(p, sr=24000, device="cuda:0")
    want = librosa_polyphase_ref(pcm.astype(np.float32) / 32768.0, 16000, 24000)
    assert sr == 24000 and len(y) == 24000 and bits_equal(y, want)
    enc = MimiEncoder(device="cuda:0", model=MimiHipModel(state_dict, device="cuda:0"))
    codes = enc.encode_audio_chunk(y, 24000)
    ref = mimi_ref.encode(torch.from_numpy(want)[None, None], state_dict, 32)[0].numpy()
    assert codes.shape == ref.shape == (32, 13)
    assert (codes == ref).mean() > 0.99, (codes == ref).mean()


@pytest.mark.gpu
def test_resample_kernel_window_variants_vs_scipy():
    """Down-sampling ratios whose per-pass input window needs 1, 2, 4 prefetch registers per thread or the
    load-then-compute path (96 kHz -> 24 kHz: > 1024 samples), against scipy live."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from scipy.signal import resample_poly
    rng = np.random.default_rng(12)
    for orig in (8000, 48000, 72000, 96000, 22050):
        g = math.gcd(orig, 24000)
        xs = [rng.normal(0, 0.2, n).astype(np.float32) for n in (orig * 3 + 17, 5, orig // 3)]
        outs = ingest.resample(xs, orig, 24000, device="cuda:0")
        for x, o in zip(xs, outs):
            want = resample_poly(x, 24000 // g, orig // g)
            # librosa: n_samples = int(np.ceil(n * ratio)) with ratio = float(target) / orig, rounded first --
            # 7350 samples at 22.05 kHz give ceil(8000.000000000001) = 8001, one zero past resample_poly's 8000
            m = int(math.ceil(len(x) * (24000.0 / orig)))
            want = want[:m] if len(want) >= m else np.concatenate([want, np.zeros(m - len(want), np.float32)])
            assert bits_equal(o.cpu().numpy(), want), (orig, len(x))


# ---- soxr_hq-spec mode (librosa's default res_type; libsoxr's published HQ spec, parity with libsoxr unpinned) ----

SOXR_PAIRS = [16000, 8000, 48000, 32000, 44100, 22050]


def _upfirdn_ref(x, up, down, hp, pre, n_out):
    """scipy.signal.upfirdn over the padded filter, trimmed as resample_poly trims: the arithmetic the kernel runs."""
    from scipy.signal import upfirdn
    y = upfirdn(hp, np.asarray(x, np.float32), up, down)
    out = np.zeros(n_out, np.float32)
    seg = y[pre:pre + n_out]
    out[:len(seg)] = seg
    return out


@pytest.mark.parametrize("rate", SOXR_PAIRS)
def test_soxr_hq_filter_meets_spec(rate):
    """The filter of every source rate -> 24 kHz, as the kernel receives it (float32 taps, /up): linear phase
    (symmetric), passband ripple < 0.01 dB up to 0.913 of the lower Nyquist, >= 120.4 dB (20 bits) rejection from the
    lower Nyquist to the up-sampled Nyquist."""
    up, down, hp, pre = ingest.soxr_hq_plan(rate, 24000)
    h = hp[np.flatnonzero(hp)[0]:].astype(np.float64) / up  # (pre-padding zeros off)
    assert len(h) % 2 == 1 and np.array_equal(h, h[::-1])
    fs_up = rate * up
    nyq = min(rate, 24000) / 2
    nfft = 1 << 21  # (a bin of fs_up / 2^21: <= 1.7 Hz at the largest up-sampled rate)
    H = np.fft.rfft(h, nfft)
    w = np.arange(len(H)) * fs_up / nfft
    mag = 20 * np.log10(np.abs(H) + 1e-300)
    spec = ingest.SOXR_HQ_SPEC
    passband = mag[w <= spec["passband_end"] * nyq]
    stopband = mag[w >= spec["stopband_begin"] * nyq]
    assert np.abs(passband).max() < 0.01, np.abs(passband).max()
    assert stopband.max() <= -spec["precision_bits"] * 20 * math.log10(2), stopband.max()


def test_soxr_hq_tones():
    """Tones through the soxr_hq-spec resampler (the kernel's arithmetic, restated by scipy.signal.upfirdn):
    a passband tone keeps its amplitude within 0.01 dB and its phase (zero delay: the output is the tone sampled at
    the new rate to -100 dB), a tone in the stopband of a down-conversion leaves <= -120 dB (20 bits)."""
    def tone(f, rate, n):
        return np.sin(2 * np.pi * f * np.arange(n) / rate).astype(np.float32)

    def resample(x, rate):
        up, down, hp, pre = ingest.soxr_hq_plan(rate, 24000)
        return _upfirdn_ref(x, up, down, hp, pre, int(math.ceil(len(x) * 24000 / rate)))

    for rate, f in ((16000, 1000.0), (16000, 7290.0), (48000, 10950.0), (44100, 3000.0)):
        n = rate * 2
        y = resample(tone(f, rate, n), rate)
        ideal = np.sin(2 * np.pi * f * np.arange(len(y)) / 24000)
        mid = slice(len(y) // 4, 3 * len(y) // 4)  # away from the clip edges (implicit zeros outside)
        gain = np.sqrt(np.mean(y[mid].astype(np.float64) ** 2) / np.mean(ideal[mid] ** 2))
        assert abs(20 * np.log10(gain)) < 0.01, (rate, f, gain)
        err = np.sqrt(np.mean((y[mid] - ideal[mid]) ** 2) / np.mean(ideal[mid] ** 2))
        assert err < 1e-5, (rate, f, err)  # (float32 arithmetic: ~-120 dB; the filter's own error is below)
    for rate, f in ((48000, 12500.0), (48000, 20000.0), (44100, 13000.0)):
        n = rate
        y = resample(tone(f, rate, n), rate)
        mid = slice(len(y) // 4, 3 * len(y) // 4)
        leak = np.sqrt(np.mean(y[mid].astype(np.float64) ** 2) / 0.5)
        assert 20 * np.log10(leak + 1e-30) <= -120.0, (rate, f, leak)


def test_soxr_hq_mode_switch_and_errors():
    assert ingest.RES_TYPES == ("polyphase", "soxr_hq")
    with pytest.raises(ValueError, match="res_type"):
        ingest.resample([np.zeros(10, np.float32)], 16000, 24000, device="cuda:0", res_type="kaiser_best")
    up, down, hp, pre = ingest.soxr_hq_plan(16000, 24000)
    assert (up, down) == (3, 2) and hp.dtype == np.float32 and pre > 0
    p_up, p_down, p_hp, _ = ingest.resample_plan(16000, 24000)
    assert (p_up, p_down) == (up, down) and len(hp) > len(p_hp)  # (the HQ spec's narrow transition band)


@pytest.mark.gpu
def test_soxr_hq_kernel_bit_exact_vs_upfirdn():
    """GPU: the soxr_hq-spec mode through the kernel equals scipy.signal.upfirdn over the same filter bit for bit,
    ragged clips in one launch, for an LDS-resident filter (16 / 48 kHz) and the long filters read from global
    memory (44.1 / 22.05 kHz: ~28-30k taps)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    for rate in (16000, 48000, 44100, 22050):
        clips = [_clip(rate, n) for n in (1, 37, 1001, 3 * rate + 17)]
        outs = ingest.resample(clips, rate, 24000, device="cuda:0", res_type="soxr_hq")
        up, down, hp, pre = ingest.soxr_hq_plan(rate, 24000)
        for c, o in zip(clips, outs):
            want = _upfirdn_ref(c, up, down, hp, pre, int(math.ceil(len(c) * 24000 / rate)))
            assert bits_equal(o.cpu().numpy(), want), (rate, len(c))
