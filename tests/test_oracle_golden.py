"""CPU: the oracle and the synthetic inputs are pinned to the golden fixtures made from transformers
``MimiModel`` and the reference's own wrapper / utils (tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from audit import margin_audit
from mimi_hip import synthetic
from mimi_hip.config import MimiConfig, encoded_length
from oracle import mimi_ref


def test_synthetic_weights_reproduce_golden_checkpoint(golden, state_dict):
    _, meta = golden
    assert synthetic.state_dict_sha256(state_dict) == meta["weights_sha256"]


def test_synthetic_audio_reproducible(golden):
    _, meta = golden
    for i, L in enumerate(meta["lengths"][:6]):
        x = synthetic.speech_like(L, meta["audio_seed"], i)
        assert synthetic.audio_sha256([x]) == meta["audio_sha256"][str(L)]
    x = synthetic.speech_like(12000, meta["audio_seed"], 100)
    assert synthetic.audio_sha256([x]) == meta["audio_sha256"]["stage12000"]


@pytest.mark.parametrize("idx", [0, 1, 2, 3, 4, 5])
def test_oracle_codes_match_golden(golden, state_dict, idx):
    arrays, meta = golden
    L = meta["lengths"][idx]
    x = synthetic.speech_like(L, meta["audio_seed"], idx)
    taps = {}
    codes = mimi_ref.encode(torch.from_numpy(x)[None, None], state_dict, taps=taps)[0].numpy()
    ref = arrays[f"codes_L{L}"].astype(np.int64)
    assert codes.shape == ref.shape == (32, encoded_length(L))
    if np.array_equal(codes, ref):  # bit-exact on the CPU that made the fixtures
        return
    # another host's BLAS: every flip must be a near-tie of the oracle's own distances
    _, margins = mimi_ref.rvq_from_embedding(taps["pre_quantizer"], state_dict, 32, return_margins=True)
    frac, bad = margin_audit(ref, codes, margins[0].numpy())
    assert not bad, (frac, bad[:5])


def test_oracle_quantizer_on_golden_embedding(golden, state_dict):
    arrays, _ = golden
    for tag in ("speech10s", "noise5s"):
        emb = torch.from_numpy(arrays[f"emb_{tag}"])[None]
        codes = mimi_ref.rvq_from_embedding(emb, state_dict, 32)[0].numpy()
        ref = arrays[f"embcodes_{tag}"].astype(np.int64)
        if not np.array_equal(codes, ref):  # bit-exact here; elsewhere only near-ties may flip
            frac, bad = margin_audit(codes, ref, arrays[f"margins_{tag}"])
            assert not bad, (tag, frac, bad[:5])


def test_batch_golden_inputs_reproducible():
    """The padded-batch fixture's clips (tests/golden/make_golden_batch.py) regenerate bit-identically."""
    import json
    import os
    here = os.path.join(os.path.dirname(__file__), "golden")
    with open(os.path.join(here, "golden_batch_meta.json")) as f:
        meta = json.load(f)
    lengths = synthetic.random_lengths(meta["B"], 1.5, 20.0, seed=meta["len_seed"])
    assert lengths == meta["lengths"]
    audio = [synthetic.speech_like(L, meta["audio_seed"], meta["audio_index0"] + i) *
             np.float32(meta["quiet_gain"].get(str(i), 1.0)) for i, L in enumerate(lengths)]
    assert synthetic.audio_sha256(audio) == meta["audio_sha256"]
    with np.load(os.path.join(here, "golden_batch.npz"), allow_pickle=False) as z:
        for i, L in enumerate(lengths):
            assert z[f"item{i}"].shape == z[f"margin{i}"].shape == (32, encoded_length(L))


def test_oracle_stage_tensors(golden, state_dict):
    arrays, meta = golden
    x = synthetic.speech_like(12000, meta["audio_seed"], 100)
    taps = {}
    mimi_ref.encode(torch.from_numpy(x)[None, None], state_dict, taps=taps)
    for key, ref in arrays.items():
        if not key.startswith("stage_"):
            continue
        name, sub = key[len("stage_"):].rsplit("_sub", 1)
        t = taps[name][0]
        t = t[..., ::int(sub)] if name.startswith(("conv", "res", "down")) else t
        err = float((t - torch.from_numpy(ref)).abs().max() / (torch.from_numpy(ref).abs().max() + 1e-30))
        assert err < 1e-5, (name, err)


def test_prefix_property(golden, state_dict):
    """encode(K=8) == encode(K=32)[:, :8] -- why the bench's K = 8 is the reference's [:8] slice."""
    x = synthetic.speech_like(24000, 7, 4)
    xt = torch.from_numpy(x)[None, None]
    c32 = mimi_ref.encode(xt, state_dict, 32)
    c8 = mimi_ref.encode(xt, state_dict, 8)
    assert torch.equal(c32[:, :8], c8)


def test_encoded_length_matches_reference_float_math():
    # values verified against TF MimiModel.get_encoded_length in the survey
    assert [encoded_length(L) for L in (240000, 240001, 1, 1920, 1921)] == [125, 126, 1, 1, 2]
    rc = mimi_ref.RefConfig()
    for L in [1, 2, 7, 1919, 1920, 1921, 3839, 3840, 3841, 12345, 240000, 1440001, 16_777_217, 33_554_435]:
        t = L
        ref_t = L
        # reference: chain of MimiConv1d lengths via the oracle's tensor math
        for k, s in [(7, 1)] + sum([[(3, 1), (1, 1), (2 * r, r)] for r in (4, 5, 6, 8)], []) + [(3, 1), (4, 2)]:
            ref_t = ref_t + mimi_ref.extra_padding(ref_t, k, s) + (k - s)
            ref_t = (ref_t - k) // s + 1
        assert encoded_length(t) == ref_t, L
    _ = rc


def test_feature_extractor_matches_encodec(golden):
    transformers = pytest.importorskip("transformers")
    from mimi_hip.feature_extraction import MimiFeatureExtractor
    ref = transformers.EncodecFeatureExtractor(feature_size=1, sampling_rate=24000, padding_value=0.0)
    ours = MimiFeatureExtractor()
    a = [np.random.RandomState(0).randn(n).astype(np.float32) for n in (5, 17, 3)]
    r = ref(raw_audio=a, sampling_rate=24000, return_tensors="pt", padding=True)
    o = ours(raw_audio=a, sampling_rate=24000, return_tensors="pt", padding=True)
    assert torch.equal(r["input_values"], o["input_values"])
    assert torch.equal(r["padding_mask"].long(), o["padding_mask"].long())
    r1 = ref(raw_audio=a[1].astype(np.float64), sampling_rate=24000, return_tensors="pt")
    o1 = ours(raw_audio=a[1].astype(np.float64), sampling_rate=24000, return_tensors="pt")
    assert torch.equal(r1["input_values"], o1["input_values"]) and r1["input_values"].dtype == torch.float32
    with pytest.raises(ValueError):
        ours(raw_audio=a[0], sampling_rate=16000)


def test_feature_extractor_golden_meta(golden):
    from mimi_hip.feature_extraction import MimiFeatureExtractor
    _, meta = golden
    a = [np.zeros(n, np.float32) for n in meta["batch_lengths"][:2]]
    o = MimiFeatureExtractor()(raw_audio=a, sampling_rate=24000, return_tensors="pt", padding=True)
    for k, (dtype, shape) in meta["feature_extractor"].items():
        assert list(o[k].shape) == shape


def test_config_defaults():
    c = MimiConfig()
    assert c.frame_size == 1920 and c.frame_rate == 12.5 and c.encodec_frame_rate == 25


def test_conv_out_len_integer_form_equals_float32_form():
    """config.conv_out_len answers ceil(L / s) directly below 2^22 samples; that must be the reference's float32
    expression ((L - s) / s + 1, ceil) for every stride the encoder uses, including the ranges' edges."""
    from mimi_hip.config import conv_out_len

    def f32_form(length, kernel, stride):
        pt = kernel - stride
        nf = np.float32(np.float32(length - kernel + pt) / np.float32(stride)) + np.float32(1.0)
        return int(np.ceil(np.float32(nf)))

    rng = np.random.default_rng(7)
    for k, s in [(7, 1), (3, 1), (1, 1), (8, 4), (10, 5), (12, 6), (16, 8), (4, 2)]:
        ls = list(range(0, 5000)) + [int(v) for v in rng.integers(5000, 1 << 22, 4000)] + \
            list(range((1 << 22) - 2000, (1 << 22) + 50))
        for L in ls:
            assert conv_out_len(L, k, s) == f32_form(L, k, s), (k, s, L)
