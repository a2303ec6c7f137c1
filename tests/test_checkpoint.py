"""The real-checkpoint boundary: ``MimiEncoder("kyutai/mimi")`` -> ``resolve_checkpoint`` -> ``MimiConfig.from_json``
-> ``mimi_load_safetensors`` -> ``mimi_finalize``, the constructor path of every shard script
(emilia-mimi/process_shard.py:53-60: ``MimiModel.from_pretrained(model_id)`` + ``AutoFeatureExtractor``).

The kyutai/mimi weights are not available offline, so the checkpoint is the seeded synthetic state dict written in
the HF layout (tests/checkpoint_util.py: model.safetensors with the decoder half beside the encode path, and the
``config.json`` transformers 5.15.0 writes for ``MimiConfig()``, tests/golden/make_hf_config.py) and placed where
huggingface_hub's offline cache keeps a snapshot.  The engine built through that path must give the same codes,
bit for bit, as the engine built from the in-memory state dict; malformed checkpoints must fail with the C ABI's
status codes (MIMI_ERR_WEIGHTS = 4, MIMI_ERR_IO = 6), raised as ``MimiHipError``.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from checkpoint_util import GOLDEN, hub_snapshot_dir, write_hf_checkpoint
from mimi_hip import synthetic
from mimi_hip.config import MimiConfig

ENCODE_FIELDS = ("sampling_rate", "audio_channels", "hidden_size", "num_filters", "num_residual_layers",
                 "upsampling_ratios", "kernel_size", "last_kernel_size", "residual_kernel_size", "compress",
                 "codebook_size", "codebook_dim", "num_quantizers", "vector_quantization_hidden_dimension",
                 "num_semantic_quantizers", "num_hidden_layers", "intermediate_size", "num_attention_heads",
                 "num_key_value_heads", "head_dim", "norm_eps", "rope_theta", "sliding_window", "use_causal_conv",
                 "pad_mode", "hidden_act", "attention_bias", "use_conv_shortcut")


def test_config_json_fixture_reads_as_defaults():
    """config.json of transformers' MimiConfig() (rope_theta under rope_parameters, _frame_rate null) gives the
    encode-path fields of the defaults the engine is built for."""
    cfg = MimiConfig.from_json(os.path.join(GOLDEN, "mimi_config.json"))
    ref = MimiConfig()
    for f in ENCODE_FIELDS:
        assert getattr(cfg, f) == getattr(ref, f), f
    assert cfg.frame_rate == 12.5 and cfg.frame_size == 1920
    cfg.validate_supported()


def test_resolve_checkpoint_follows_hub_cache(tmp_path, monkeypatch):
    from mimi_hip.model import resolve_checkpoint
    monkeypatch.delenv("MIMI_HIP_CHECKPOINT", raising=False)
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path))
    with pytest.raises(FileNotFoundError):
        resolve_checkpoint("kyutai/mimi")
    old = hub_snapshot_dir(str(tmp_path), revision="a" * 40)
    snap = hub_snapshot_dir(str(tmp_path), revision="b" * 40)   # refs/main -> b...
    assert resolve_checkpoint("kyutai/mimi") == snap
    with open(os.path.join(tmp_path, "models--kyutai--mimi", "refs", "main"), "w") as f:
        f.write("a" * 40)
    assert resolve_checkpoint("kyutai/mimi") == old
    monkeypatch.setenv("MIMI_HIP_CHECKPOINT", str(snap))
    assert resolve_checkpoint("kyutai/mimi") == str(snap)
    assert resolve_checkpoint(str(old)) == str(old)


def test_hf_checkpoint_writer_roundtrip(tmp_path):
    """The helper writes exactly the state dict (plus decode-only tensors) in safetensors' format."""
    from safetensors.numpy import load_file
    sd = synthetic.make_state_dict(seed=0, num_quantizers=2)
    path = write_hf_checkpoint(sd, str(tmp_path))
    got = load_file(path)
    for k, v in sd.items():
        assert got[k].dtype == np.float32 and np.array_equal(got[k], v), k
    assert any(k.startswith("decoder.") for k in got) and any(k.startswith("upsample.") for k in got)
    assert os.path.exists(os.path.join(tmp_path, "config.json"))


def _status(fn, *args):
    from mimi_hip import _lib
    st = fn(*args)
    return st, _lib.load().mimi_last_error().decode()


@pytest.mark.gpu
def test_mimi_encoder_from_hub_name_matches_state_dict_engine(tmp_path, monkeypatch, state_dict, golden):
    """MimiEncoder("kyutai/mimi", device="cuda:0") built from an HF-layout snapshot in the offline hub cache gives
    the state-dict engine's codes bit for bit on the golden 5-item batch (pad-to-longest + trim), on a single-item
    encode_audio_chunk, and at K = 8 (the shard scripts' slice)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.encoder import MimiEncoder
    from mimi_hip.model import MimiHipModel
    monkeypatch.delenv("MIMI_HIP_CHECKPOINT", raising=False)
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "hub"))
    write_hf_checkpoint(state_dict, hub_snapshot_dir(str(tmp_path / "hub")))
    hub = MimiEncoder("kyutai/mimi", device="cuda:0")
    assert hub.model.config.num_quantizers == 32 and hub.model.config.upsampling_ratios == [8, 6, 5, 4]
    ref_engine = MimiHipModel(state_dict, device="cuda:0")
    ref = MimiEncoder(device="cuda:0", model=ref_engine)
    arrays, meta = golden
    audio = [synthetic.speech_like(L, meta["audio_seed"], 200 + i) for i, L in enumerate(meta["batch_lengths"])]
    got, want = hub.encode_audio_batch(audio, 24000), ref.encode_audio_batch(audio, 24000)
    assert len(got) == len(want) == len(audio)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g.dtype == np.int64 and g.shape == w.shape and np.array_equal(g, w), i
    assert np.array_equal(hub.encode_audio_chunk(audio[3], 24000), ref.encode_audio_chunk(audio[3], 24000))
    x = torch.from_numpy(synthetic.clip_batch(2, 48000, seed=5)).cuda()
    assert torch.equal(hub.model.encode_int32(x, 8), ref_engine.encode_int32(x, 8))
    # the f16x3 calibration saw the same weights: identical fixed activation scales
    sa, sb = hub.model.act_scales(), ref_engine.act_scales()
    assert sa.keys() == sb.keys() and all(sa[k][0] == sb[k][0] for k in sa)
    assert hub.model.f16_reruns == 0


@pytest.mark.gpu
def test_malformed_checkpoints_fail_with_status(tmp_path):
    """An F16 encode-path tensor and a missing tensor -> MIMI_ERR_WEIGHTS (4); a truncated file or a corrupt header
    -> MIMI_ERR_IO (6); decode-only tensors in another dtype are skipped unread.  The Python constructor raises
    MimiHipError with the same status."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip import _lib
    from mimi_hip.model import MimiHipModel
    lib = _lib.load()
    sd = synthetic.make_state_dict(seed=0, num_quantizers=2)

    def engine():
        h = ctypes.c_void_p()
        _lib.check(lib.mimi_create(None, 0, ctypes.byref(h)))
        return h

    w0 = "encoder.layers.0.conv.weight"
    p16 = write_hf_checkpoint(sd, str(tmp_path / "f16"), overrides={w0: sd[w0].astype(np.float16)})
    h = engine()
    st, msg = _status(lib.mimi_load_safetensors, h, p16.encode())
    lib.mimi_destroy(h)
    assert st == 4 and "F16" in msg, (st, msg)

    gone = "encoder_transformer.layers.3.mlp.fc2.weight"
    pmiss = write_hf_checkpoint(sd, str(tmp_path / "missing"), overrides={gone: None})
    h = engine()
    assert lib.mimi_load_safetensors(h, pmiss.encode()) == 0
    st, msg = _status(lib.mimi_finalize, h)
    lib.mimi_destroy(h)
    assert st == 4 and gone in msg, (st, msg)
    with pytest.raises(_lib.MimiHipError) as ei:
        MimiHipModel.from_pretrained(str(tmp_path / "missing"), device="cuda:0")
    assert ei.value.status == 4

    pok = write_hf_checkpoint(sd, str(tmp_path / "ok"), decoder_dtype=np.float16)
    h = engine()
    assert lib.mimi_load_safetensors(h, pok.encode()) == 0  # F16 decoder tensors: skipped, not an error
    assert lib.mimi_finalize(h) == 0
    lib.mimi_destroy(h)

    blob = open(pok, "rb").read()
    for name, data in (("trunc_data", blob[:len(blob) // 2]), ("trunc_header", blob[:100]),
                       ("bad_len", (len(blob) * 4).to_bytes(8, "little") + blob[8:]),
                       ("bad_json", blob[:8] + b"[" + blob[9:]), ("empty", b"")):
        p = tmp_path / f"{name}.safetensors"
        p.write_bytes(data)
        h = engine()
        st, msg = _status(lib.mimi_load_safetensors, h, str(p).encode())
        lib.mimi_destroy(h)
        assert st == 6, (name, st, msg)
    h = engine()
    st, _ = _status(lib.mimi_load_safetensors, h, str(tmp_path / "does_not_exist.safetensors").encode())
    lib.mimi_destroy(h)
    assert st == 6


# ---- the one-call C constructor: mimi_config_from_json + mimi_create_from_dir --------------------------------------

def _c_config_from_json(path):
    """C: config.json -> (status, struct as a dict, message)."""
    from mimi_hip import _lib
    lib = _lib.load()
    c = _lib.MimiConfigC()
    st = lib.mimi_config_from_json(str(path).encode(), ctypes.byref(c))
    msg = lib.mimi_last_error().decode()
    d = {name: (list(getattr(c, name)) if name == "upsampling_ratios" else getattr(c, name))
         for name, _ in _lib.MimiConfigC._fields_}
    return st, d, msg


def _py_config_struct(path):
    """The Python host's reading of the same file (MimiConfig.from_json + validate_supported + config_from_py)."""
    from mimi_hip import _lib
    cfg = MimiConfig.from_json(str(path))
    cfg.validate_supported()
    c = _lib.config_from_py(cfg)
    return {name: (list(getattr(c, name)) if name == "upsampling_ratios" else getattr(c, name))
            for name, _ in _lib.MimiConfigC._fields_}


def _variant(tmp_path, name, edit):
    import json
    with open(os.path.join(GOLDEN, "mimi_config.json")) as f:
        raw = json.load(f)
    edit(raw)
    p = tmp_path / f"{name}.json"
    p.write_text(json.dumps(raw, indent=1))
    return p


def test_c_config_from_json_equals_python_host(tmp_path):
    """CPU, C ABI only: the golden config.json (transformers 5.15.0 MimiConfig()) and variants of it read by
    mimi_config_from_json give the struct the Python host builds from MimiConfig.from_json, field for field --
    rope_theta at the top level, head_dim null, a frame_rate override (the downsample kernel follows it), other
    ratios, and unknown keys; a directory path reads its config.json."""
    st, got, msg = _c_config_from_json(os.path.join(GOLDEN, "mimi_config.json"))
    assert st == 0, msg
    assert got == _py_config_struct(os.path.join(GOLDEN, "mimi_config.json"))
    assert got["downsample_kernel"] == 4 and got["head_dim"] == 64 and got["rope_theta"] == 10000.0
    variants = {
        "top_rope": lambda r: (r.pop("rope_parameters"), r.__setitem__("rope_theta", 5000.0)),
        "head_dim_null": lambda r: r.__setitem__("head_dim", None),
        "frame_rate_25": lambda r: r.__setitem__("frame_rate", 25.0),
        "ratios": lambda r: r.__setitem__("upsampling_ratios", [8, 6, 5, 2]),
        "ratios_null": lambda r: r.__setitem__("upsampling_ratios", None),
        "unknown_keys": lambda r: r.update({"foo": {"bar": [1, 2, {"baz": "é\\n"}]}, "num_quantizers": 16}),
        "eps": lambda r: r.__setitem__("norm_eps", 1e-6),
    }
    for name, edit in variants.items():
        p = _variant(tmp_path, name, edit)
        st, got, msg = _c_config_from_json(p)
        assert st == 0, (name, msg)
        assert got == _py_config_struct(p), name
    assert _c_config_from_json(tmp_path / "frame_rate_25.json")[1]["downsample_kernel"] == 2
    d = tmp_path / "ckpt"
    d.mkdir()
    (d / "config.json").write_text((tmp_path / "eps.json").read_text())
    st, got, _ = _c_config_from_json(d)
    assert st == 0 and abs(got["norm_eps"] - 1e-6) < 1e-12


def test_c_config_from_json_rejects_what_python_rejects(tmp_path):
    """Architectures outside the kyutai/mimi family -> MIMI_ERR_UNSUPPORTED (5) with the Python host's wording
    (MimiConfig.validate_supported raises ValueError for the same files); malformed JSON, a field of the wrong type
    or a missing file -> MIMI_ERR_IO (6)."""
    unsupported = {
        "stereo": (lambda r: r.__setitem__("audio_channels", 2), "audio_channels must be 1 (mono)"),
        "gqa": (lambda r: r.__setitem__("num_key_value_heads", 4), "GQA"),
        "noncausal": (lambda r: r.__setitem__("use_causal_conv", False), "use_causal_conv must be True"),
        "reflect": (lambda r: r.__setitem__("pad_mode", "reflect"), "pad_mode must be 'constant'"),
        "two_layers": (lambda r: r.__setitem__("num_residual_layers", 2), "num_residual_layers must be 1"),
        "silu": (lambda r: r.__setitem__("hidden_act", "silu"), "hidden_act must be 'gelu'"),
        "bias": (lambda r: r.__setitem__("attention_bias", True), "attention_bias must be False"),
        "head_dim": (lambda r: r.__setitem__("head_dim", 32), "head_dim * num_attention_heads"),
    }
    for name, (edit, words) in unsupported.items():
        p = _variant(tmp_path, name, edit)
        st, _, msg = _c_config_from_json(p)
        assert st == 5 and words in msg, (name, st, msg)
        with pytest.raises(ValueError, match=words.replace("*", r"\*").replace("(", r"\(").replace(")", r"\)")):
            _py_config_struct(p)
    bad = {"truncated": '{"hidden_size": 512', "trailing": "{} x", "not_object": "[1, 2]",
           "bad_number": '{"hidden_size": 5.1.2}', "string_int": '{"hidden_size": "512"}',
           "float_int": '{"kernel_size": 7.5}', "bad_escape": '{"a": "\\q"}', "ctrl": '{"a": "x\ty"}',
           "deep": "[" * 100 + "]" * 100, "empty": ""}
    for name, text in bad.items():
        p = tmp_path / f"bad_{name}.json"
        p.write_text(text)
        st, _, msg = _c_config_from_json(p)
        assert st == 6 and msg, (name, st, msg)
    st, _, msg = _c_config_from_json(tmp_path / "does_not_exist.json")
    assert st == 6 and "does_not_exist" in msg


def test_c_create_from_dir_checks_before_the_device(tmp_path):
    """CPU: mimi_create_from_dir reads config.json and picks the checkpoint file before it touches a device -- an
    unsupported config (5), a directory without .safetensors (6) and a missing path (6) fail the same on any host;
    a well-formed directory gets as far as the device (here: none, so MIMI_ERR_HIP or MIMI_ERR_INVALID_ARGUMENT),
    and *out stays NULL on every failure."""
    from mimi_hip import _lib
    if torch.cuda.is_available():
        pytest.skip("CPU-only check (the GPU test below creates a real engine)")
    lib = _lib.load()

    def create(path):
        h = ctypes.c_void_p(1234)
        st = lib.mimi_create_from_dir(str(path).encode(), 0, ctypes.byref(h))
        return st, h.value, lib.mimi_last_error().decode()

    d = tmp_path / "stereo"
    d.mkdir()
    (d / "config.json").write_text(_variant(tmp_path, "s", lambda r: r.__setitem__("audio_channels", 2)).read_text())
    (d / "model.safetensors").write_bytes(b"\0" * 16)
    st, h, msg = create(d)
    assert st == 5 and h is None and "audio_channels" in msg
    e = tmp_path / "empty"
    e.mkdir()
    (e / "config.json").write_text(open(os.path.join(GOLDEN, "mimi_config.json")).read())
    (e / ".hidden.safetensors").write_bytes(b"\0" * 16)  # (glob skips dot files)
    st, h, msg = create(e)
    assert st == 6 and h is None and "no .safetensors" in msg
    st, h, msg = create(tmp_path / "missing")
    assert st == 6 and h is None
    sd = synthetic.make_state_dict(seed=0, num_quantizers=2)
    ok = tmp_path / "ok"
    write_hf_checkpoint(sd, str(ok))
    st, h, msg = create(ok)
    assert st in (1, 2) and h is None, (st, msg)


@pytest.mark.gpu
def test_c_create_from_dir_matches_from_pretrained(tmp_path, state_dict):
    """GPU, C ABI only: an engine from mimi_create_from_dir on an HF-layout directory (config.json + model.safetensors
    with decoder tensors beside the encode path) encodes the codes of MimiHipModel.from_pretrained on the same
    directory, bit for bit (mimi_encode on the caller's device buffers, K = 8 and 32); a lone .safetensors file
    works too (default config)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip import _lib
    from mimi_hip.model import MimiHipModel
    lib = _lib.load()
    d = tmp_path / "ckpt"
    st_path = write_hf_checkpoint(state_dict, str(d))
    ref = MimiHipModel.from_pretrained(str(d), device="cuda:0")
    x = torch.from_numpy(synthetic.clip_batch(3, 72000, seed=11)).cuda()
    for path in (d, st_path):
        h = ctypes.c_void_p()
        _lib.check(lib.mimi_create_from_dir(str(path).encode(), 0, ctypes.byref(h)))
        try:
            for K in (8, 32):
                T = lib.mimi_encoded_length(72000)
                out = torch.empty(3, K, T, dtype=torch.int32, device="cuda:0")
                torch.cuda.synchronize()
                _lib.check(lib.mimi_encode(h, ctypes.c_void_p(x.data_ptr()), 3, 72000, K,
                                           ctypes.c_void_p(out.data_ptr()), None))
                torch.cuda.synchronize()
                want = ref.encode_int32(x, K)
                assert torch.equal(out, want.view_as(out)), (str(path), K)
        finally:
            lib.mimi_destroy(h)
