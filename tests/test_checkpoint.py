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
