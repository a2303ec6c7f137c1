"""Generate the golden fixtures (run in the survey container only; outputs are committed).

    python tests/golden/make_golden.py

The reference's arithmetic lives in third-party ``transformers`` 5.15.0 (``MimiModel``), importable here but
not on the GPU box, and the reference repo ships no tests or golden vectors, so the fixtures
are generated here from:

* ``transformers.MimiModel`` loaded with the seeded synthetic checkpoint (``mimi_hip.synthetic``; its SHA-256
  is stored and re-checked on the box) -- model-level codes for a set of lengths, the pre-quantizer
  embeddings and per-code top-2 distance margins;
* the reference's own ``MimiEncoder`` wrapper class (``/root/reference/libritts-r-mimi/process_libritts_r.py:33-105``,
  identical to the other copies) driving that model, for the pad-to-longest / trim batch semantics;
* the reference's ``utils.codes_to_chars`` (``/root/reference/librispeech-mimi/utils.py:18-37``).

Missing third-party modules the reference scripts import at module level (librosa, not installed) are
stubbed with empty modules; nothing from them is called.  The oracle restatement (``oracle/mimi_ref.py``) is
checked against ``transformers`` here: identical codes and bit-identical per-stage tensors.
"""
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden")
REF = "/root/reference"

from mimi_hip import synthetic  # noqa: E402
from mimi_hip.config import MimiConfig, encoded_length  # noqa: E402
from oracle import mimi_ref  # noqa: E402

LENGTHS = [1, 1919, 1920, 1921, 24000, 72007, 240000, 1440000]
BATCH_LENGTHS = [150001, 240000, 37000, 1921, 96000]
AUDIO_SEED = 7


def stub_module(name):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    sys.modules[name] = m
    return m


def load_reference_module(path, name):
    d = os.path.dirname(path)
    sys.path.insert(0, d)
    try:
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod
    finally:
        sys.path.remove(d)
        sys.modules.pop("utils", None)


def main():
    torch.set_num_threads(8)
    import transformers  # noqa: F401  (import before stubbing so its own optional-import probes are clean)
    from transformers import EncodecFeatureExtractor, MimiConfig as TMimiConfig, MimiModel
    stub_module("librosa")

    cfg = MimiConfig()
    sd = synthetic.make_state_dict(cfg, seed=0)
    sha = synthetic.state_dict_sha256(sd)
    model = MimiModel(TMimiConfig()).eval()
    res = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not res.unexpected_keys, res.unexpected_keys
    assert all(k.startswith(("decoder", "upsample")) or "output_proj" in k for k in res.missing_keys), \
        [k for k in res.missing_keys if not k.startswith(("decoder", "upsample"))]
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    rc = mimi_ref.RefConfig()

    meta = {"weights_seed": 0, "weights_sha256": sha, "audio_seed": AUDIO_SEED, "transformers": "5.15.0",
            "torch": torch.__version__, "lengths": LENGTHS, "batch_lengths": BATCH_LENGTHS}
    arrays = {}
    audio_hashes = {}

    # ---- 1. model-level codes (K = 32; K = 8 is a prefix, checked) + oracle agreement ----
    with torch.no_grad():
        for i, L in enumerate(LENGTHS):
            x = synthetic.speech_like(L, AUDIO_SEED, i)
            audio_hashes[str(L)] = synthetic.audio_sha256([x])
            xt = torch.from_numpy(x)[None, None]
            codes = model.encode(xt).audio_codes[0]
            codes8 = model.encode(xt, num_quantizers=8).audio_codes[0]
            assert torch.equal(codes[:8], codes8), "prefix property"
            ora = mimi_ref.encode(xt, sd)[0]
            assert torch.equal(ora, codes), f"oracle != transformers at L={L}"
            assert codes.shape[-1] == encoded_length(L), (codes.shape, encoded_length(L))
            arrays[f"codes_L{L}"] = codes.numpy().astype(np.int16)
            print(f"L={L:8d} T={codes.shape[-1]:4d} distinct L0 codes {len(np.unique(codes[0]))}")

        # ---- 2. pre-quantizer embeddings + codes + margins for the bit-exact quantizer test ----
        for tag, x in (("speech10s", synthetic.speech_like(240000, AUDIO_SEED, 6)),
                       ("speech60s", synthetic.speech_like(1440000, AUDIO_SEED, 7)),
                       ("noise5s", synthetic.noise_clip(120000, AUDIO_SEED, 0, std=0.1))):
            xt = torch.from_numpy(x)[None, None]
            taps = {}
            codes = mimi_ref.encode(xt, sd, taps=taps)
            emb = taps["pre_quantizer"]
            # transformers' own pre-quantizer tensor for the same input (bit-identical check)
            e2 = model.encoder(xt)
            e2 = model.encoder_transformer(e2.transpose(1, 2), return_dict=False)[0].transpose(1, 2)
            e2 = model.downsample(e2)
            assert torch.equal(e2, emb), f"oracle pre-quantizer != transformers ({tag})"
            c2, margins = mimi_ref.rvq_from_embedding(emb, sd, 32, rc, return_margins=True)
            assert torch.equal(c2, codes)
            arrays[f"emb_{tag}"] = emb[0].numpy()
            arrays[f"embcodes_{tag}"] = codes[0].numpy().astype(np.int16)
            arrays[f"margins_{tag}"] = margins[0].numpy().astype(np.float32)
            audio_hashes[tag] = synthetic.audio_sha256([x])
            print(f"{tag}: min rel margin {float(margins.min()):.3e}")

        # ---- 3. per-stage tensors for a 0.5 s clip (channel-first, reference layout) ----
        x = synthetic.speech_like(12000, AUDIO_SEED, 100)
        audio_hashes["stage12000"] = synthetic.audio_sha256([x])
        taps = {}
        mimi_ref.encode(torch.from_numpy(x)[None, None], sd, taps=taps)
        for name, t in taps.items():
            t = t[0]
            sub = 1
            while t.numel() // sub > 100_000:
                sub *= 2
            arrays[f"stage_{name}_sub{sub}"] = t[..., ::sub].numpy() if name.startswith(("conv", "res", "down")) \
                else t.numpy()
        enc = model.encoder(torch.from_numpy(x)[None, None])[0]
        assert torch.equal(enc, taps["encoder"][0]), "oracle encoder != transformers encoder"

    # ---- 4. the reference MimiEncoder wrapper: chunk + padded batch semantics ----
    wrap_mod = load_reference_module(os.path.join(REF, "libritts-r-mimi", "process_libritts_r.py"), "ref_libritts")
    enc = object.__new__(wrap_mod.MimiEncoder)
    enc.device = "cpu"
    enc.model = model
    enc.feature_extractor = EncodecFeatureExtractor(feature_size=1, sampling_rate=24000, padding_value=0.0)
    batch_audio = [synthetic.speech_like(L, AUDIO_SEED, 200 + i) for i, L in enumerate(BATCH_LENGTHS)]
    audio_hashes["batch"] = synthetic.audio_sha256(batch_audio)
    outs = enc.encode_audio_batch(batch_audio, 24000)
    for i, o in enumerate(outs):
        arrays[f"batch_item{i}"] = o.astype(np.int16)
    single = enc.encode_audio_batch([batch_audio[2]], 24000)[0]
    arrays["batch_single"] = single.astype(np.int16)
    chunk = enc.encode_audio_chunk(batch_audio[3], 24000)
    arrays["chunk_item3"] = chunk.astype(np.int16)
    assert enc.encode_audio_batch([], 24000) == []
    fe = enc.feature_extractor(raw_audio=batch_audio[:2], sampling_rate=24000, return_tensors="pt", padding=True)
    meta["feature_extractor"] = {k: [str(v.dtype), list(v.shape)] for k, v in fe.items()}
    print("batch shapes", [o.shape for o in outs])

    # ---- 5. codes_to_chars from the reference utils ----
    utils_mod = load_reference_module(os.path.join(REF, "librispeech-mimi", "utils.py"), "ref_utils")
    c8 = arrays["codes_L240000"][:8].astype(np.int64)
    s = utils_mod.codes_to_chars(c8, codebook_size=2048)
    back = utils_mod.chars_to_codes(s, num_codebooks=8, codebook_size=2048)
    assert back == c8.tolist()
    with open(os.path.join(OUT, "codes_to_chars.json"), "w") as f:
        json.dump({"codes": c8.tolist(), "chars_utf32": [ord(ch) for ch in s]}, f)

    meta["audio_sha256"] = audio_hashes
    with open(os.path.join(OUT, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    np.savez_compressed(os.path.join(OUT, "golden.npz"), **arrays)
    print("wrote", os.path.join(OUT, "golden.npz"), os.path.getsize(os.path.join(OUT, "golden.npz")), "bytes")


if __name__ == "__main__":
    main()
