"""Golden fixtures for the padded-batch path (run in the survey container only; outputs are committed).

    python tests/golden/make_golden_batch.py

Every batched reference shard script encodes through ``MimiEncoder.encode_audio_batch`` (pad to the longest
item with zeros, one ``MimiModel.encode``, trim item i to ``ceil(L_i / 1920)`` frames:
``/root/reference/emilia-mimi/process_shard.py:88-140``, identical in the other copies).  This script drives
the reference's own wrapper class (``/root/reference/libritts-r-mimi/process_libritts_r.py:33-105``) around
``transformers`` 5.15.0 ``MimiModel`` loaded with the seeded synthetic checkpoint on a B = 32 batch of
mixed-length clips (U[1.5, 20] s, some longer than 10.24 s so the window-250 attention path runs, two of them
at -40 dB and -60 dB), and stores per item:

* the wrapper's int64 codes (K = 32, the wrapper's default), as uint16;
* the top-2 relative distance margins of every code, computed by the oracle (``oracle/mimi_ref.py``) on the
  SAME padded batch -- the oracle's codes on that batch are asserted equal to the wrapper's, so the margins
  belong to the reference's own embedding -- for the near-tie audit of ``tests/test_gpu_parity.py``.

The audio is regenerated on the GPU box from ``mimi_hip.synthetic`` (hashes stored); no reference code or text
is stored, only inputs' seeds and outputs.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import OUT, REF, load_reference_module, stub_module  # noqa: E402

from mimi_hip import synthetic  # noqa: E402
from oracle import mimi_ref  # noqa: E402

B = 32
LEN_SEED = 21
AUDIO_SEED = 7
QUIET = {3: 0.01, 7: 0.001}  # item -> gain (-40 dB, -60 dB)


def batch_audio():
    lengths = synthetic.random_lengths(B, 1.5, 20.0, seed=LEN_SEED)
    audio = []
    for i, L in enumerate(lengths):
        a = synthetic.speech_like(L, AUDIO_SEED, 400 + i)
        if i in QUIET:
            a = a * np.float32(QUIET[i])
        audio.append(a)
    return lengths, audio


def main():
    torch.set_num_threads(8)
    import transformers  # noqa: F401
    from transformers import EncodecFeatureExtractor, MimiConfig as TMimiConfig, MimiModel
    stub_module("librosa")

    sd = synthetic.make_state_dict(seed=0)
    model = MimiModel(TMimiConfig()).eval()
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)

    lengths, audio = batch_audio()
    assert sum(L > 10.24 * 24000 for L in lengths) >= 2, lengths
    wrap_mod = load_reference_module(os.path.join(REF, "libritts-r-mimi", "process_libritts_r.py"), "ref_libritts")
    enc = object.__new__(wrap_mod.MimiEncoder)
    enc.device = "cpu"
    enc.model = model
    enc.feature_extractor = EncodecFeatureExtractor(feature_size=1, sampling_rate=24000, padding_value=0.0)
    outs = enc.encode_audio_batch(audio, 24000)
    del model

    # oracle on the identical padded batch: codes must equal the wrapper's, margins for the audit
    Lmax = max(lengths)
    x = np.zeros((B, 1, Lmax), dtype=np.float32)
    for i, a in enumerate(audio):
        x[i, 0, :len(a)] = a
    taps = {}
    codes = mimi_ref.encode(torch.from_numpy(x), sd, taps=taps)
    _, margins = mimi_ref.rvq_from_embedding(taps["pre_quantizer"], sd, 32, return_margins=True)
    arrays = {}
    for i, o in enumerate(outs):
        T = o.shape[1]
        assert np.array_equal(codes[i, :, :T].numpy(), o), f"oracle != reference wrapper on item {i}"
        arrays[f"item{i}"] = o.astype(np.uint16)
        arrays[f"margin{i}"] = margins[i, :, :T].numpy().astype(np.float16)
    meta = {"B": B, "len_seed": LEN_SEED, "audio_seed": AUDIO_SEED, "audio_index0": 400,
            "quiet_gain": {str(k): v for k, v in QUIET.items()}, "lengths": lengths,
            "audio_sha256": synthetic.audio_sha256(audio), "weights_sha256": synthetic.state_dict_sha256(sd),
            "transformers": transformers.__version__, "torch": torch.__version__,
            "min_margin": float(margins.min())}
    np.savez_compressed(os.path.join(OUT, "golden_batch.npz"), **arrays)
    with open(os.path.join(OUT, "golden_batch_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("lengths (s):", [round(L / 24000, 2) for L in lengths])
    print("wrote golden_batch.npz", os.path.getsize(os.path.join(OUT, "golden_batch.npz")), "bytes")


if __name__ == "__main__":
    main()
