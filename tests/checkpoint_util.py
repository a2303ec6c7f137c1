"""Test helper: write a Mimi state dict as an HF-layout checkpoint directory (model.safetensors + config.json), the
layout of the ``kyutai/mimi`` Hub repo that ``MimiModel.from_pretrained`` reads (emilia-mimi/process_shard.py:57-60).

Besides the encode-path tensors a real checkpoint holds the decoder half and the quantizer's
decode-only projections; a few of those are written too (with the real names) so the loader's skip rules are
exercised -- the engine must read the encode path and ignore the rest.
"""
import os
import shutil

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# decode-only tensors of the HF MimiModel (TF/modeling_mimi.py: MimiDecoder, upsample, output_proj), small shapes
DECODE_ONLY = {
    "decoder.layers.0.conv.weight": (8, 4, 7),
    "decoder.layers.0.conv.bias": (8,),
    "decoder.layers.2.conv.weight": (4, 8, 16),
    "decoder_transformer.layers.0.self_attn.q_proj.weight": (16, 16),
    "upsample.conv.weight": (16, 1, 4),
    "quantizer.semantic_residual_vector_quantizer.output_proj.weight": (16, 8, 1),
    "quantizer.acoustic_residual_vector_quantizer.output_proj.weight": (16, 8, 1),
}


def write_hf_checkpoint(sd, directory, decoder_dtype=np.float32, overrides=None):
    """sd: {name: float32 array} -> directory/model.safetensors (+ config.json from the golden fixture)."""
    from safetensors.numpy import save_file
    os.makedirs(directory, exist_ok=True)
    tensors = {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in sd.items()}
    rng = np.random.default_rng(0)
    for k, shape in DECODE_ONLY.items():
        tensors[k] = rng.standard_normal(shape).astype(decoder_dtype)
    for k, v in (overrides or {}).items():
        if v is None:
            tensors.pop(k, None)
        else:
            tensors[k] = v
    path = os.path.join(directory, "model.safetensors")
    save_file(tensors, path, metadata={"format": "pt"})
    shutil.copy(os.path.join(GOLDEN, "mimi_config.json"), os.path.join(directory, "config.json"))
    return path


def hub_snapshot_dir(cache_root, repo_id="kyutai/mimi", revision="0123456789abcdef0123456789abcdef01234567"):
    """$HF_HUB_CACHE/models--<org>--<name>/snapshots/<revision> (huggingface_hub's cache layout)."""
    repo = os.path.join(cache_root, "models--" + repo_id.replace("/", "--"))
    d = os.path.join(repo, "snapshots", revision)
    os.makedirs(d, exist_ok=True)
    os.makedirs(os.path.join(repo, "refs"), exist_ok=True)
    with open(os.path.join(repo, "refs", "main"), "w") as f:
        f.write(revision)
    return d
