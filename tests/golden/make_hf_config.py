"""Writes tests/golden/mimi_config.json: the HF ``config.json`` of a Mimi checkpoint, as ``transformers``
(5.15.0) serialises ``MimiConfig()`` -- the encode-path fields equal kyutai/mimi's.  The real-
checkpoint boundary test (tests/test_checkpoint.py) places it beside an HF-layout model.safetensors under
$HF_HUB_CACHE/models--kyutai--mimi/snapshots/<rev>/, the layout ``MimiModel.from_pretrained("kyutai/mimi")`` reads
(emilia-mimi/process_shard.py:57-60).  Run in the build container (transformers importable):

    python tests/golden/make_hf_config.py
"""
import json
import os

from transformers import MimiConfig

HERE = os.path.dirname(os.path.abspath(__file__))

if __name__ == "__main__":
    cfg = json.loads(MimiConfig().to_json_string())
    cfg["architectures"] = ["MimiModel"]
    with open(os.path.join(HERE, "mimi_config.json"), "w") as f:
        json.dump(cfg, f, indent=2, sort_keys=True)
        f.write("\n")
    print("wrote", os.path.join(HERE, "mimi_config.json"), len(cfg), "fields")
