"""Generate tests/golden/segmenter.json (run in the survey container only; the output is committed).

    python tests/golden/make_segmenter_golden.py

Drives the reference's own ``SubShardProcessor.process_audio_entry`` (``/root/reference/yodas2-mimi/
process_shard.py:373-533``) on synthetic entries with a ``RecordingEncoder`` (tests/golden/recording_encoder.py)
in place of the model, and records, per case: the entry, the waveform's seed and length, the encoder call log
(kind + lengths, i.e. the exact batching) and the resulting ``codes`` dict.  ``librosa`` is absent: the
module is stubbed with a ``load`` that returns the case's seeded waveform (the reference calls it once per
entry, ``:389``); the audio file it globs for is an empty placeholder in a temp dir.
"""
import importlib.machinery
import importlib.util
import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from recording_encoder import RecordingEncoder  # noqa: E402

REF = "/root/reference/yodas2-mimi/process_shard.py"
SR = 24000


def waveform(seed, n):
    return np.random.default_rng(seed).normal(0.0, 0.1, n).astype(np.float32)


def cid(audio_id, i, s, e):
    return f"{audio_id}-{i:05d}-{s:08d}-{e:08d}"


def cases():
    out = []
    # 1. mixed chunks: normal, a zero-length one (skipped), long ones (split), one past the end (skipped)
    a = "Y65x5_9PNO8"
    spans = [(0, 250), (250, 900), (900, 900), (900, 2300), (2300, 2350), (2350, 2351), (2400, 4400),
             (4400, 4700), (4700, 4750), (4750, 5000), (5000, 5600), (5600, 5610), (9000, 9100), (5610, 5900)]
    out.append({"name": "mixed", "audio_id": a, "seed": 1, "n": int(58.0 * SR),
                "text": {cid(a, i, s, e): f"t{i}" for i, (s, e) in enumerate(spans)},
                "batch_size": 3, "max_chunk_duration": 5.0})
    # 2. hyphenated audio id, chunk running past the end (truncated slice), batch larger than the entry
    a = "Yg-Y2--S7q8"
    spans = [(100, 400), (400, 1000), (1000, 1900), (1900, 2600)]
    out.append({"name": "hyphen_id_truncated", "audio_id": a, "seed": 2, "n": int(22.5 * SR),
                "text": {cid(a, i, s, e): f"t{i}" for i, (s, e) in enumerate(spans)},
                "batch_size": 8, "max_chunk_duration": 60.0})
    # 3. long chunk first and last, exact multiple of the split size, single-chunk batches
    a = "abc"
    spans = [(0, 1200), (1200, 1300), (1300, 1301), (1301, 2500), (2500, 2900)]
    out.append({"name": "long_edges", "audio_id": a, "seed": 3, "n": int(30.0 * SR),
                "text": {cid(a, i, s, e): f"t{i}" for i, (s, e) in enumerate(spans)},
                "batch_size": 1, "max_chunk_duration": 4.0})
    # 4. every chunk filtered out
    a = "empty"
    out.append({"name": "all_filtered", "audio_id": a, "seed": 4, "n": int(1.0 * SR),
                "text": {cid(a, 0, 50, 50): "x", cid(a, 1, 500, 600): "y"},
                "batch_size": 4, "max_chunk_duration": 60.0})
    return out


def main():
    # import transformers' Mimi classes before stubbing librosa, so its optional-import probes see the real
    # environment (as tests/golden/make_golden.py does)
    from transformers import AutoFeatureExtractor, MimiModel  # noqa: F401
    librosa = types.ModuleType("librosa")
    librosa.__spec__ = importlib.machinery.ModuleSpec("librosa", None)
    current = {}
    librosa.load = lambda path, sr=None: (current["wave"], sr)
    sys.modules["librosa"] = librosa
    spec = importlib.util.spec_from_file_location("yodas2_process_shard", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)

    results = []
    with tempfile.TemporaryDirectory() as tmp:
        for c in cases():
            d = Path(tmp) / c["name"]
            d.mkdir()
            (d / f"{c['audio_id']}.wav").write_bytes(b"")
            current["wave"] = waveform(c["seed"], c["n"])
            enc = RecordingEncoder()
            proc = object.__new__(mod.SubShardProcessor)
            proc.encoder, proc.batch_size, proc.max_chunk_duration = enc, c["batch_size"], c["max_chunk_duration"]
            proc.audio_extract_dir = d
            entry = {"audio_id": c["audio_id"], "text": dict(c["text"])}
            res = proc.process_audio_entry(entry, sample_rate=SR)
            c = dict(c, calls=enc.calls, codes=res["codes"])
            results.append(c)
            print(f"{c['name']}: {len(c['calls'])} encoder calls, {len(c['codes'])} chunks coded")
        # start > end raises
        d = Path(tmp) / "bad"
        d.mkdir()
        (d / "bad.wav").write_bytes(b"")
        current["wave"] = waveform(5, SR)
        proc = object.__new__(mod.SubShardProcessor)
        proc.encoder, proc.batch_size, proc.max_chunk_duration = RecordingEncoder(), 2, 60.0
        proc.audio_extract_dir = d
        try:
            proc.process_audio_entry({"audio_id": "bad", "text": {cid("bad", 0, 90, 10): "z"}}, sample_rate=SR)
            raised = None
        except ValueError as e:
            raised = str(e)
    meta = {"source": "yodas2-mimi/process_shard.py:373-533 (SubShardProcessor.process_audio_entry)",
            "sample_rate": SR, "waveform": "numpy default_rng(seed).normal(0, 0.1, n) float32",
            "bad_start_after_end_error": raised}
    with open(os.path.join(HERE, "segmenter.json"), "w") as f:
        json.dump({"meta": meta, "cases": results}, f, separators=(",", ":"))
    print("wrote segmenter.json")


if __name__ == "__main__":
    main()
