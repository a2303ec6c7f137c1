"""CPU: the YODAS2 segmenter / batch scheduler (mimi_hip.segmenter) against the reference's own
``SubShardProcessor.process_audio_entry`` (yodas2-mimi/process_shard.py:373-533), pinned by
tests/golden/segmenter.json (made by tests/golden/make_segmenter_golden.py with a recording encoder)."""
import copy
import json
import os
import sys

import numpy as np
import pytest

from mimi_hip.segmenter import encode_segments, parse_chunk_id, process_audio_entry, slice_segments

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
from recording_encoder import RecordingEncoder, fake_codes  # noqa: E402


def _golden():
    with open(os.path.join(GOLDEN, "segmenter.json")) as f:
        return json.load(f)


def _wave(seed, n):
    return np.random.default_rng(seed).normal(0.0, 0.1, n).astype(np.float32)


G = _golden()


@pytest.mark.parametrize("case", G["cases"], ids=[c["name"] for c in G["cases"]])
def test_segmenter_matches_reference(case):
    enc = RecordingEncoder()
    entry = {"audio_id": case["audio_id"], "text": dict(case["text"])}
    res = process_audio_entry(entry, _wave(case["seed"], case["n"]), enc, batch_size=case["batch_size"],
                              max_chunk_duration=case["max_chunk_duration"])
    assert enc.calls == case["calls"]           # the same slices, batches and long-chunk pieces, in order
    assert list(res["codes"]) == list(case["codes"])
    assert res["codes"] == case["codes"]        # uint16 lists, as the reference stores them


def test_start_after_end_raises():
    with pytest.raises(ValueError) as e:
        process_audio_entry({"audio_id": "bad", "text": {"bad-00000-00000090-00000010": "z"}}, _wave(5, 24000),
                            RecordingEncoder(), batch_size=2)
    assert str(e.value) == G["meta"]["bad_start_after_end_error"]


def test_missing_audio_leaves_entry_alone():
    entry = {"audio_id": "x", "text": {"x-00000-00000000-00000100": "a"}}
    assert "codes" not in process_audio_entry(entry, None, RecordingEncoder())


def test_parse_chunk_id():
    assert parse_chunk_id("Yg-Y2--S7q8-00026-00003279-00003300") == ("Yg-Y2--S7q8", "00026", 3279, 3300)
    # the reference asserts four parts (yodas2-mimi/process_shard.py:405) and never parses the index field
    with pytest.raises(AssertionError, match="Invalid chunk_id format"):
        parse_chunk_id("no-dashes")
    assert parse_chunk_id("a-idx-00000001-00000002")[1] == "idx"


def test_bucketed_mode_same_chunks_fewer_pad_samples():
    """Throughput mode: the same chunk set and per-chunk codes for an encoder whose output does not depend
    on batch composition (the recording encoder), and less padding than parity mode."""
    case = next(c for c in G["cases"] if c["name"] == "mixed")
    wave = _wave(case["seed"], case["n"])
    segs = slice_segments(wave, case["text"], 24000, case["max_chunk_duration"])
    ref = encode_segments(RecordingEncoder(), segs, case["batch_size"], 24000, case["max_chunk_duration"])
    enc = RecordingEncoder()
    got = encode_segments(enc, segs, case["batch_size"], 24000, case["max_chunk_duration"], bucketed=True)
    assert list(got) == list(ref)
    assert all(np.array_equal(got[k], ref[k]) for k in ref)

    def pad(calls):
        return sum(len(ls) * max(ls) - sum(ls) for kind, ls in calls if kind == "batch")

    assert pad(enc.calls) <= pad(case["calls"])


def test_long_chunk_codes_are_concatenated_pieces():
    wave = _wave(9, 24000 * 11)
    segs = slice_segments(wave, {"a-00000-00000000-00001100": "t"}, 24000, max_chunk_duration=4.0)
    assert len(segs) == 1 and segs[0].long
    out = encode_segments(RecordingEncoder(), segs, 4, 24000, 4.0)["a-00000-00000000-00001100"]
    want = np.concatenate([fake_codes(wave[s:s + 96000]) for s in range(0, len(wave), 96000)], axis=1)
    assert out.dtype == np.uint16 and np.array_equal(out, want.astype(np.uint16))


def test_input_entry_text_not_mutated():
    case = G["cases"][0]
    text = copy.deepcopy(case["text"])
    process_audio_entry({"audio_id": case["audio_id"], "text": text}, _wave(case["seed"], case["n"]),
                        RecordingEncoder(), batch_size=case["batch_size"], max_chunk_duration=case["max_chunk_duration"])
    assert text == case["text"]
