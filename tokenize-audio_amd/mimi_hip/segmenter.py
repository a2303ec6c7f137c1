"""YODAS2 segmenter and batch scheduler: the host side that feeds the encoder in the YODAS2 shard script.

Mirrors ``SubShardProcessor.process_audio_entry`` (``yodas2-mimi/process_shard.py:373-533``) minus the file
I/O: the caller hands over the decoded 24 kHz waveform of one audio file (the reference's ``librosa.load``,
``:389``) and the entry's ``text`` dict, whose keys are chunk ids ``{audio_id}-{index:05d}-{start_cs:08d}-
{end_cs:08d}`` with times in centiseconds.

Reference semantics kept exactly (pinned by ``tests/golden/segmenter.json``, made by driving the reference's
own method with a recording encoder):

* chunk ids split from the right, so audio ids may contain hyphens (``:404-408``);
* ``start == end`` chunks are skipped, ``start > end`` raises ``ValueError`` (``:413-422``);
* samples ``[int(start_cs * sr / 100), int(end_cs * sr / 100))`` (``:426-428``); empty slices are skipped
  (``:430-433``);
* a slice longer than ``max_chunk_duration`` seconds is a LONG chunk (``:436-442``): it is cut into pieces
  of ``int(max_chunk_duration * sr)`` samples, each encoded alone with ``encode_audio_chunk`` and the codes
  concatenated along time (``:461-485``);
* normal chunks go to ``encode_audio_batch`` in batches of up to ``batch_size`` consecutive chunks, a batch
  ending early at the next LONG chunk (``:493-519``);
* codes are stored as uint16 (``:517-519``, ``:484``).

``bucketed=True`` is this engine's throughput mode (not in the reference): the normal chunks of the entry
are batched in descending length order so each padded batch wastes less, and the output dict is in the
original chunk order.  A chunk's codes can then differ from parity mode on its LAST frame only: the padded
tail of a batch depends on its composition.  Parity mode is the default.
"""
from typing import Dict, List, Optional, Tuple

import numpy as np

__all__ = ["parse_chunk_id", "Segment", "slice_segments", "encode_segments", "process_audio_entry"]


def parse_chunk_id(chunk_id: str) -> Tuple[str, str, int, int]:
    """``{audio_id}-{index:05d}-{start_cs:08d}-{end_cs:08d}`` -> (audio_id, index, start_cs, end_cs).

    Ref ``yodas2-mimi/process_shard.py:402-412``: ``rsplit('-', 3)``, an ``AssertionError`` unless there are four
    parts, and only the two timestamps parsed as integers (the index field is never parsed, so it stays a string)."""
    parts = chunk_id.rsplit("-", 3)
    if len(parts) != 4:
        raise AssertionError(f"Invalid chunk_id format: {chunk_id}")
    return parts[0], parts[1], int(parts[2]), int(parts[3])


class Segment:
    """One chunk of an audio file: its id, its samples (a view into the file's waveform) and whether it is
    longer than the scheduler's maximum (then it is split before encoding)."""
    __slots__ = ("chunk_id", "audio", "long")

    def __init__(self, chunk_id: str, audio: np.ndarray, long: bool):
        self.chunk_id = chunk_id
        self.audio = audio
        self.long = long

    def __repr__(self):
        return f"Segment({self.chunk_id!r}, {len(self.audio)} samples{', long' if self.long else ''})"


def slice_segments(audio: np.ndarray, text_dict: Dict[str, str], sample_rate: int = 24000,
                   max_chunk_duration: float = 60.0) -> List[Segment]:
    """Cut the entry's chunks out of the file's waveform, in ``text_dict`` order (ref ``:399-442``)."""
    segs = []
    for chunk_id in text_dict:
        _, _, start_cs, end_cs = parse_chunk_id(chunk_id)
        if start_cs == end_cs:
            continue  # broken zero-length segments exist in the corpus (ref :416-419)
        if start_cs > end_cs:
            raise ValueError(f"Invalid chunk_id format: {chunk_id}")
        start = int(start_cs * sample_rate / 100)
        end = int(end_cs * sample_rate / 100)
        seg = audio[start:end]
        if len(seg) == 0:
            continue  # transcript runs past the end of the audio (ref :430-433)
        segs.append(Segment(chunk_id, seg, len(seg) / sample_rate > max_chunk_duration))
    return segs


def _encode_long(encoder, seg: Segment, sample_rate: int, max_chunk_duration: float) -> np.ndarray:
    # ref :461-485: fixed-size pieces, each encoded alone, codes concatenated along time
    step = int(max_chunk_duration * sample_rate)
    pieces = [seg.audio[s:min(s + step, len(seg.audio))] for s in range(0, len(seg.audio), step)]
    codes = [encoder.encode_audio_chunk(p, sample_rate=sample_rate) for p in pieces]
    return np.concatenate(codes, axis=1).astype(np.uint16)


def encode_segments(encoder, segments: List[Segment], batch_size: int = 32, sample_rate: int = 24000,
                    max_chunk_duration: float = 60.0, bucketed: bool = False) -> Dict[str, np.ndarray]:
    """chunk_id -> uint16 codes [K, T] for every segment, in segment order (ref ``:448-522``)."""
    if batch_size < 1:
        raise ValueError("batch_size must be >= 1")
    out: Dict[str, np.ndarray] = {}
    if bucketed:
        longs = {s.chunk_id: _encode_long(encoder, s, sample_rate, max_chunk_duration) for s in segments if s.long}
        normal = sorted((s for s in segments if not s.long), key=lambda s: -len(s.audio))  # stable
        done = {}
        for i in range(0, len(normal), batch_size):
            batch = normal[i:i + batch_size]
            for s, c in zip(batch, encoder.encode_audio_batch([s.audio for s in batch], sample_rate=sample_rate)):
                done[s.chunk_id] = c.astype(np.uint16)
        for s in segments:
            out[s.chunk_id] = longs[s.chunk_id] if s.long else done[s.chunk_id]
        return out
    i, n = 0, len(segments)
    while i < n:
        if segments[i].long:
            out[segments[i].chunk_id] = _encode_long(encoder, segments[i], sample_rate, max_chunk_duration)
            i += 1
            continue
        j = i
        while j < min(i + batch_size, n) and not segments[j].long:
            j += 1
        batch = segments[i:j]
        codes = encoder.encode_audio_batch([s.audio for s in batch], sample_rate=sample_rate)
        for s, c in zip(batch, codes):
            out[s.chunk_id] = c.astype(np.uint16)
        i = j
    return out


def process_audio_entry(entry: Dict, audio: Optional[np.ndarray], encoder, batch_size: int = 32,
                        sample_rate: int = 24000, max_chunk_duration: float = 60.0, bucketed: bool = False,
                        as_lists: bool = True) -> Dict:
    """``entry`` (with ``audio_id`` and ``text``) plus its decoded waveform -> ``entry`` with ``codes``.

    ``audio=None`` stands for a file that is missing or failed to load: the entry comes back without codes,
    as in the reference (``:378-393``).  ``as_lists`` stores ``codes.tolist()`` as the reference does (the
    JSON writer's input); ``False`` keeps the uint16 arrays."""
    if audio is None:
        return entry
    segs = slice_segments(np.asarray(audio), entry["text"], sample_rate, max_chunk_duration)
    codes = encode_segments(encoder, segs, batch_size, sample_rate, max_chunk_duration, bucketed)
    entry["codes"] = {k: v.tolist() for k, v in codes.items()} if as_lists else codes
    return entry
