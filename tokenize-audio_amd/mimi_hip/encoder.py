"""Drop-in ``MimiEncoder`` wrapper (the class copy-pasted into the reference's shard scripts).

Same constructor and methods as ``/root/reference/emilia-mimi/process_shard.py:50-140`` (identical copies
in ``libritts-r-mimi/process_libritts_r.py:33-105``, ``yodas2-mimi/process_shard.py:185-275``,
``librispeech-mimi/process_librispeech_dev-test.py:30-119``, ``mls-en-mimi-pretrain/process_shard.py:60-150``,
...), backed by the HIP engine:

* ``encode_audio_chunk(audio, sr)`` -> int64 ``[K, T]`` (batch dim removed, no trim)            ``:62-86``
* ``encode_audio_batch(list, sr)`` -> ``[]`` for an empty list; delegates to ``encode_audio_chunk`` for a
  single item; otherwise pad-to-longest, ONE encode, trim item i to ``int(ceil(L_i / (sr / 12.5)))``
  frames                                                                                        ``:88-140``

How a padded batch is encoded: item i keeps frames [0, ceil(L_i / 1920)), and every one of them depends only on
the item's samples below E_i = min(Lmax, 1920 ceil(L_i / 1920)) (every conv is causal, and a length that is a
multiple of 1920 needs no extra padding at any stage), which are its own samples followed by the batch's zero
padding.  So the batch runs as ONE ragged encode (``mimi_encode_ragged``) with item i at length E_i: the codes the
caller keeps are the padded batch's, and the compute the padding would cost is skipped (U[1.5, 20] s YODAS2
batches: about 45 % of a pad-to-longest encode).  ``ragged=False`` runs the literal padded encode instead.
Ragged mode equals the literal padded encode up to near-ties only: an item of 256 or fewer 25 Hz frames can run
different kernels (the T <= 256 attention instead of the banded one) than the same item inside a longer padded
batch, so a code whose top-2 distances differ by a rounding error may flip.  Against the reference wrapper's own
output this path is held to the derived near-tie audit (``tests/test_gpu_parity.py``
``test_padded_batch_b32_vs_reference_wrapper[ragged]``: 0.999993 exact, the one flip at margin 1e-7).
An empty item among non-empty ones comes back as a ``(K, 0)`` array, as in the reference's padded batch.

Threads: every thread that calls ``encode_audio_batch`` / ``encode_batches`` / ``encode_audio_chunks`` gets its own
staging pipeline (pinned, input and output buffers and streams), so concurrent callers sharing one ``MimiEncoder``
-- the YODAS2 ``ThreadPoolExecutor`` (``yodas2-mimi/process_shard.py:691-717``) -- never share a buffer.

Added for the per-utterance callers (MLS ``mls-en-mimi-pretrain/process_shard.py:268-307`` and LibriSpeech call
``encode_audio_chunk`` once per utterance): ``encode_audio_chunks(list, sr)`` returns exactly
``[encode_audio_chunk(a, sr) for a in list]`` -- each item encoded alone at its own length, bit for bit -- as
ragged batches of several utterances at once.

And for shard drivers that can hand over their batches ahead of time (the YODAS2 sub-shard loop,
``yodas2-mimi/process_shard.py:494-525``): ``encode_batches(batches, sr)`` yields ``encode_audio_batch(b, sr)`` for
each batch in order, pipelined -- the next batch's host copy into pinned memory and its host->device copy (on a
copy stream) run while the GPU encodes the current one, and results come back as soon as they are final.

A shard script switches by replacing its ``class MimiEncoder`` with ``from mimi_hip import MimiEncoder``.
"""
from __future__ import annotations

import logging
import math
import threading
from typing import Iterable, Iterator, List, Optional, Sequence

import numpy as np
import torch

from .config import encoded_length
from .feature_extraction import MimiFeatureExtractor
from .model import MimiHipModel

logger = logging.getLogger(__name__)

FRAME = 1920  # samples per 12.5 Hz frame at 24 kHz (MimiConfig.frame_size)


def padded_batch_lengths(lengths: Sequence[int]) -> List[int]:
    """Per-item encode lengths that reproduce a pad-to-longest batch's kept frames (module docstring)."""
    lmax = max(lengths)
    return [min(lmax, FRAME * math.ceil(n / FRAME)) for n in lengths]


class _Pipeline:
    """Double-buffered ragged encodes: pinned host staging -> device on a copy stream -> encode on a compute stream.
    Slot k's buffers are reused by the (k + depth)-th submit, after the result of the k-th was collected (its
    encode finished reading them).  With several engines (MimiEncoder concurrency > 1) slot k encodes on engine
    k % n, each engine on its own compute stream with its own workspace, so consecutive batches run on the GPU
    at the same time; every engine has the same weights and activation scales, so the codes are the same."""

    def __init__(self, models, K: int, depth: int = 2):
        models = list(models) if isinstance(models, (list, tuple)) else [models]
        self.models, self.model, self.K = models, models[0], K
        self.depth = max(depth, len(models))
        self.dev = self.model.device
        self.copy = torch.cuda.Stream(device=self.dev)
        self.comps = [torch.cuda.Stream(device=self.dev) for _ in models]
        self.comp = self.comps[0]
        self.slots = [dict(pin=None, din=None, out=None) for _ in range(self.depth)]
        self.n = 0

    def _buf(self, slot, key, numel, dtype, pinned):
        b = slot[key]
        if b is None or b.numel() < numel:
            b = (torch.empty(numel, dtype=dtype, pin_memory=True) if pinned
                 else torch.empty(numel, dtype=dtype, device=self.dev))
            slot[key] = b
        return b

    def submit(self, arrays: List[np.ndarray], enc_lens: List[int], keep: List[int]):
        B, L = len(arrays), max(enc_lens)
        k = self.n % self.depth
        slot = self.slots[k]
        model, comp = self.models[k % len(self.models)], self.comps[k % len(self.models)]
        self.n += 1
        pin = self._buf(slot, "pin", B * L, torch.float32, True)[:B * L].view(B, L)
        pn = pin.numpy()
        for i, a in enumerate(arrays):  # the item's samples, then zeros up to its encode length (never past it)
            n = a.shape[0]
            pn[i, :n] = a
            if enc_lens[i] > n:
                pn[i, n:enc_lens[i]] = 0.0
        din = self._buf(slot, "din", B * L, torch.float32, False)[:B * L].view(B, L)
        T = encoded_length(L, self.model.config)
        out = self._buf(slot, "out", B * self.K * T, torch.int32, False)[:B * self.K * T].view(B, self.K, T)
        with torch.cuda.stream(self.copy):
            din.copy_(pin, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy)
        comp.wait_event(ev)
        with torch.cuda.stream(comp):
            ticket = model.encode_ragged_async(din, enc_lens, self.K, out=out)
        return ticket, keep

    @staticmethod
    def collect(handle) -> List[np.ndarray]:
        ticket, keep = handle
        codes = ticket.wait().cpu().numpy()  # final once waited (the f16x3 overflow check runs there)
        return [codes[i, :, :t].astype(np.int64) for i, t in enumerate(keep)]


class MimiEncoder:
    """Wrapper for Mimi model encoding (HIP engine)."""

    def __init__(self, model_id: str = "kyutai/mimi", device: str = "cuda", model: Optional[MimiHipModel] = None,
                 num_quantizers: Optional[int] = None, concurrency: int = 1, ragged: bool = True,
                 chunk_batch: int = 32):
        logger.info(f"Loading Mimi model: {model_id}")
        self.device = device
        self.feature_extractor = MimiFeatureExtractor.from_pretrained(model_id)
        self.model = model if model is not None else MimiHipModel.from_pretrained(model_id, device=device)
        self.model = self.model.to(device)
        self.model.eval()
        # The reference always encodes all 32 codebooks and the caller slices [:8]; the codes of the
        # first K levels do not depend on the later ones (split RVQ, TF/modeling_mimi.py:1060-1066), so a
        # caller that only keeps K may set num_quantizers=K for the same result with less work.
        self.num_quantizers = num_quantizers
        # concurrency: engines the pipelined paths (encode_batches, encode_audio_chunks) alternate between, each with
        # its own workspace and compute stream, so consecutive batches overlap on the GPU (clones share the weights'
        # values and the activation scales: the same codes)
        self.concurrency = max(1, int(concurrency))
        self._engines = [self.model]
        self._engines_lock = threading.Lock()
        self.ragged = bool(ragged) and hasattr(self.model, "encode_ragged_async")
        self.chunk_batch = max(1, int(chunk_batch))
        self._local = threading.local()  # per-thread _Pipeline (its buffers are never shared between callers)
        logger.info("Mimi model loaded successfully")

    @property
    def _K(self) -> int:
        return self.num_quantizers or self.model.config.num_quantizers

    def _check(self, arrays, sample_rate):
        # the feature extractor's checks and float32 cast (ENC/feature_extraction_encodec.py:130-150)
        if sample_rate is not None and sample_rate != self.feature_extractor.sampling_rate:
            raise ValueError(
                f"The model corresponding to this feature extractor: {self.feature_extractor} was trained using a "
                f"sampling rate of {self.feature_extractor.sampling_rate}. Please make sure that the provided audio "
                f"input was sampled with {self.feature_extractor.sampling_rate} and not {sample_rate}.")
        out = []
        for a in arrays:
            a = np.asarray(a, dtype=np.float32)
            if a.ndim != 1:
                raise ValueError(f"Expected mono audio but example has {a.shape[-1]} channels")
            out.append(a)
        return out

    def _encode_padded(self, arrays: List[np.ndarray]) -> np.ndarray:
        """Right-pad with 0.0 to the longest on the device, one encode -> int32 [B, K, T] on the host."""
        if not hasattr(self.model, "encode_async"):  # any other MimiModel.encode-compatible model: reference path
            inputs = self.feature_extractor(raw_audio=arrays if len(arrays) > 1 else arrays[0],
                                            sampling_rate=self.feature_extractor.sampling_rate, return_tensors="pt",
                                            padding=True)
            inputs = {k: v.to(self.device) for k, v in inputs.items()}
            return self.model.encode(inputs["input_values"], inputs["padding_mask"],
                                     num_quantizers=self.num_quantizers).audio_codes.cpu().numpy()
        dev = self.model.device
        lmax = max(a.shape[0] for a in arrays)
        if lmax == 0:
            raise ValueError("empty audio")
        x = torch.zeros((len(arrays), lmax), dtype=torch.float32, device=dev)
        for i, a in enumerate(arrays):
            if a.shape[0]:
                x[i, :a.shape[0]].copy_(torch.from_numpy(a))
        return self.model.encode_async(x, self._K).wait().cpu().numpy()

    def _engine_list(self):
        n = self.concurrency if hasattr(self.model, "clone") else 1
        with self._engines_lock:
            while len(self._engines) < n:
                m = self.model.clone()
                if hasattr(m, "calibrate"):
                    m.calibrate()  # (now, not inside the clone's first encode)
                self._engines.append(m)
            return self._engines[:n]

    def _pipeline(self) -> _Pipeline:
        pipe = getattr(self._local, "pipe", None)
        if pipe is None or pipe.K != self._K:
            pipe = self._local.pipe = _Pipeline(self._engine_list(), self._K)
        return pipe

    def encode_audio_chunk(self, audio_array: np.ndarray, sample_rate: int = 24000) -> np.ndarray:
        with torch.no_grad():
            (a,) = self._check([audio_array], sample_rate)
            if a.shape[0] and hasattr(self.model, "encode_host"):
                # one utterance needs no padding: host samples in, host codes out in one engine call
                return self.model.encode_host(a[None], self._K)[0].astype(np.int64)
            return self._encode_padded([a])[0].astype(np.int64)

    def _batch_plan(self, items: List[np.ndarray], sample_rate: int):
        if all(a.shape[0] == 0 for a in items):
            raise ValueError("empty audio")
        samples_per_frame = sample_rate / 12.5
        # item i keeps the frames its own samples produce, int(ceil(L_i / samples_per_frame)), of the padded
        # batch's codes (the reference's trim)
        keep = [int(np.ceil(len(a) / samples_per_frame)) for a in items]
        # an empty item keeps 0 frames (the reference pads it and trims to (K, 0)); it is encoded as one zero
        # sample so the ragged encode has no zero-length item
        enc = [max(1, n) for n in padded_batch_lengths([len(a) for a in items])]
        return enc, keep

    def encode_audio_batch(self, audio_arrays: List[np.ndarray], sample_rate: int = 24000) -> List[np.ndarray]:
        if len(audio_arrays) == 0:
            return []
        if len(audio_arrays) == 1:
            return [self.encode_audio_chunk(audio_arrays[0], sample_rate)]
        with torch.no_grad():
            items = self._check(audio_arrays, sample_rate)
            if self.ragged:
                enc_lens, keep = self._batch_plan(items, sample_rate)
                pipe = self._pipeline()
                return pipe.collect(pipe.submit(items, enc_lens, keep))
            codes = self._encode_padded(items)
            samples_per_frame = sample_rate / 12.5
            return [codes[i, :, :int(np.ceil(len(a) / samples_per_frame))].astype(np.int64)
                    for i, a in enumerate(items)]

    def encode_batches(self, batches: Iterable[Sequence[np.ndarray]], sample_rate: int = 24000
                       ) -> Iterator[List[np.ndarray]]:
        """Yields ``encode_audio_batch(batch, sample_rate)`` for each batch, in order (the same codes), with the next
        batch's host staging and host->device copy overlapping the current batch's encode."""
        if not self.ragged:
            for b in batches:
                yield self.encode_audio_batch(list(b), sample_rate)
            return
        pipe = self._pipeline()
        pending = None  # (handle, or the finished result of a 0/1-item batch)
        with torch.no_grad():
            for b in batches:
                b = list(b)
                if len(b) <= 1:
                    cur = ("done", [self.encode_audio_chunk(b[0], sample_rate)] if b else [])
                else:
                    items = self._check(b, sample_rate)
                    enc_lens, keep = self._batch_plan(items, sample_rate)
                    cur = ("run", pipe.submit(items, enc_lens, keep))
                if pending is not None:
                    yield pending[1] if pending[0] == "done" else pipe.collect(pending[1])
                pending = cur
            if pending is not None:
                yield pending[1] if pending[0] == "done" else pipe.collect(pending[1])

    def encode_audio_chunks(self, audio_arrays: List[np.ndarray], sample_rate: int = 24000) -> List[np.ndarray]:
        """``[self.encode_audio_chunk(a, sample_rate) for a in audio_arrays]``, bit for bit: each utterance encoded
        alone at its own length, as ragged batches of up to ``chunk_batch`` utterances (grouped by length),
        pipelined."""
        if not self.ragged or len(audio_arrays) <= 1:
            return [self.encode_audio_chunk(a, sample_rate) for a in audio_arrays]
        items = self._check(audio_arrays, sample_rate)
        if any(a.shape[0] == 0 for a in items):
            raise ValueError("empty audio")
        order = sorted(range(len(items)), key=lambda i: items[i].shape[0])
        groups = [order[i:i + self.chunk_batch] for i in range(0, len(order), self.chunk_batch)]
        out: List[Optional[np.ndarray]] = [None] * len(items)
        pipe = self._pipeline()
        pending = None
        with torch.no_grad():
            for g in groups + [None]:
                cur = None
                if g is not None:
                    lens = [items[i].shape[0] for i in g]
                    cur = (g, pipe.submit([items[i] for i in g], lens,
                                          [encoded_length(n, self.model.config) for n in lens]))
                if pending is not None:
                    for i, c in zip(pending[0], pipe.collect(pending[1])):
                        out[i] = c
                pending = cur
        return out
