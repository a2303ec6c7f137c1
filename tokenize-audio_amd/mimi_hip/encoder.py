"""Drop-in ``MimiEncoder`` wrapper (the class copy-pasted into the reference's shard scripts).

Same constructor and methods as ``/root/reference/emilia-mimi/process_shard.py:50-140`` (identical copies
in ``libritts-r-mimi/process_libritts_r.py:33-105``, ``yodas2-mimi/process_shard.py:185-275``,
``librispeech-mimi/process_librispeech_dev-test.py:30-119``, ``mls-en-mimi-pretrain/process_shard.py:60-150``,
...), backed by the HIP engine:

* ``encode_audio_chunk(audio, sr)`` -> int64 ``[K, T]`` (batch dim removed, no trim)            ``:62-86``
* ``encode_audio_batch(list, sr)`` -> ``[]`` for an empty list; delegates to ``encode_audio_chunk`` for a
  single item; otherwise pad-to-longest, ONE encode, trim item i to ``int(ceil(L_i / (sr / 12.5)))``
  frames                                                                                        ``:88-140``

Added for the per-utterance callers (MLS ``mls-en-mimi-pretrain/process_shard.py:268-307`` and LibriSpeech call
``encode_audio_chunk`` once per utterance): ``encode_audio_chunks(list, sr)`` returns exactly
``[encode_audio_chunk(a, sr) for a in list]`` -- each item encoded alone at its own length, batch 1 -- but runs
``concurrency`` engines (same weights and calibration, so the same codes) on their own streams from as many host
threads, so several batch-1 encodes fill the GPU at once.  A driver keeps its per-utterance loop semantics by
encoding a window of upcoming utterances per call.

The inputs and outputs are the reference's; the data path is leaner.  The reference runs the feature
extractor and moves ``input_values`` and the int64 ``padding_mask`` (8 B per sample) to the device, although
the model ignores the mask (``TF/modeling_mimi.py:1244, :1247``).  Here the items are copied straight into a
zeroed device batch (the same values as the extractor's right padding with 0.0, after its float32 cast), no
mask is built or moved, and the int32 codes come back to the host before the int64 widening.

A shard script switches by replacing its ``class MimiEncoder`` with ``from mimi_hip import MimiEncoder``.
"""
from __future__ import annotations

import logging
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

import numpy as np
import torch

from .feature_extraction import MimiFeatureExtractor
from .model import MimiHipModel

logger = logging.getLogger(__name__)


class MimiEncoder:
    """Wrapper for Mimi model encoding (HIP engine)."""

    def __init__(self, model_id: str = "kyutai/mimi", device: str = "cuda", model: Optional[MimiHipModel] = None,
                 num_quantizers: Optional[int] = None, concurrency: int = 1):
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
        self.concurrency = max(1, int(concurrency))
        self._lanes = None  # [(engine, stream)] built on the first encode_audio_chunks call
        self._lanes_lock = threading.Lock()
        logger.info("Mimi model loaded successfully")

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
        K = self.num_quantizers or self.model.config.num_quantizers
        return self.model.encode_async(x, K).wait().cpu().numpy()

    def encode_audio_chunk(self, audio_array: np.ndarray, sample_rate: int = 24000) -> np.ndarray:
        with torch.no_grad():
            (a,) = self._check([audio_array], sample_rate)
            return self._encode_padded([a])[0].astype(np.int64)

    def encode_audio_batch(self, audio_arrays: List[np.ndarray], sample_rate: int = 24000) -> List[np.ndarray]:
        if len(audio_arrays) == 0:
            return []
        if len(audio_arrays) == 1:
            return [self.encode_audio_chunk(audio_arrays[0], sample_rate)]
        with torch.no_grad():
            items = self._check(audio_arrays, sample_rate)
            codes = self._encode_padded(items)
            samples_per_frame = sample_rate / 12.5
            # item i keeps the frames its own samples produce, int(ceil(L_i / samples_per_frame)), of the padded
            # batch's codes (the reference's trim)
            return [codes[i, :, :int(np.ceil(len(a) / samples_per_frame))].astype(np.int64)
                    for i, a in enumerate(items)]

    def _get_lanes(self):
        with self._lanes_lock:
            if self._lanes is None:
                engines = [self.model] + [self.model.clone() for _ in range(self.concurrency - 1)]
                self._lanes = [(e, torch.cuda.Stream(device=e.device)) for e in engines]
            return self._lanes

    def encode_audio_chunks(self, audio_arrays: List[np.ndarray], sample_rate: int = 24000) -> List[np.ndarray]:
        """``[self.encode_audio_chunk(a, sample_rate) for a in audio_arrays]``, with ``concurrency`` engines
        encoding different items at once (item i on lane i mod concurrency, in order within a lane)."""
        if not hasattr(self.model, "encode_async") or self.concurrency == 1 or len(audio_arrays) <= 1:
            return [self.encode_audio_chunk(a, sample_rate) for a in audio_arrays]
        items = self._check(audio_arrays, sample_rate)
        if any(a.shape[0] == 0 for a in items):
            raise ValueError("empty audio")
        lanes = self._get_lanes()
        K = self.num_quantizers or self.model.config.num_quantizers
        out: List[Optional[np.ndarray]] = [None] * len(items)

        def run(k):  # lane k: its items in order, the next one enqueued before the previous one is waited for
            engine, stream = lanes[k]
            pending = None
            with torch.no_grad(), torch.cuda.stream(stream):
                for i in list(range(k, len(items), len(lanes))) + [None]:
                    ticket = None
                    if i is not None:
                        x = torch.from_numpy(items[i]).to(engine.device, non_blocking=False).reshape(1, -1)
                        ticket = (i, engine.encode_async(x, K))
                    if pending is not None:
                        j, t = pending
                        out[j] = t.wait()[0].cpu().numpy().astype(np.int64)
                    pending = ticket

        n = min(len(lanes), len(items))
        with ThreadPoolExecutor(n) as ex:
            list(ex.map(run, range(n)))
        return out
