"""Drop-in ``MimiEncoder`` wrapper (the class copy-pasted into the reference's shard scripts).

Same constructor and methods as ``/root/reference/emilia-mimi/process_shard.py:50-140`` (identical copies
in ``libritts-r-mimi/process_libritts_r.py:33-105``, ``yodas2-mimi/process_shard.py:185-275``,
``librispeech-mimi/process_librispeech_dev-test.py:30-119``, ``mls-en-mimi-pretrain/process_shard.py:60-150``,
...), backed by the HIP engine:

* ``encode_audio_chunk(audio, sr)`` -> int64 ``[K, T]`` (batch dim removed, no trim)            ``:62-86``
* ``encode_audio_batch(list, sr)`` -> ``[]`` for an empty list; delegates to ``encode_audio_chunk`` for a
  single item; otherwise pad-to-longest, ONE encode, trim item i to ``int(ceil(L_i / (sr / 12.5)))``
  frames                                                                                        ``:88-140``

A shard script switches by replacing its ``class MimiEncoder`` with ``from mimi_hip import MimiEncoder``.
"""
from __future__ import annotations

import logging
from typing import List, Optional

import numpy as np
import torch

from .feature_extraction import MimiFeatureExtractor
from .model import MimiHipModel

logger = logging.getLogger(__name__)


class MimiEncoder:
    """Wrapper for Mimi model encoding (HIP engine)."""

    def __init__(self, model_id: str = "kyutai/mimi", device: str = "cuda", model: Optional[MimiHipModel] = None,
                 num_quantizers: Optional[int] = None):
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
        logger.info("Mimi model loaded successfully")

    def encode_audio_chunk(self, audio_array: np.ndarray, sample_rate: int = 24000) -> np.ndarray:
        with torch.no_grad():
            inputs = self.feature_extractor(raw_audio=audio_array, sampling_rate=sample_rate, return_tensors="pt")
            inputs = {k: v.to(self.device) for k, v in inputs.items()}
            encoder_outputs = self.model.encode(inputs["input_values"], inputs["padding_mask"],
                                                num_quantizers=self.num_quantizers)
            audio_codes = encoder_outputs.audio_codes
            return audio_codes.cpu().numpy()[0]

    def encode_audio_batch(self, audio_arrays: List[np.ndarray], sample_rate: int = 24000) -> List[np.ndarray]:
        if len(audio_arrays) == 0:
            return []
        if len(audio_arrays) == 1:
            return [self.encode_audio_chunk(audio_arrays[0], sample_rate)]
        with torch.no_grad():
            original_lengths = [len(audio) for audio in audio_arrays]
            inputs = self.feature_extractor(raw_audio=audio_arrays, sampling_rate=sample_rate, return_tensors="pt",
                                            padding=True)
            inputs = {k: v.to(self.device) for k, v in inputs.items()}
            encoder_outputs = self.model.encode(input_values=inputs["input_values"],
                                                padding_mask=inputs["padding_mask"],
                                                num_quantizers=self.num_quantizers)
            audio_codes = encoder_outputs.audio_codes.cpu()
            frame_rate = sample_rate / 12.5
            results = []
            for i, orig_length in enumerate(original_lengths):
                actual_frames = int(np.ceil(orig_length / frame_rate))
                results.append(audio_codes[i, :, :actual_frames].numpy())
            return results
