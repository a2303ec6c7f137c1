"""``EncodecFeatureExtractor`` behaviour for the kyutai/mimi preprocessor (host side, numpy).

``ENC/feature_extraction_encodec.py:81-202`` with the kyutai/mimi preprocessor config (feature_size 1,
sampling_rate 24000, padding_value 0.0, no chunking, right padding, attention mask returned):
float64 -> float32 cast (``:146-150``), lists -> batch, right-pad to the longest with 0.0 and an int
``padding_mask`` (``:181-190``), ``input_values`` shaped ``[B, 1, L]`` (``:193-196``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import numpy as np
import torch


class MimiFeatureExtractor:
    model_input_names = ["input_values", "padding_mask"]

    def __init__(self, feature_size: int = 1, sampling_rate: int = 24000, padding_value: float = 0.0):
        if feature_size != 1:
            raise ValueError("only mono (feature_size=1) is supported")
        self.feature_size = feature_size
        self.sampling_rate = sampling_rate
        self.padding_value = padding_value

    @classmethod
    def from_pretrained(cls, *_args, **_kw) -> "MimiFeatureExtractor":
        return cls()

    def __call__(self, raw_audio: Union[np.ndarray, Sequence[float], Sequence[np.ndarray]],
                 padding: Optional[Union[bool, str]] = None, truncation: bool = False,
                 max_length: Optional[int] = None, return_tensors: Optional[str] = None,
                 sampling_rate: Optional[int] = None) -> dict:
        if sampling_rate is not None and sampling_rate != self.sampling_rate:
            raise ValueError(
                f"The model corresponding to this feature extractor: {self} was trained using a sampling rate of "
                f"{self.sampling_rate}. Please make sure that the provided audio input was sampled with "
                f"{self.sampling_rate} and not {sampling_rate}.")
        if padding and truncation:
            raise ValueError("Both padding and truncation were set. Make sure you only set one.")
        if padding is None:
            padding = True
        is_batched = bool(isinstance(raw_audio, (list, tuple)) and len(raw_audio) > 0
                          and isinstance(raw_audio[0], (np.ndarray, tuple, list)))
        if is_batched:
            arrays: List[np.ndarray] = [np.asarray(a, dtype=np.float32).T for a in raw_audio]
        else:
            if not isinstance(raw_audio, np.ndarray):
                raw_audio = np.asarray(raw_audio, dtype=np.float32)
            elif raw_audio.dtype == np.float64:
                raw_audio = raw_audio.astype(np.float32)
            arrays = [np.asarray(raw_audio).T]
        for a in arrays:
            if a.ndim != 1:
                raise ValueError(f"Expected mono audio but example has {a.shape[-1]} channels")
        lengths = [a.shape[0] for a in arrays]
        if padding in (True, "longest"):
            target = max(lengths)
        elif padding == "max_length":
            if max_length is None:
                raise ValueError("padding='max_length' needs max_length")
            target = max_length
        else:
            target = None
        if truncation and max_length is not None:
            arrays = [a[:max_length] for a in arrays]
            lengths = [a.shape[0] for a in arrays]
        out = {}
        if target is not None:
            vals = np.full((len(arrays), target), self.padding_value, dtype=np.float32)
            mask = np.zeros((len(arrays), target), dtype=np.int32)
            for i, a in enumerate(arrays):
                vals[i, :a.shape[0]] = a
                mask[i, :a.shape[0]] = 1
            out["padding_mask"] = mask
            out["input_values"] = vals[:, None, :]
        else:
            out["input_values"] = [a[None, :] for a in arrays]
        if return_tensors == "pt":
            out = {k: (torch.from_numpy(np.ascontiguousarray(v)) if isinstance(v, np.ndarray)
                       else [torch.from_numpy(x) for x in v]) for k, v in out.items()}
            if "padding_mask" in out:
                out["padding_mask"] = out["padding_mask"].long()
        elif return_tensors == "np" and "padding_mask" in out:
            out["padding_mask"] = out["padding_mask"].astype(np.int64)
        return out
