"""Mimi configuration (the fields the encode path reads) and the conv length arithmetic.

Defaults are those of ``transformers`` 5.15.0 ``MimiConfig`` (``TF/configuration_mimi.py:86-123``), which
equal the ``kyutai/mimi`` checkpoint's config for every encode-path field.  ``from_json`` reads a
checkpoint directory's ``config.json`` (HF layout) so a local ``kyutai/mimi`` snapshot drops in.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from typing import List, Optional

import numpy as np


@dataclasses.dataclass
class MimiConfig:
    sampling_rate: int = 24_000
    audio_channels: int = 1
    hidden_size: int = 512
    num_filters: int = 64
    num_residual_layers: int = 1
    upsampling_ratios: Optional[List[int]] = None
    kernel_size: int = 7
    last_kernel_size: int = 3
    residual_kernel_size: int = 3
    dilation_growth_rate: int = 2
    use_causal_conv: bool = True
    pad_mode: str = "constant"
    compress: int = 2
    codebook_size: int = 2048
    codebook_dim: int = 256
    num_quantizers: int = 32
    use_conv_shortcut: bool = False
    vector_quantization_hidden_dimension: int = 256
    num_semantic_quantizers: int = 1
    num_hidden_layers: int = 8
    intermediate_size: int = 2048
    num_attention_heads: int = 8
    num_key_value_heads: int = 8
    head_dim: Optional[int] = None
    hidden_act: str = "gelu"
    max_position_embeddings: int = 8000
    norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    sliding_window: int = 250
    layer_scale_initial_scale: float = 0.01
    attention_bias: bool = False
    frame_rate_override: Optional[float] = None

    def __post_init__(self):
        if not self.upsampling_ratios:
            self.upsampling_ratios = [8, 6, 5, 4]
        self.head_dim = self.head_dim or self.hidden_size // self.num_attention_heads

    # TF/configuration_mimi.py:143-145
    @property
    def encodec_frame_rate(self) -> int:
        return math.ceil(self.sampling_rate / math.prod(self.upsampling_ratios))

    # TF/configuration_mimi.py:152-175
    @property
    def frame_size(self) -> int:
        strides = [1]
        for ratio in reversed(self.upsampling_ratios):
            for _ in range(self.num_residual_layers):
                strides.extend([1, 1])
                if self.use_conv_shortcut:
                    strides.append(1)
            strides.append(ratio)
        strides.append(1)
        strides.append(2)
        return math.prod(strides)

    @property
    def frame_rate(self) -> float:
        if self.frame_rate_override is not None:
            return self.frame_rate_override
        return self.sampling_rate / self.frame_size

    def validate_supported(self) -> None:
        """The HIP engine implements the architecture family of the kyutai/mimi checkpoint."""
        problems = []
        if self.audio_channels != 1:
            problems.append("audio_channels must be 1 (mono)")
        if not self.use_causal_conv:
            problems.append("use_causal_conv must be True")
        if self.pad_mode != "constant":
            problems.append("pad_mode must be 'constant'")
        if self.use_conv_shortcut:
            problems.append("use_conv_shortcut must be False")
        if self.num_residual_layers != 1:
            problems.append("num_residual_layers must be 1")
        if self.hidden_act != "gelu":
            problems.append("hidden_act must be 'gelu'")
        if self.attention_bias:
            problems.append("attention_bias must be False")
        if self.num_key_value_heads != self.num_attention_heads:
            problems.append("GQA (num_key_value_heads != num_attention_heads) is not supported")
        if self.head_dim * self.num_attention_heads != self.hidden_size:
            problems.append("head_dim * num_attention_heads must equal hidden_size")
        if problems:
            raise ValueError("unsupported Mimi config: " + "; ".join(problems))

    @classmethod
    def from_json(cls, path: str) -> "MimiConfig":
        if os.path.isdir(path):
            path = os.path.join(path, "config.json")
        with open(path) as f:
            raw = json.load(f)
        fields = {f.name for f in dataclasses.fields(cls)}
        kw = {k: v for k, v in raw.items() if k in fields}
        rope = raw.get("rope_parameters") or {}
        if "rope_theta" in raw:
            kw["rope_theta"] = raw["rope_theta"]
        elif isinstance(rope, dict) and "rope_theta" in rope:
            kw["rope_theta"] = rope["rope_theta"]
        if raw.get("frame_rate") is not None:
            kw["frame_rate_override"] = raw["frame_rate"]
        return cls(**kw)


def conv_out_len(length: int, kernel: int, stride: int) -> int:
    """Output length of a causal ``MimiConv1d`` (``TF/modeling_mimi.py:269-279, 327-347``).

    Replicates the reference's float32 arithmetic exactly: ``(L - k + (k - s)) / s + 1`` is a true
    division of int64 tensors (-> float32), then ``ceil``; the padded input is ``n_frames*s + k`` long,
    giving ``n_frames + 1`` outputs.
    """
    if 0 <= length < (1 << 22):
        # (L - s) / s + 1 = L / s, and below 2^22 samples no float32 rounding moves its ceil (every quotient's
        # fractional part, a multiple of 1 / s, is further from an integer than half an ulp): ceil(L / s) exactly,
        # without numpy scalars (~70 us per encoded_length on the per-utterance path)
        return -(-length // stride)
    pt = kernel - stride
    nf = np.float32(np.float32(length - kernel + pt) / np.float32(stride)) + np.float32(1.0)
    n_frames = int(np.ceil(np.float32(nf))) - 1
    return n_frames + 1


def conv_extra_padding(length: int, kernel: int, stride: int) -> int:
    pt = kernel - stride
    n_frames = conv_out_len(length, kernel, stride) - 1
    ideal = n_frames * stride + kernel - pt
    return ideal - length


def encoded_length(length: int, cfg: Optional[MimiConfig] = None) -> int:
    """Frames produced for ``length`` samples (``MimiModel.get_encoded_length``, ``:1265-1278``)."""
    cfg = cfg or MimiConfig()
    t = conv_out_len(length, cfg.kernel_size, 1)
    for ratio in reversed(cfg.upsampling_ratios):
        t = conv_out_len(t, cfg.residual_kernel_size, 1)
        t = conv_out_len(t, 1, 1)
        t = conv_out_len(t, 2 * ratio, ratio)
    t = conv_out_len(t, cfg.last_kernel_size, 1)
    t = conv_out_len(t, 2 * int(cfg.encodec_frame_rate / cfg.frame_rate), 2)
    return t
