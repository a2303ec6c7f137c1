"""ORACLE — test infrastructure only, never shipped, never on the product path.

CPU restatement of the Mimi encode path of ``transformers`` 5.15.0 (third-party; absent from
/root/reference; the reference scripts call it through ``MimiModel.encode``, e.g.
``/root/reference/emilia-mimi/process_shard.py:124-127``).  ``TF/`` below is
``transformers/models/mimi/`` and ``ENC/`` is ``transformers/models/encodec/``.

Written from scratch with torch-CPU functional ops in the reference's op order and layout
(channel-first, fp32), so that on the same CPU it reproduces ``MimiModel.encode`` bit-for-bit (pinned by
``tests/golden/make_golden.py`` against the real ``transformers`` model in the survey container).  On
the GPU box it is the parity checker for small inputs and the ``cpu_baseline`` of ``bench.py``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F


@dataclass
class RefConfig:
    """Encode-path fields of ``MimiConfig`` (``TF/configuration_mimi.py:86-123``)."""
    num_filters: int = 64
    upsampling_ratios: List[int] = field(default_factory=lambda: [8, 6, 5, 4])
    kernel_size: int = 7
    last_kernel_size: int = 3
    residual_kernel_size: int = 3
    compress: int = 2
    hidden_size: int = 512
    num_hidden_layers: int = 8
    num_attention_heads: int = 8
    head_dim: int = 64
    norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    sliding_window: int = 250
    num_quantizers: int = 32
    num_semantic_quantizers: int = 1
    codebook_eps: float = 1e-5  # MimiEuclideanCodebook(epsilon=1e-5), TF/modeling_mimi.py:967


# ---------------------------------------------------------------------------------------------
# convs
# ---------------------------------------------------------------------------------------------
def extra_padding(length: int, kernel: int, stride: int) -> int:
    """``MimiConv1d._get_extra_padding_for_conv1d`` (TF/modeling_mimi.py:269-279), same tensor math."""
    k = torch.tensor(kernel, dtype=torch.int64)
    s = torch.tensor(stride, dtype=torch.int64)
    pt = k - s
    n_frames = (length - k + pt) / s + 1
    n_frames = torch.ceil(n_frames).to(torch.int64) - 1
    ideal = n_frames * s + k - pt
    return int(ideal - length)


def causal_conv1d(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], stride: int = 1,
                  pad_mode: str = "constant") -> torch.Tensor:
    """``MimiConv1d.forward`` causal branch (TF/modeling_mimi.py:327-347): left pad k-s, right pad extra."""
    kernel = w.shape[-1]
    extra = extra_padding(x.shape[-1], kernel, stride)
    x = F.pad(x, (kernel - stride, extra), mode=pad_mode, value=0.0) if pad_mode == "constant" \
        else F.pad(x, (kernel - stride, extra), mode=pad_mode)
    return F.conv1d(x, w, b, stride=stride)


def seanet_encoder(x: torch.Tensor, sd: Dict[str, torch.Tensor], cfg: RefConfig,
                   taps: Optional[dict] = None) -> torch.Tensor:
    """``MimiEncoder.forward`` (TF/modeling_mimi.py:450-492); ``MimiResnetBlock`` :408-447."""
    x = causal_conv1d(x, sd["encoder.layers.0.conv.weight"], sd["encoder.layers.0.conv.bias"])
    if taps is not None:
        taps["conv0"] = x
    idx = 1
    for si, ratio in enumerate(reversed(cfg.upsampling_ratios)):
        # residual block: x + conv1(ELU(conv3(ELU(x))))   (ELU before each conv, identity shortcut)
        p = f"encoder.layers.{idx}.block."
        h = causal_conv1d(F.elu(x), sd[p + "1.conv.weight"], sd[p + "1.conv.bias"])
        h = causal_conv1d(F.elu(h), sd[p + "3.conv.weight"], sd[p + "3.conv.bias"])
        x = x + h
        if taps is not None:
            taps[f"res{si}"] = x
        idx += 2  # resblock, ELU
        p = f"encoder.layers.{idx}.conv."
        x = causal_conv1d(F.elu(x), sd[p + "weight"], sd[p + "bias"], stride=ratio)
        if taps is not None:
            taps[f"down{si}"] = x
        idx += 1
    idx += 1  # ELU
    p = f"encoder.layers.{idx}.conv."
    x = causal_conv1d(F.elu(x), sd[p + "weight"], sd[p + "bias"])
    if taps is not None:
        taps["encoder"] = x
    return x


# ---------------------------------------------------------------------------------------------
# transformer
# ---------------------------------------------------------------------------------------------
def rope_cos_sin(T: int, cfg: RefConfig):
    """``MimiRotaryEmbedding`` (TF/modeling_mimi.py:529-565), default rope, attention_scaling 1."""
    dim = cfg.head_dim
    inv_freq = 1.0 / (cfg.rope_theta ** (torch.arange(0, dim, 2, dtype=torch.int64).to(torch.float) / dim))
    pos = torch.arange(T)[None, :]
    inv_freq_expanded = inv_freq[None, :, None].float().expand(1, -1, 1)
    freqs = (inv_freq_expanded @ pos[:, None, :].float()).transpose(1, 2)
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos(), emb.sin()


def rotate_half(x):
    x1 = x[..., : x.shape[-1] // 2]
    x2 = x[..., x.shape[-1] // 2:]
    return torch.cat((-x2, x1), dim=-1)


def attention(q, k, v, cfg: RefConfig):
    """sdpa with the sliding-window causal mask (``masking_utils.py:76-101``: kv_idx <= q_idx and
    kv_idx > q_idx - sliding_window).  For T <= window the reference skips the mask and passes
    ``is_causal=True`` (``integrations/sdpa_attention.py:120``); we do the same."""
    T = q.shape[-2]
    scale = 1.0 / math.sqrt(cfg.head_dim)
    if T <= cfg.sliding_window:
        return F.scaled_dot_product_attention(q, k, v, attn_mask=None, dropout_p=0.0, scale=scale,
                                              is_causal=True)
    i = torch.arange(T)[:, None]
    j = torch.arange(T)[None, :]
    mask = (j <= i) & (j > i - cfg.sliding_window)
    return F.scaled_dot_product_attention(q, k, v, attn_mask=mask[None, None], dropout_p=0.0, scale=scale,
                                          is_causal=False)


def transformer(x: torch.Tensor, sd: Dict[str, torch.Tensor], cfg: RefConfig,
                taps: Optional[dict] = None) -> torch.Tensor:
    """``MimiTransformerModel.forward`` (:801-928) with ``MimiTransformerLayer`` (:742-779).  x: [B,T,C]."""
    B, T, C = x.shape
    H, D = cfg.num_attention_heads, cfg.head_dim
    cos, sin = rope_cos_sin(T, cfg)
    cos, sin = cos[:, None], sin[:, None]  # unsqueeze_dim=1 -> [1,1,T,D]
    for l in range(cfg.num_hidden_layers):
        p = f"encoder_transformer.layers.{l}."
        res = x
        h = F.layer_norm(x, (C,), sd[p + "input_layernorm.weight"], sd[p + "input_layernorm.bias"], cfg.norm_eps)
        q = F.linear(h, sd[p + "self_attn.q_proj.weight"]).view(B, T, H, D).transpose(1, 2)
        k = F.linear(h, sd[p + "self_attn.k_proj.weight"]).view(B, T, H, D).transpose(1, 2)
        v = F.linear(h, sd[p + "self_attn.v_proj.weight"]).view(B, T, H, D).transpose(1, 2)
        q = (q * cos) + (rotate_half(q) * sin)
        k = (k * cos) + (rotate_half(k) * sin)
        a = attention(q, k, v, cfg).transpose(1, 2).contiguous().reshape(B, T, C)
        a = F.linear(a, sd[p + "self_attn.o_proj.weight"])
        x = res + sd[p + "self_attn_layer_scale.scale"] * a
        res = x
        h = F.layer_norm(x, (C,), sd[p + "post_attention_layernorm.weight"],
                         sd[p + "post_attention_layernorm.bias"], cfg.norm_eps)
        h = F.linear(F.gelu(F.linear(h, sd[p + "mlp.fc1.weight"])), sd[p + "mlp.fc2.weight"])
        x = res + sd[p + "mlp_layer_scale.scale"] * h
        if taps is not None:
            taps[f"xfmr{l}"] = x
    return x


# ---------------------------------------------------------------------------------------------
# quantizer
# ---------------------------------------------------------------------------------------------
def codebook_embed(sd, prefix: str, cfg: RefConfig) -> torch.Tensor:
    """``MimiEuclideanCodebook.embed`` (:979-983)."""
    return sd[prefix + "embed_sum"] / sd[prefix + "cluster_usage"].clamp(min=cfg.codebook_eps)[:, None]


def euclid_argmin(r: torch.Tensor, embed: torch.Tensor) -> torch.Tensor:
    """``quantize`` (:985-990): cdist(p=2) -> argmin (first index on ties)."""
    d = torch.cdist(r[None].float(), embed[None].float(), p=2)[0]
    return d.argmin(dim=-1)


def rvq_encode(emb: torch.Tensor, sd, which: str, nq: int, cfg: RefConfig) -> torch.Tensor:
    """``MimiResidualVectorQuantizer.encode`` (:1050-1068).  emb [B,C,T] -> codes [nq,B,T]."""
    pre = f"quantizer.{which}_residual_vector_quantizer."
    x = F.conv1d(emb, sd[pre + "input_proj.weight"])
    B, D, T = x.shape
    residual = x
    out = []
    for l in range(nq):
        embed = codebook_embed(sd, pre + f"layers.{l}.codebook.", cfg)
        flat = residual.permute(0, 2, 1).reshape(-1, D)
        idx = euclid_argmin(flat, embed).view(B, T)
        q = F.embedding(idx, embed).permute(0, 2, 1)
        residual = residual - q
        out.append(idx)
    return torch.stack(out)


def split_rvq_encode(emb, sd, K: int, cfg: RefConfig) -> torch.Tensor:
    """``MimiSplitResidualVectorQuantizer.encode`` (:1099-1126): semantic then acoustic on the SAME emb."""
    codes = rvq_encode(emb, sd, "semantic", cfg.num_semantic_quantizers, cfg)
    if K > cfg.num_semantic_quantizers:
        ac = rvq_encode(emb, sd, "acoustic", K - cfg.num_semantic_quantizers, cfg)
        codes = torch.cat([codes, ac], dim=0)
    return codes


# ---------------------------------------------------------------------------------------------
# model
# ---------------------------------------------------------------------------------------------
def pre_quantizer(x: torch.Tensor, sd, cfg: RefConfig, taps: Optional[dict] = None) -> torch.Tensor:
    """``_encode_frame`` up to the quantizer (:1245-1259).  x [B,1,L] -> [B,512,T]."""
    e = seanet_encoder(x, sd, cfg, taps)
    e = transformer(e.transpose(1, 2), sd, cfg, taps).transpose(1, 2)
    e = causal_conv1d(e, sd["downsample.conv.weight"], None, stride=2, pad_mode="replicate")
    if taps is not None:
        taps["downsample"] = e
    return e


def encode(input_values, sd, num_quantizers: Optional[int] = None, cfg: Optional[RefConfig] = None,
           taps: Optional[dict] = None) -> torch.Tensor:
    """``MimiModel.encode`` (:1297-1386) -> int64 codes [B, K, T].  The padding mask is ignored there
    (:1244, :1247), so it is not an argument here."""
    cfg = cfg or RefConfig()
    K = cfg.num_quantizers if num_quantizers is None else int(num_quantizers)
    if K > cfg.num_quantizers:
        raise ValueError("num_quantizers > config.num_quantizers")
    x = torch.as_tensor(np.asarray(input_values) if not torch.is_tensor(input_values) else input_values)
    if x.dim() == 1:
        x = x[None, None]
    x = x.float()
    sdt = {k: (v if torch.is_tensor(v) else torch.from_numpy(np.asarray(v))) for k, v in sd.items()}
    with torch.no_grad():
        e = pre_quantizer(x, sdt, cfg, taps)
        if taps is not None:
            taps["pre_quantizer"] = e
        codes = split_rvq_encode(e, sdt, K, cfg)
    return codes.transpose(0, 1)


def rvq_from_embedding(emb, sd, K: int, cfg: Optional[RefConfig] = None, return_margins: bool = False,
                       return_second: bool = False):
    """Quantizer alone on a given pre-quantizer embedding [B,512,T] -> codes [B,K,T] (+ per-code relative
    margin (d2 - d1) / d2 between the best and second-best distance, for the near-tie audit; + d2 itself with
    return_second, for the perturbation-derived audit threshold of tests/audit.py)."""
    cfg = cfg or RefConfig()
    sdt = {k: (v if torch.is_tensor(v) else torch.from_numpy(np.asarray(v))) for k, v in sd.items()}
    emb = emb if torch.is_tensor(emb) else torch.from_numpy(np.asarray(emb))
    with torch.no_grad():
        codes = split_rvq_encode(emb.float(), sdt, K, cfg).transpose(0, 1)
        if not return_margins:
            return codes
        margins, seconds = [], []
        for which, levels in (("semantic", range(cfg.num_semantic_quantizers)),
                              ("acoustic", range(K - cfg.num_semantic_quantizers))):
            pre = f"quantizer.{which}_residual_vector_quantizer."
            x = F.conv1d(emb.float(), sdt[pre + "input_proj.weight"])
            B, D, T = x.shape
            r = x
            for l in levels:
                embed = codebook_embed(sdt, pre + f"layers.{l}.codebook.", cfg)
                flat = r.permute(0, 2, 1).reshape(-1, D)
                d = torch.cdist(flat[None], embed[None], p=2)[0]
                top2 = torch.topk(d, 2, dim=-1, largest=False).values
                margins.append(((top2[:, 1] - top2[:, 0]) / top2[:, 1].clamp_min(1e-30)).view(B, T))
                seconds.append(top2[:, 1].view(B, T))
                idx = d.argmin(dim=-1).view(B, T)
                r = r - F.embedding(idx, embed).permute(0, 2, 1)
        if return_second:
            return codes, torch.stack(margins, dim=1), torch.stack(seconds, dim=1)
        return codes, torch.stack(margins, dim=1)
