"""Deterministic synthetic Mimi checkpoints and speech-like audio.

The real ``kyutai/mimi`` checkpoint and the LibriSpeech / Emilia / YODAS2 audio the reference scripts
encode are not available offline, so tests and the bench use a seeded stand-in of the same shapes.

Everything here is *bit-reproducible across machines*: values come from a counter-based splitmix64
stream in numpy uint64 arithmetic, and the only float operations are exact int->float conversions and
separate element-wise IEEE ops (one rounding each, no BLAS, no transcendental functions), so the GPU
box regenerates exactly the bytes that the golden fixtures were made from in the survey container.
``state_dict_sha256`` lets a test prove that.

Parameter names and shapes are the HF ``MimiModel`` encode-path names (SURVEY.md §2.2;
``TF/modeling_mimi.py:450-492`` encoder, ``:729-779`` transformer, ``:1196-1206`` downsample,
``:964-1126`` quantizer).

Codebooks are *data-initialised* (SURVEY.md §7 step 1): each level's codebook is a Gaussian-like
cloud fitted to that level's real residual distribution (mean + top principal directions + diagonal
remainder), whose statistics were measured once with the oracle and are committed, small, in
``data/codebook_stats.npz``.  Without them every residual maps to a handful of codes.
"""
from __future__ import annotations

import hashlib
import os
from typing import Dict, Iterable, List, Optional

import numpy as np

from .config import MimiConfig

_U64 = np.uint64
_STATS_PATH = os.path.join(os.path.dirname(__file__), "data", "codebook_stats.npz")


# --------------------------------------------------------------------------------------------
# counter-based PRNG
# --------------------------------------------------------------------------------------------
def _key(*parts) -> int:
    h = hashlib.sha256("/".join(str(p) for p in parts).encode()).digest()
    return int.from_bytes(h[:8], "little")


def splitmix64(counter: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser over a uint64 counter array (wrapping arithmetic)."""
    z = counter.astype(_U64) + _U64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> _U64(30))) * _U64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> _U64(27))) * _U64(0x94D049BB133111EB)
    return z ^ (z >> _U64(31))


def random_bits(n: int, *key_parts) -> np.ndarray:
    k = _U64(_key(*key_parts))
    return splitmix64(np.arange(n, dtype=_U64) ^ k)


def uniform_pm1(n: int, *key_parts) -> np.ndarray:
    """n float32 values uniform on [-1, 1) with 24-bit resolution (exact in float32)."""
    b = random_bits(n, *key_parts)
    i = (b >> _U64(40)).astype(np.int64) - (1 << 23)
    return i.astype(np.float32) * np.float32(2.0 ** -23)


def uniform01_f64(n: int, *key_parts) -> np.ndarray:
    b = random_bits(n, *key_parts)
    return (b >> _U64(11)).astype(np.float64) * (2.0 ** -53)


def gaussianish(n: int, *key_parts) -> np.ndarray:
    """Irwin-Hall(4) approximation of N(0,1) in float32: sum of 4 uniforms, rescaled (all exact ops)."""
    u = np.zeros(n, dtype=np.float32)
    for j in range(4):
        u = u + uniform_pm1(n, *key_parts, "ih", j)
    # var(U[-1,1)) = 1/3 -> var(sum of 4) = 4/3 -> scale by sqrt(3/4)
    return u * np.float32(np.sqrt(0.75))


# --------------------------------------------------------------------------------------------
# weights
# --------------------------------------------------------------------------------------------
def _uniform_std(shape, std: float, *key_parts) -> np.ndarray:
    n = int(np.prod(shape))
    return (uniform_pm1(n, *key_parts) * np.float32(std * np.sqrt(3.0))).reshape(shape)


def encoder_conv_specs(cfg: MimiConfig) -> List[dict]:
    """The SEANet encoder convs in layer order, with their HF parameter prefixes
    (``TF/modeling_mimi.py:455-476``)."""
    specs = []
    idx = 0
    specs.append(dict(name=f"encoder.layers.{idx}.conv", cin=cfg.audio_channels, cout=cfg.num_filters,
                      k=cfg.kernel_size, stride=1, kind="first"))
    idx += 1
    scale = 1
    for ratio in reversed(cfg.upsampling_ratios):
        c = scale * cfg.num_filters
        for j in range(cfg.num_residual_layers):
            d = cfg.dilation_growth_rate ** j
            hidden = c // cfg.compress
            specs.append(dict(name=f"encoder.layers.{idx}.block.1.conv", cin=c, cout=hidden,
                              k=cfg.residual_kernel_size, stride=1, dilation=d, kind="res3"))
            specs.append(dict(name=f"encoder.layers.{idx}.block.3.conv", cin=hidden, cout=c,
                              k=1, stride=1, kind="res1"))
            idx += 1
        idx += 1  # ELU
        specs.append(dict(name=f"encoder.layers.{idx}.conv", cin=c, cout=2 * c, k=2 * ratio,
                          stride=ratio, kind="down"))
        idx += 1
        scale *= 2
    idx += 1  # ELU
    specs.append(dict(name=f"encoder.layers.{idx}.conv", cin=scale * cfg.num_filters, cout=cfg.hidden_size,
                      k=cfg.last_kernel_size, stride=1, kind="final"))
    return specs


def _load_codebook_stats():
    if not os.path.exists(_STATS_PATH):
        return None
    with np.load(_STATS_PATH, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def make_codebook(level: int, cfg: MimiConfig, seed: int, stats: Optional[dict]) -> np.ndarray:
    """Codebook ``level`` (0 = semantic, 1.. = acoustic) as float32 [codebook_size, codebook_dim]."""
    n, d = cfg.codebook_size, cfg.codebook_dim
    tag = ("cb", seed, level)
    if stats is None or level >= stats["mean"].shape[0]:
        # fallback: isotropic cloud at a level-dependent scale
        return gaussianish(n * d, *tag, "iso").reshape(n, d) * np.float32(0.5 ** level)
    mean = stats["mean"][level].astype(np.float32)          # [d]
    comps = stats["comps"][level].astype(np.float32)        # [r, d], rows scaled by their std
    diag = stats["diag"][level].astype(np.float32)          # [d] std of the remainder
    r = comps.shape[0]
    z = gaussianish(n * r, *tag, "z").reshape(n, r)
    e = np.broadcast_to(mean, (n, d)).copy()
    for j in range(r):  # fixed order, element-wise IEEE ops only (no BLAS)
        e = e + z[:, j:j + 1] * comps[j][None, :]
    e = e + gaussianish(n * d, *tag, "diag").reshape(n, d) * diag[None, :]
    return e.astype(np.float32)


def make_state_dict(cfg: Optional[MimiConfig] = None, seed: int = 0,
                    num_quantizers: Optional[int] = None, codebook_stats: Optional[dict] = "auto"
                    ) -> Dict[str, np.ndarray]:
    """Encode-path state dict with HF parameter names, float32 numpy arrays.

    ``num_quantizers`` limits how many RVQ levels get codebooks (default: all ``cfg.num_quantizers``);
    the encode path only ever reads the first K levels.
    """
    cfg = cfg or MimiConfig()
    if isinstance(codebook_stats, str):
        codebook_stats = _load_codebook_stats()
    sd: Dict[str, np.ndarray] = {}
    for s in encoder_conv_specs(cfg):
        fan_in = s["cin"] * s["k"]
        sd[s["name"] + ".weight"] = _uniform_std((s["cout"], s["cin"], s["k"]), np.sqrt(2.0 / fan_in),
                                                 seed, s["name"], "w")
        sd[s["name"] + ".bias"] = _uniform_std((s["cout"],), 0.5 / np.sqrt(fan_in), seed, s["name"], "b")
    h, inter = cfg.hidden_size, cfg.intermediate_size
    for l in range(cfg.num_hidden_layers):
        p = f"encoder_transformer.layers.{l}."
        for nm in ("q_proj", "k_proj", "v_proj", "o_proj"):
            sd[p + f"self_attn.{nm}.weight"] = _uniform_std((h, h), 1.0 / np.sqrt(h), seed, p, nm)
        sd[p + "mlp.fc1.weight"] = _uniform_std((inter, h), 1.0 / np.sqrt(h), seed, p, "fc1")
        sd[p + "mlp.fc2.weight"] = _uniform_std((h, inter), 1.0 / np.sqrt(inter), seed, p, "fc2")
        for ln in ("input_layernorm", "post_attention_layernorm"):
            sd[p + ln + ".weight"] = np.float32(1.0) + uniform_pm1(h, seed, p, ln, "w") * np.float32(0.2)
            sd[p + ln + ".bias"] = uniform_pm1(h, seed, p, ln, "b") * np.float32(0.1)
        for ls in ("self_attn_layer_scale", "mlp_layer_scale"):
            u = uniform_pm1(h, seed, p, ls)
            sd[p + ls + ".scale"] = np.float32(0.15) + u * np.float32(0.1)
    ds_k = 2 * int(cfg.encodec_frame_rate / cfg.frame_rate)
    sd["downsample.conv.weight"] = _uniform_std((h, h, ds_k), 1.0 / np.sqrt(h * ds_k), seed, "ds")
    vqd = cfg.vector_quantization_hidden_dimension
    K = cfg.num_quantizers if num_quantizers is None else num_quantizers
    for q in ("semantic", "acoustic"):
        pre = f"quantizer.{q}_residual_vector_quantizer."
        sd[pre + "input_proj.weight"] = _uniform_std((vqd, h, 1), 1.0 / np.sqrt(h), seed, pre, "proj")
    nsem = cfg.num_semantic_quantizers
    for level in range(K):
        if level < nsem:
            pre = f"quantizer.semantic_residual_vector_quantizer.layers.{level}.codebook."
        else:
            pre = f"quantizer.acoustic_residual_vector_quantizer.layers.{level - nsem}.codebook."
        e = make_codebook(level, cfg, seed, codebook_stats)
        usage = np.float32(0.5) + (uniform_pm1(cfg.codebook_size, seed, pre, "use") + np.float32(1.0)) \
            * np.float32(0.75)
        # one dead entry per level exercises the clamp(min=1e-5) path of MimiEuclideanCodebook.embed
        usage[level % cfg.codebook_size] = np.float32(0.0)
        sd[pre + "embed_sum"] = (e * usage[:, None]).astype(np.float32)
        sd[pre + "embed_sum"][level % cfg.codebook_size] = e[level % cfg.codebook_size] * np.float32(1e-6)
        sd[pre + "cluster_usage"] = usage
        sd[pre + "initialized"] = np.ones((1,), dtype=np.float32)
    return sd


def state_dict_sha256(sd: Dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        v = np.ascontiguousarray(sd[k], dtype=np.float32)
        h.update(k.encode())
        h.update(str(v.shape).encode())
        h.update(v.tobytes())
    return h.hexdigest()


# --------------------------------------------------------------------------------------------
# audio (3 harmonics, f0 ~ U[90, 250] Hz, random envelope, small noise, clipped)
# --------------------------------------------------------------------------------------------
def _parabolic_sine(phase01: np.ndarray) -> np.ndarray:
    """Transcendental-free periodic wave ~ sin(2*pi*p): 4x(1-|x|) on x = 2p-1, negated."""
    x = phase01 * 2.0 - 1.0
    return -(x * 4.0) * (1.0 - np.abs(x))


def speech_like(num_samples: int, seed: int = 0, index: int = 0, sr: int = 24000,
                noise_std: float = 0.01) -> np.ndarray:
    """A deterministic speech-like float32 waveform of ``num_samples`` samples."""
    n = int(num_samples)
    if n <= 0:
        return np.zeros(0, dtype=np.float32)
    p = uniform01_f64(16, "audio", seed, index, "params")
    f0a, f0b = 90.0 + 160.0 * p[0], 90.0 + 160.0 * p[1]
    amps = (0.35 + 0.3 * p[2], 0.15 + 0.2 * p[3], 0.05 + 0.15 * p[4])
    t = np.arange(n, dtype=np.float64)
    # instantaneous f0 glides linearly; phase accumulated in closed form (exact ops only)
    frac = t / float(max(n, 1))
    f0 = f0a + (f0b - f0a) * frac
    base_phase = t * (f0a / sr) + (t * t) * ((f0b - f0a) / (2.0 * sr * max(n, 1)))
    sig = np.zeros(n, dtype=np.float64)
    for hnum, a in enumerate(amps, start=1):
        ph = base_phase * hnum
        ph = ph - np.floor(ph)
        sig = sig + _parabolic_sine(ph) * a
    # piecewise-linear envelope with knots every 0.1 s (syllable-ish), values in [0, 1]
    hop = sr // 10
    nk = n // hop + 2
    knots = uniform01_f64(nk, "audio", seed, index, "env")
    knots = np.where(knots < 0.25, 0.0, knots)  # pauses
    pos = t / hop
    i0 = np.floor(pos).astype(np.int64)
    w = pos - i0
    env = knots[i0] * (1.0 - w) + knots[i0 + 1] * w
    sig = sig * env
    _ = f0  # kept for readability of the model above
    noise = uniform01_f64(n, "audio", seed, index, "noise") * 2.0 - 1.0
    sig = sig + noise * (noise_std * np.sqrt(3.0))
    sig = np.clip(sig, -1.0, 1.0)
    return sig.astype(np.float32)


def noise_clip(num_samples: int, seed: int = 0, index: int = 0, std: float = 0.1) -> np.ndarray:
    """The robustness set: zero-mean noise with the given std (uniform, exact ops)."""
    u = uniform01_f64(int(num_samples), "noise", seed, index) * 2.0 - 1.0
    return (u * (std * np.sqrt(3.0))).astype(np.float32)


def clip_batch(num: int, num_samples: int, seed: int = 0) -> np.ndarray:
    return np.stack([speech_like(num_samples, seed, i) for i in range(num)])


def random_lengths(num: int, lo_s: float, hi_s: float, seed: int = 0, sr: int = 24000) -> List[int]:
    u = uniform01_f64(num, "lengths", seed)
    return [int(lo_s * sr + (hi_s - lo_s) * sr * x) for x in u]


def audio_sha256(arrays: Iterable[np.ndarray]) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float32).tobytes())
    return h.hexdigest()
