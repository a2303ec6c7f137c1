"""ctypes binding of ``libmimi_hip.so`` (C ABI declared in ``include/mimi_hip.h``).

The library is built in-tree (``python __graft_entry__.py`` or ``make -C tokenize-audio_amd/csrc``).  There
is deliberately no fallback: if the library is missing the product path raises, it never silently runs
something else.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

LIB_NAME = "libmimi_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

MIMI_OK = 0
PRECISIONS = {"f32": 0, "bf16x6": 1, "bf16x3": 2, "f16x3": 3}
STATUS_NAMES = {
    0: "MIMI_OK", 1: "MIMI_ERR_INVALID_ARGUMENT", 2: "MIMI_ERR_HIP", 3: "MIMI_ERR_OUT_OF_MEMORY",
    4: "MIMI_ERR_WEIGHTS", 5: "MIMI_ERR_UNSUPPORTED", 6: "MIMI_ERR_IO", 7: "MIMI_ERR_STATE",
}

# every symbol include/mimi_hip.h declares (tests check the library exports exactly these)
EXPORTED_SYMBOLS = (
    "mimi_config_default", "mimi_config_from_json", "mimi_create_from_dir", "mimi_create", "mimi_set_weight", "mimi_load_safetensors", "mimi_finalize",
    "mimi_encode", "mimi_encode_async", "mimi_encode_wait", "mimi_encode_host", "mimi_encode_ragged", "mimi_encode_ragged_async", "mimi_rvq_encode", "mimi_set_precision", "mimi_get_precision", "mimi_calibrate", "mimi_f16_reruns", "mimi_rvq_chain_reruns", "mimi_set_graphs", "mimi_graph_replays", "mimi_set_option", "mimi_act_scales", "mimi_encoded_length",
    "mimi_encoded_length_cfg",
    "mimi_workspace_bytes", "mimi_destroy", "mimi_last_error", "mimi_set_profiling", "mimi_profile_read",
    "mimi_profile_reset", "mimi_profile_sequence", "mimi_set_taps", "mimi_get_tap", "mimi_resample_poly",
    "mimi_bpe_create", "mimi_bpe_best", "mimi_bpe_merge", "mimi_bpe_destroy", "mimi_flac_info", "mimi_flac_decode",
    "mimi_split_check", "mimi_gelu_check",
)
RESAMPLE_MAX_TAPS = 65536  # MIMI_RESAMPLE_MAX_TAPS


class MimiConfigC(ctypes.Structure):
    _fields_ = [
        ("sampling_rate", ctypes.c_int32), ("audio_channels", ctypes.c_int32), ("hidden_size", ctypes.c_int32),
        ("num_filters", ctypes.c_int32), ("num_ratios", ctypes.c_int32), ("upsampling_ratios", ctypes.c_int32 * 8),
        ("kernel_size", ctypes.c_int32), ("last_kernel_size", ctypes.c_int32),
        ("residual_kernel_size", ctypes.c_int32), ("compress", ctypes.c_int32), ("codebook_size", ctypes.c_int32),
        ("codebook_dim", ctypes.c_int32), ("num_quantizers", ctypes.c_int32),
        ("num_semantic_quantizers", ctypes.c_int32), ("vq_hidden_dim", ctypes.c_int32),
        ("num_hidden_layers", ctypes.c_int32), ("intermediate_size", ctypes.c_int32),
        ("num_attention_heads", ctypes.c_int32), ("head_dim", ctypes.c_int32), ("sliding_window", ctypes.c_int32),
        ("downsample_kernel", ctypes.c_int32), ("downsample_stride", ctypes.c_int32),
        ("norm_eps", ctypes.c_float), ("rope_theta", ctypes.c_float), ("codebook_eps", ctypes.c_float),
    ]


class MimiHipError(RuntimeError):
    def __init__(self, status: int, message: str):
        self.status = status
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")


def _oom_base():
    try:
        import torch
        return torch.cuda.OutOfMemoryError
    except Exception:  # torch-less use of the binding
        return MemoryError


class MimiHipOutOfMemoryError(MimiHipError, _oom_base()):
    """MIMI_ERR_OUT_OF_MEMORY.  Also a ``torch.cuda.OutOfMemoryError``, so a caller's OOM guard written for the
    reference's torch encode (e.g. the YODAS2 long-chunk split, yodas2-mimi/process_shard.py:434-493) sees it."""


_lib = None
_lock = threading.Lock()


def _declare(lib):
    c = ctypes
    vp = c.c_void_p
    sig = {
        "mimi_config_default": (None, [c.POINTER(MimiConfigC)]),
        "mimi_config_from_json": (c.c_int, [c.c_char_p, c.POINTER(MimiConfigC)]),
        "mimi_create_from_dir": (c.c_int, [c.c_char_p, c.c_int, c.POINTER(vp)]),
        "mimi_create": (c.c_int, [c.POINTER(MimiConfigC), c.c_int, c.POINTER(vp)]),
        "mimi_set_weight": (c.c_int, [vp, c.c_char_p, vp, c.c_int64]),
        "mimi_load_safetensors": (c.c_int, [vp, c.c_char_p]),
        "mimi_finalize": (c.c_int, [vp]),
        "mimi_encode": (c.c_int, [vp, vp, c.c_int32, c.c_int64, c.c_int32, vp, vp]),
        "mimi_encode_async": (c.c_int, [vp, vp, c.c_int32, c.c_int64, c.c_int32, vp, vp, c.POINTER(c.c_int64)]),
        "mimi_encode_wait": (c.c_int, [vp, c.c_int64]),
        "mimi_encode_host": (c.c_int, [vp, vp, c.c_int32, c.c_int64, c.c_int32, vp, vp]),
        "mimi_encode_ragged": (c.c_int, [vp, vp, vp, c.c_int32, c.c_int64, c.c_int32, vp, vp]),
        "mimi_encode_ragged_async": (c.c_int, [vp, vp, vp, c.c_int32, c.c_int64, c.c_int32, vp, vp,
                                               c.POINTER(c.c_int64)]),
        "mimi_rvq_encode": (c.c_int, [vp, vp, c.c_int64, c.c_int32, vp, vp]),
        "mimi_set_precision": (c.c_int, [vp, c.c_int32]),
        "mimi_get_precision": (c.c_int, [vp]),
        "mimi_calibrate": (c.c_int, [vp]),
        "mimi_f16_reruns": (c.c_int64, [vp]),
        "mimi_rvq_chain_reruns": (c.c_int64, [vp]),
        "mimi_set_graphs": (c.c_int, [vp, c.c_int32]),
        "mimi_graph_replays": (c.c_int64, [vp]),
        "mimi_set_option": (c.c_int, [vp, c.c_char_p, c.c_int64]),
        "mimi_act_scales": (c.c_int, [vp, c.c_int32, c.c_char_p, c.POINTER(c.c_float), c.POINTER(c.c_float),
                                      c.POINTER(c.c_int32)]),
        "mimi_encoded_length": (c.c_int64, [c.c_int64]),
        "mimi_encoded_length_cfg": (c.c_int64, [c.POINTER(MimiConfigC), c.c_int64]),
        "mimi_workspace_bytes": (c.c_int64, [vp, c.c_int32, c.c_int64]),
        "mimi_destroy": (None, [vp]),
        "mimi_last_error": (c.c_char_p, []),
        "mimi_set_profiling": (c.c_int, [vp, c.c_int]),
        "mimi_profile_read": (c.c_int, [vp, c.c_int32, c.c_char_p, c.POINTER(c.c_double), c.POINTER(c.c_int64),
                                        c.POINTER(c.c_double), c.POINTER(c.c_int32)]),
        "mimi_profile_reset": (c.c_int, [vp]),
        "mimi_profile_sequence": (c.c_int, [vp, c.c_int32, c.c_char_p, c.POINTER(c.c_int32)]),
        "mimi_set_taps": (c.c_int, [vp, c.c_int]),
        "mimi_get_tap": (c.c_int, [vp, c.c_char_p, vp, c.c_int64, c.POINTER(c.c_int64), c.POINTER(c.c_int64)]),
        "mimi_bpe_create": (c.c_int, [c.c_int, vp, c.c_int64, vp, vp, c.c_int64, c.c_int32, c.c_int32, c.c_int32,
                                      c.POINTER(vp)]),
        "mimi_bpe_best": (c.c_int, [vp, c.POINTER(c.c_int32), c.POINTER(c.c_int32), c.POINTER(c.c_int64)]),
        "mimi_bpe_merge": (c.c_int, [vp, c.c_int32, c.c_int32, c.c_int32, c.c_int32]),
        "mimi_bpe_destroy": (None, [vp]),
        "mimi_flac_info": (c.c_int, [vp, c.c_int64, c.POINTER(c.c_int32), c.POINTER(c.c_int32),
                                     c.POINTER(c.c_int32), c.POINTER(c.c_int64)]),
        "mimi_flac_decode": (c.c_int, [vp, c.c_int64, vp, c.c_int64, c.POINTER(c.c_int64)]),
        "mimi_split_check": (c.c_int, [vp, c.c_int64, c.c_float, vp, vp]),
        "mimi_gelu_check": (c.c_int, [vp, c.c_int64, vp, vp]),
        "mimi_resample_poly": (c.c_int, [vp, vp, vp, c.c_int32, vp, vp, vp, c.c_int64, vp, c.c_int32, c.c_int32,
                                         c.c_int32, c.c_int64, vp]),
    }
    ab = bool(os.environ.get("MIMI_HIP_LIB"))  # an A/B run against an older build may lack newer entry points
    for name, (res, args) in sig.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def load(path: Optional[str] = None):
    """Load (once) and return the library.  Raises ``ImportError`` if it has not been built."""
    global _lib
    with _lock:
        if _lib is None:
            p = path or os.environ.get("MIMI_HIP_LIB", LIB_PATH)
            if not os.path.exists(p):
                raise ImportError(
                    f"{LIB_NAME} not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                    f"or `make -C tokenize-audio_amd/csrc` (the Mimi encode path has no non-HIP fallback)")
            _lib = _declare(ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL))
        return _lib


def check(status: int) -> None:
    if status != MIMI_OK:
        msg = load().mimi_last_error()
        cls = MimiHipOutOfMemoryError if status == 3 else MimiHipError
        raise cls(status, msg.decode() if msg else "")


def default_config() -> MimiConfigC:
    cfg = MimiConfigC()
    load().mimi_config_default(ctypes.byref(cfg))
    return cfg


def config_from_py(cfg) -> MimiConfigC:
    """mimi_hip.config.MimiConfig -> C struct."""
    c = default_config()
    c.sampling_rate = cfg.sampling_rate
    c.audio_channels = cfg.audio_channels
    c.hidden_size = cfg.hidden_size
    c.num_filters = cfg.num_filters
    c.num_ratios = len(cfg.upsampling_ratios)
    for i, r in enumerate(cfg.upsampling_ratios):
        c.upsampling_ratios[i] = r
    c.kernel_size = cfg.kernel_size
    c.last_kernel_size = cfg.last_kernel_size
    c.residual_kernel_size = cfg.residual_kernel_size
    c.compress = cfg.compress
    c.codebook_size = cfg.codebook_size
    c.codebook_dim = cfg.codebook_dim
    c.num_quantizers = cfg.num_quantizers
    c.num_semantic_quantizers = cfg.num_semantic_quantizers
    c.vq_hidden_dim = cfg.vector_quantization_hidden_dimension
    c.num_hidden_layers = cfg.num_hidden_layers
    c.intermediate_size = cfg.intermediate_size
    c.num_attention_heads = cfg.num_attention_heads
    c.head_dim = cfg.head_dim
    c.sliding_window = cfg.sliding_window
    c.downsample_kernel = 2 * int(cfg.encodec_frame_rate / cfg.frame_rate)
    c.downsample_stride = 2
    c.norm_eps = cfg.norm_eps
    c.rope_theta = cfg.rope_theta
    return c
