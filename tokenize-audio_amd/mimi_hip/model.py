"""``MimiHipModel``: the ``MimiModel.encode`` drop-in over the HIP engine.

Mirrors the model-level API every reference wrapper calls:

* ``model.encode(input_values[B, C, L], padding_mask=None, num_quantizers=None)`` ->
  ``MimiEncoderOutput`` with ``.audio_codes`` int64 ``[B, K, T]`` on the model's device, and tuple
  indexing (``out[0]`` is the codes; ``librispeech-mimi/utils.py:64-66`` does ``audio_codes[0][0]``).
  ``TF/modeling_mimi.py:1297-1386``: K defaults to ``config.num_quantizers`` (32), ``ValueError`` for
  K > 32 and for channels not in {1, 2}; ``padding_mask`` is accepted and ignored exactly as there
  (``:1244, :1247``).
* ``.to(device)``, ``.eval()``, ``get_encoded_length``, ``from_pretrained(local_dir | "kyutai/mimi")``.

The arithmetic runs in ``libmimi_hip.so`` (HIP kernels for gfx950); torch only supplies device memory and
the current stream.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import glob
import os
import threading
from dataclasses import dataclass
from typing import Dict, Optional, Union

import numpy as np
import torch

from . import _lib
from .config import MimiConfig, encoded_length


@dataclass
class MimiEncoderOutput:
    """Same fields as ``transformers`` ``MimiEncoderOutput`` (``TF/modeling_mimi.py:167-187``)."""
    audio_codes: torch.Tensor
    encoder_past_key_values: Optional[object] = None
    padding_cache: Optional[object] = None

    def to_tuple(self):
        return tuple(v for v in (self.audio_codes, self.encoder_past_key_values, self.padding_cache)
                     if v is not None)

    def __getitem__(self, i):
        if isinstance(i, str):
            return getattr(self, i)
        return self.to_tuple()[i]

    def __iter__(self):
        return iter(self.to_tuple())

    def __len__(self):
        return len(self.to_tuple())


def _resolve_device(device) -> torch.device:
    d = torch.device(device) if not isinstance(device, torch.device) else device
    if d.type != "cuda":
        raise ValueError(f"MimiHipModel runs on a HIP device ('cuda' under ROCm), got {d}")
    if d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def resolve_checkpoint(name_or_path: str) -> str:
    """Map ``"kyutai/mimi"`` (a Hub name; no network here) or a local directory/file to a local path.

    Order: an existing path; ``$MIMI_HIP_CHECKPOINT``; the huggingface_hub cache (``$HF_HUB_CACHE``, else
    ``$HF_HOME/hub``, else ``~/.cache/huggingface/hub``), ``models--<org>--<name>/snapshots/<rev>`` with ``<rev>``
    from ``refs/main`` when present (the snapshot ``from_pretrained`` would load offline), else the newest."""
    if os.path.exists(name_or_path):
        return name_or_path
    env = os.environ.get("MIMI_HIP_CHECKPOINT")
    if env and os.path.exists(env):
        return env
    hub = os.environ.get("HF_HUB_CACHE") or os.path.join(
        os.environ.get("HF_HOME", os.path.expanduser("~/.cache/huggingface")), "hub")
    repo = os.path.join(hub, "models--" + name_or_path.replace("/", "--"))
    ref = os.path.join(repo, "refs", "main")
    if os.path.exists(ref):
        with open(ref) as f:
            snap = os.path.join(repo, "snapshots", f.read().strip())
        if os.path.isdir(snap):
            return snap
    snaps = sorted(glob.glob(os.path.join(repo, "snapshots", "*")), key=os.path.getmtime)
    if snaps:
        return snaps[-1]
    raise FileNotFoundError(
        f"checkpoint {name_or_path!r} is not available locally; pass a directory holding model.safetensors "
        f"(+ config.json), set MIMI_HIP_CHECKPOINT, or use 'synthetic:<seed>' for the seeded test checkpoint")


class EncodeTicket:
    """An encode in flight (``MimiHipModel.encode_async``)."""

    def __init__(self, model: "MimiHipModel", ticket: int, out: torch.Tensor, audio: torch.Tensor):
        self._model, self._ticket, self.out, self._audio = model, ticket, out, audio

    def wait(self) -> torch.Tensor:
        if self._ticket:
            t, self._ticket = self._ticket, 0
            _lib.check(self._model._lib.mimi_encode_wait(self._model._h, t))
            self._audio = None
        return self.out


class MimiHipModel:
    """Encode-only Mimi on MI355X."""

    def __init__(self, state_dict: Optional[Dict[str, np.ndarray]] = None, config: Optional[MimiConfig] = None,
                 device: Union[str, torch.device] = "cuda", safetensors_path: Optional[str] = None):
        self.config = config or MimiConfig()
        self.config.validate_supported()
        self._lib = _lib.load()
        self.device = _resolve_device(device)
        self._cfg_c = _lib.config_from_py(self.config)
        handle = ctypes.c_void_p()
        _lib.check(self._lib.mimi_create(ctypes.byref(self._cfg_c), self.device.index, ctypes.byref(handle)))
        self._h = handle
        self._lock = threading.Lock()
        self._src = (state_dict, config, safetensors_path)  # for clone()
        try:
            if safetensors_path is not None:
                _lib.check(self._lib.mimi_load_safetensors(self._h, safetensors_path.encode()))
            if state_dict is not None:
                for name, value in state_dict.items():
                    if name.startswith(("decoder", "upsample")):
                        continue
                    arr = value.detach().cpu().numpy() if torch.is_tensor(value) else np.asarray(value)
                    arr = np.ascontiguousarray(arr, dtype=np.float32)
                    _lib.check(self._lib.mimi_set_weight(self._h, name.encode(), arr.ctypes.data, arr.size))
            _lib.check(self._lib.mimi_finalize(self._h))
        except Exception:
            self.close()
            raise

    # ---- construction helpers -------------------------------------------------------------------
    @classmethod
    def from_pretrained(cls, name_or_path: str = "kyutai/mimi", device="cuda", **kw) -> "MimiHipModel":
        if name_or_path.startswith("synthetic"):
            from . import synthetic
            seed = int(name_or_path.split(":", 1)[1]) if ":" in name_or_path else 0
            return cls(synthetic.make_state_dict(seed=seed), device=device)
        path = resolve_checkpoint(name_or_path)
        cfg = MimiConfig()
        if os.path.isdir(path):
            if os.path.exists(os.path.join(path, "config.json")):
                cfg = MimiConfig.from_json(path)
            files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
            if not files:
                raise FileNotFoundError(f"no .safetensors file in {path}")
            path = files[0]
        return cls(config=cfg, device=device, safetensors_path=path, **kw)

    def clone(self, device: Union[str, torch.device, None] = None) -> "MimiHipModel":
        """Another engine with the same weights and config (its own workspace; same calibration, so the same codes):
        independent encodes on several engines run concurrently (``MimiEncoder.encode_audio_chunks``)."""
        sd, cfg, path = self._src
        m = MimiHipModel(sd, config=cfg or self.config, device=device or self.device, safetensors_path=path)
        m.set_precision(self.precision)
        return m

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.mimi_destroy(h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- nn.Module-ish no-ops the wrappers call -------------------------------------------------
    def to(self, device=None, *args, **kwargs):
        if device is not None and not isinstance(device, torch.dtype):
            d = _resolve_device(device)
            if d != self.device:
                raise ValueError(f"engine lives on {self.device}; create a new MimiHipModel for {d}")
        return self

    def eval(self):
        return self

    def train(self, mode: bool = True):
        return self

    def get_encoded_length(self, input_length):
        if torch.is_tensor(input_length):
            return input_length.new_tensor([encoded_length(int(x), self.config) for x in input_length.flatten()]
                                           ).view_as(input_length)
        return encoded_length(int(input_length), self.config)

    # ---- encode --------------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check_k(self, K: int) -> int:
        """The reference's num_quantizers checks (TF/modeling_mimi.py:1335-1340); the C side would replace
        K <= 0 by config.num_quantizers, so a caller's 0 must not reach it with an output sized for 0 levels."""
        K = int(K)
        if K > self.config.num_quantizers:
            raise ValueError(
                f"The number of quantizers (i.e codebooks) asked should be lower than the total number of "
                f"quantizers {self.config.num_quantizers}, but is currently {K}.")
        if K < self.config.num_semantic_quantizers:
            raise ValueError(
                f"The number of quantizers (i.e codebooks) asked should be higher than the number of semantic "
                f"quantizers {self.config.num_semantic_quantizers}, but is currently {K}.")
        return K

    def _device_audio(self, audio: torch.Tensor) -> torch.Tensor:
        """device f32 [B, L], contiguous (the C ABI reads audio.data_ptr() as such)."""
        if audio.dim() != 2:
            raise ValueError(f"audio must be [batch, length], got {tuple(audio.shape)}")
        return audio.to(device=self.device, dtype=torch.float32).contiguous()

    def _out(self, B: int, K: int, T: int, out: Optional[torch.Tensor]) -> torch.Tensor:
        if out is None:
            return torch.empty((B, K, T), dtype=torch.int32, device=self.device)
        if (tuple(out.shape) != (B, K, T) or out.dtype != torch.int32 or out.device != self.device
                or not out.is_contiguous()):
            raise ValueError(f"out must be a contiguous int32 [{B}, {K}, {T}] tensor on {self.device}")
        return out

    def encode(self, input_values: torch.Tensor, padding_mask: Optional[torch.Tensor] = None,
               num_quantizers: Optional[int] = None, encoder_past_key_values=None, padding_cache=None,
               use_streaming: Optional[bool] = None, return_dict: Optional[bool] = None):
        if use_streaming:
            raise NotImplementedError("streaming encode (padding cache / KV cache) is not on the batch path")
        K = self._check_k(self.config.num_quantizers if num_quantizers is None else num_quantizers)
        if not torch.is_tensor(input_values):
            input_values = torch.as_tensor(np.asarray(input_values))
        if input_values.dim() != 3:
            raise ValueError(f"input_values must be [batch, channels, length], got {tuple(input_values.shape)}")
        B, channels, L = input_values.shape
        if channels < 1 or channels > 2:
            raise ValueError(f"Number of audio channels must be 1 or 2, but got {channels}")
        if channels != self.config.audio_channels:
            raise ValueError(f"expected {self.config.audio_channels} audio channel(s), got {channels}")
        T = encoded_length(L, self.config)
        codes = torch.empty((B, K, T), dtype=torch.int32, device=self.device)
        if B == 0 or L == 0:
            return MimiEncoderOutput(codes.long())
        x = input_values.to(device=self.device, dtype=torch.float32).reshape(B, L).contiguous()
        # (no Python lock: the engine serialises enqueues itself and waits outside its lock, so threads sharing
        # one engine overlap -- the YODAS2 thread pool, yodas2-mimi/process_shard.py:691-717)
        _lib.check(self._lib.mimi_encode(self._h, ctypes.c_void_p(x.data_ptr()), B, L, K,
                                         ctypes.c_void_p(codes.data_ptr()), self._stream()))
        out = codes.long()
        if return_dict is False:
            return (out, None, None)
        return MimiEncoderOutput(out)

    def encode_int32(self, audio: torch.Tensor, num_quantizers: int, out: Optional[torch.Tensor] = None
                     ) -> torch.Tensor:
        """Lean path for the bench / shard driver: device f32 [B, L] in, device int32 [B, K, T] out."""
        K = self._check_k(num_quantizers)
        audio = self._device_audio(audio)
        B, L = audio.shape
        out = self._out(B, K, encoded_length(L, self.config), out)
        _lib.check(self._lib.mimi_encode(self._h, ctypes.c_void_p(audio.data_ptr()), B, L, K,
                                         ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def encode_host(self, audio: np.ndarray, num_quantizers: int) -> np.ndarray:
        """Host f32 [B, L] in, host int32 [B, K, T] out, in one C call (``mimi_encode_host``: the engine's own device
        and pinned buffers, one host synchronisation) on the current stream -- the per-utterance path of
        ``MimiEncoder.encode_audio_chunk``.  The same codes as ``encode_int32`` on a device copy."""
        K = self._check_k(num_quantizers)
        a = np.ascontiguousarray(audio, dtype=np.float32)
        if a.ndim != 2 or a.shape[0] < 1 or a.shape[1] < 1:
            raise ValueError(f"audio must be a non-empty [batch, length] array, got {tuple(a.shape)}")
        B, L = a.shape
        out = np.empty((B, K, encoded_length(L, self.config)), dtype=np.int32)
        _lib.check(self._lib.mimi_encode_host(self._h, ctypes.c_void_p(a.ctypes.data), B, L, K,
                                              ctypes.c_void_p(out.ctypes.data), self._stream()))
        return out

    def encode_async(self, audio: torch.Tensor, num_quantizers: int, out: Optional[torch.Tensor] = None
                     ) -> "EncodeTicket":
        """Enqueue an encode of device f32 [B, L] on the current stream and return without waiting
        (``mimi_encode_async``); ``ticket.wait()`` returns the int32 [B, K, T] codes once they are final (the
        f16x3 overflow check runs there).  The ticket keeps ``audio`` alive until then."""
        K = self._check_k(num_quantizers)
        audio = self._device_audio(audio)
        B, L = audio.shape
        out = self._out(B, K, encoded_length(L, self.config), out)
        t = ctypes.c_int64()
        _lib.check(self._lib.mimi_encode_async(self._h, ctypes.c_void_p(audio.data_ptr()), B, L, K,
                                               ctypes.c_void_p(out.data_ptr()), self._stream(), ctypes.byref(t)))
        return EncodeTicket(self, t.value, out, audio)

    def encode_ragged_async(self, audio: torch.Tensor, lengths, num_quantizers: int,
                            out: Optional[torch.Tensor] = None) -> "EncodeTicket":
        """Ragged batch (``mimi_encode_ragged_async``): item b = ``audio[b, :lengths[b]]`` of a device f32 [B, Lmax]
        tensor, encoded exactly as it would be alone at its own length (bit for bit), in one pass that skips every
        item's rows past its length.  ``ticket.wait()`` returns int32 [B, K, T(Lmax)]; item b's codes are
        ``[:, :encoded_length(lengths[b])]`` (the frames past are unspecified)."""
        K = self._check_k(num_quantizers)
        audio = self._device_audio(audio)
        B, L = audio.shape
        lens = np.ascontiguousarray(np.asarray(lengths, dtype=np.int64).reshape(-1))
        if lens.shape != (B,) or (B and (int(lens.min()) < 1 or int(lens.max()) > L)):
            raise ValueError(f"lengths must be {B} values in [1, {L}]")
        out = self._out(B, K, encoded_length(L, self.config), out)
        t = ctypes.c_int64()
        _lib.check(self._lib.mimi_encode_ragged_async(self._h, ctypes.c_void_p(audio.data_ptr()),
                                                      ctypes.c_void_p(lens.ctypes.data), B, L, K,
                                                      ctypes.c_void_p(out.data_ptr()), self._stream(),
                                                      ctypes.byref(t)))
        return EncodeTicket(self, t.value, out, audio)

    def encode_ragged(self, audio: torch.Tensor, lengths, num_quantizers: int,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.encode_ragged_async(audio, lengths, num_quantizers, out).wait()

    def quantize(self, embedding: torch.Tensor, num_quantizers: int) -> torch.Tensor:
        """Quantizer alone on a pre-quantizer embedding [B, 512, T] -> int64 codes [B, K, T]."""
        B, C, T = embedding.shape
        emb = embedding.to(device=self.device, dtype=torch.float32).permute(0, 2, 1).contiguous()
        codes = torch.empty((num_quantizers, B * T), dtype=torch.int32, device=self.device)
        with self._lock:
            _lib.check(self._lib.mimi_rvq_encode(self._h, ctypes.c_void_p(emb.data_ptr()), B * T, num_quantizers,
                                                 ctypes.c_void_p(codes.data_ptr()), self._stream()))
        return codes.view(num_quantizers, B, T).permute(1, 0, 2).long()

    # ---- instrumentation ------------------------------------------------------------------------
    def set_precision(self, mode: str):
        """'f16x3' (default: fp32 emulated on the fp16 matrix cores, 2 planes at calibrated fixed scales),
        'bf16x6' (3 bf16 planes), 'f32' (fp32 MFMA) or 'bf16x3' (2 bf16 planes, ~1e-5)."""
        _lib.check(self._lib.mimi_set_precision(self._h, _lib.PRECISIONS[mode]))

    @property
    def precision(self) -> str:
        v = self._lib.mimi_get_precision(self._h)
        return {i: k for k, i in _lib.PRECISIONS.items()}[v]

    def calibrate(self):
        """Run the f16x3 activation-scale calibration now (otherwise it runs inside the first f16x3 encode)."""
        _lib.check(self._lib.mimi_calibrate(self._h))

    @property
    def f16_reruns(self) -> int:
        """Encodes that took the f16x3 overflow fallback (per-item re-encode, bf16x6 where an item overflows)."""
        return int(self._lib.mimi_f16_reruns(self._h))

    @property
    def rvq_chain_reruns(self) -> int:
        """Encodes re-run on the per-level RVQ kernels because the persistent RVQ chain gave up (never returned)."""
        return int(self._lib.mimi_rvq_chain_reruns(self._h))

    def set_graphs(self, enable: bool = True):
        """hipGraph replay of repeated f16x3 encode shapes (default on; identical codes, fewer launches)."""
        _lib.check(self._lib.mimi_set_graphs(self._h, int(enable)))

    @property
    def graph_replays(self) -> int:
        return int(self._lib.mimi_graph_replays(self._h))

    def set_option(self, key: str, value: int):
        """Kernel-variant option (identical codes either way): "stage0_fused" 0 = stage-0 block and down conv 0 as
        two kernels, 1 = one fused kernel (default); "ln_fused" 0 = LayerNorm launches before q/k/v and fc1, on small
        grids (batch 1-4) 1 = fc1 computes the LayerNorm of its rows itself (default), 2 = fc1 and q/k/v do."""
        _lib.check(self._lib.mimi_set_option(self._h, key.encode(), int(value)))

    def act_scales(self):
        """f16x3 diagnostics: {tensor: (fixed scale, max|x| of the last encode, headroom 2^15 / (scale * max))}."""
        n = 256
        names = ctypes.create_string_buffer(64 * n)
        sc = (ctypes.c_float * n)()
        mx = (ctypes.c_float * n)()
        cnt = ctypes.c_int32()
        _lib.check(self._lib.mimi_act_scales(self._h, n, names, sc, mx, ctypes.byref(cnt)))
        out = {}
        for i in range(cnt.value):
            name = names.raw[64 * i:64 * (i + 1)].split(b"\0", 1)[0].decode()
            head = 32768.0 / (sc[i] * mx[i]) if sc[i] > 0 and mx[i] > 0 else float("inf")
            out[name] = (sc[i], mx[i], head)
        return out

    def set_profiling(self, enable=True):
        """True / 1: events between every stage; 2: around each encode's first stage only; False / 0: off."""
        _lib.check(self._lib.mimi_set_profiling(self._h, int(enable)))

    def profile_reset(self):
        _lib.check(self._lib.mimi_profile_reset(self._h))

    def profile_read(self):
        n = 64
        names = ctypes.create_string_buffer(128 * n)
        ms = (ctypes.c_double * n)()
        launches = (ctypes.c_int64 * n)()
        fb = (ctypes.c_double * (2 * n))()
        cnt = ctypes.c_int32()
        _lib.check(self._lib.mimi_profile_read(self._h, n, names, ms, launches, fb, ctypes.byref(cnt)))
        out = {}
        for i in range(cnt.value):
            nm = names.raw[128 * i:128 * (i + 1)].split(b"\0", 1)[0].decode()
            stage, _, kernel = nm.partition("|")
            key, j = stage, 2
            while key in out:  # one stage run by two kernel symbols (e.g. the last layer's fc2): "fc2#2"
                key, j = f"{stage}#{j}", j + 1
            out[key] = dict(kernel=kernel, ms=ms[i], launches=launches[i], flops=fb[2 * i], bytes=fb[2 * i + 1])
        return out

    def profile_sequence(self):
        """[(stage, kernel symbol)] of the last profiled encode in launch order (mimi_profile_sequence)."""
        n = 512
        names = ctypes.create_string_buffer(128 * n)
        cnt = ctypes.c_int32()
        _lib.check(self._lib.mimi_profile_sequence(self._h, n, names, ctypes.byref(cnt)))
        out = []
        for i in range(cnt.value):
            nm = names.raw[128 * i:128 * (i + 1)].split(b"\0", 1)[0].decode()
            stage, _, kernel = nm.partition("|")
            out.append((stage, kernel))
        return out

    def set_taps(self, enable: bool = True):
        _lib.check(self._lib.mimi_set_taps(self._h, int(enable)))

    def get_tap(self, name: str) -> np.ndarray:
        numel = ctypes.c_int64()
        dims = (ctypes.c_int64 * 3)()
        _lib.check(self._lib.mimi_get_tap(self._h, name.encode(), None, 0, ctypes.byref(numel), dims))
        buf = np.empty(numel.value, dtype=np.float32)
        _lib.check(self._lib.mimi_get_tap(self._h, name.encode(), ctypes.c_void_p(buf.ctypes.data), buf.size,
                                          ctypes.byref(numel), dims))
        return buf.reshape(dims[0], dims[1], dims[2])
