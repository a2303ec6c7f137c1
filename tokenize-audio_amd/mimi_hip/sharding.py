"""Utterance-sharded multi-GPU encode: one process per GPU, utterance i -> rank i % N.

The reference scales only by independent SLURM jobs, one GPU each (``*/submit/job_template.sh``); inside a
node this driver does the same thing with one process per GPU launched by ``torchrun``:

* partition: round-robin by utterance index (``shard_indices``); no state crosses utterances;
* batching: each rank forms batches from ITS utterances in original order (``make_batches``), so a padded
  batch has exactly the composition the reference wrapper would give those utterances, which is what the
  pad-to-longest tail-frame semantics depend on (``emilia-mimi/process_shard.py:88-140``);
* encode: the drop-in ``MimiEncoder`` of this package on the rank's GPU -- no collective on the data path; its
  ``encode_batches`` pipeline is used when present (the next batch is loaded, staged and copied to the GPU while
  the current one encodes), and a rank only ever reads its own utterances (``audio`` may be a lazy sequence, or
  ``loader(i)`` loads utterance i on demand);
* merge: codes are gathered to rank 0 on the host (``torch.distributed.gather_object``; ~400 B per
  audio-second) and put back in original index order.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence

import numpy as np


def shard_indices(n_items: int, world: int, rank: int) -> List[int]:
    """Utterance indices owned by ``rank`` (round-robin)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} / world {world}")
    return list(range(rank, n_items, world))


def make_batches(indices: Sequence[int], batch_size: int) -> List[List[int]]:
    """Consecutive batches of ``batch_size`` over the given indices, original order kept."""
    if batch_size <= 0:
        raise ValueError("batch_size must be positive")
    idx = list(indices)
    return [idx[i:i + batch_size] for i in range(0, len(idx), batch_size)]


def encode_shard(encode_batch: Callable[[List[np.ndarray]], List[np.ndarray]], audio, world: int, rank: int,
                 batch_size: int, encode_batches: Optional[Callable] = None) -> dict:
    """Encode this rank's utterances; returns {index: codes}.  ``audio[i]`` is only read for this rank's indices,
    one batch at a time (lazily, when ``encode_batches`` -- a pipelined batch iterator -- asks for it)."""
    out = {}
    batches = make_batches(shard_indices(len(audio), world, rank), batch_size)
    if encode_batches is not None:
        results = encode_batches([audio[i] for i in b] for b in batches)
    else:
        results = (encode_batch([audio[i] for i in b]) for b in batches)
    for batch, codes in zip(batches, results):
        if len(codes) != len(batch):
            raise RuntimeError("encoder returned a different number of items than it was given")
        out.update(zip(batch, codes))
    return out


class LazyAudio:
    """A sequence of ``n`` utterances loaded on demand by ``loader(i)`` (a rank touches only its own indices)."""

    def __init__(self, n: int, loader: Callable[[int], np.ndarray]):
        self.n, self.loader = n, loader

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        if not 0 <= i < self.n:
            raise IndexError(i)
        return self.loader(i)


def merge_shards(parts: Sequence[dict], n_items: int) -> List[np.ndarray]:
    merged = {}
    for p in parts:
        overlap = merged.keys() & p.keys()
        if overlap:
            raise RuntimeError(f"utterances encoded twice: {sorted(overlap)[:5]}")
        merged.update(p)
    missing = [i for i in range(n_items) if i not in merged]
    if missing:
        raise RuntimeError(f"utterances missing after merge: {missing[:5]}")
    return [merged[i] for i in range(n_items)]


class DistributedMimiEncoder:
    """Per-rank driver.  ``encode_all(audio)`` returns the merged codes (original order) on rank 0 and
    ``None`` elsewhere.  ``encoder`` defaults to ``mimi_hip.MimiEncoder`` on ``cuda:LOCAL_RANK``."""

    def __init__(self, model_id: str = "kyutai/mimi", batch_size: int = 32, encoder=None,
                 num_quantizers: Optional[int] = None, sample_rate: int = 24000):
        import torch.distributed as dist
        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.world = self.dist.get_world_size() if self.dist else 1
        self.rank = self.dist.get_rank() if self.dist else 0
        self.batch_size = batch_size
        self.sample_rate = sample_rate
        if encoder is None:
            import torch

            from .encoder import MimiEncoder
            local = int(os.environ.get("LOCAL_RANK", "0"))
            # the current device must be this rank's GPU: an nccl process group stages gather_object there
            torch.cuda.set_device(local)
            encoder = MimiEncoder(model_id, device=f"cuda:{local}", num_quantizers=num_quantizers)
        self.encoder = encoder

    def encode_all(self, audio: Optional[Sequence[np.ndarray]] = None, n_items: Optional[int] = None,
                   loader: Optional[Callable[[int], np.ndarray]] = None) -> Optional[List[np.ndarray]]:
        """Encode the shard (``audio``, or ``n_items`` utterances loaded by ``loader(i)``); the merged codes on rank
        0, None elsewhere."""
        if audio is None:
            if loader is None or n_items is None:
                raise ValueError("pass audio, or n_items and loader")
            audio = LazyAudio(n_items, loader)
        eb = getattr(self.encoder, "encode_batches", None)
        part = encode_shard(lambda b: self.encoder.encode_audio_batch(b, self.sample_rate), audio, self.world,
                            self.rank, self.batch_size,
                            encode_batches=(lambda it: eb(it, self.sample_rate)) if eb else None)
        if self.dist is None:
            return merge_shards([part], len(audio))
        parts = [None] * self.world if self.rank == 0 else None
        self.dist.gather_object(part, parts, dst=0)
        return merge_shards(parts, len(audio)) if self.rank == 0 else None
