"""CPU: the utterance-sharded multi-GPU driver, world_size 2 over gloo (no GPU needed).

Each rank encodes its round-robin share with the SAME batch composition rule the single-process wrapper
uses; the merged result must equal a single-process run over the same per-rank batches."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mimi_hip import sharding


def test_partition_and_batches():
    assert sharding.shard_indices(7, 2, 0) == [0, 2, 4, 6]
    assert sharding.shard_indices(7, 2, 1) == [1, 3, 5]
    assert sharding.make_batches([1, 3, 5, 7, 9], 2) == [[1, 3], [5, 7], [9]]
    with pytest.raises(ValueError):
        sharding.shard_indices(3, 2, 2)
    all_idx = sorted(i for r in range(3) for i in sharding.shard_indices(10, 3, r))
    assert all_idx == list(range(10))


def test_merge_checks():
    a = {0: np.zeros(1), 2: np.ones(1)}
    b = {1: np.full(1, 5.0)}
    out = sharding.merge_shards([a, b], 3)
    assert [float(x[0]) for x in out] == [0.0, 5.0, 1.0]
    with pytest.raises(RuntimeError):
        sharding.merge_shards([a, {0: np.zeros(1)}], 3)
    with pytest.raises(RuntimeError):
        sharding.merge_shards([a], 3)


class _FakeEncoder:
    """Deterministic stand-in whose output depends on the batch composition (like pad-to-longest does)."""

    def encode_audio_batch(self, batch, sr):
        lmax = max(len(a) for a in batch)
        return [np.array([len(a), lmax, int(a[0] * 1000)], dtype=np.int64) for a in batch]


def _worker(rank, world, port, audio, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        enc = sharding.DistributedMimiEncoder(encoder=_FakeEncoder(), batch_size=2)
        out = enc.encode_all(audio)
        if rank == 0:
            q.put([o.tolist() for o in out])
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_matches_single_process_per_rank_batches():
    rng = np.random.RandomState(0)
    audio = [rng.rand(int(n)).astype(np.float32) + 0.01 for n in rng.randint(5, 50, size=9)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, audio, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # expected: each rank batches its own items in order; batch composition decides lmax
    fake = _FakeEncoder()
    exp = {}
    for r in range(2):
        for b in sharding.make_batches(sharding.shard_indices(len(audio), 2, r), 2):
            exp.update(zip(b, fake.encode_audio_batch([audio[i] for i in b], 24000)))
    assert got == [exp[i].tolist() for i in range(len(audio))]
