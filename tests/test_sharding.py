"""CPU: the utterance-sharded multi-GPU driver, world_size 2 over gloo (no GPU needed).

Each rank encodes its round-robin share with the SAME batch composition rule the single-process wrapper
uses; the merged result must equal a single-process run over the same per-rank batches."""
import os
import socket

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import assert_codes_in_range
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


class _FakePipelinedEncoder(_FakeEncoder):
    """As _FakeEncoder, with the pipelined batch iterator: pulls batch i + 1 before yielding batch i's codes."""

    def encode_batches(self, batches, sr):
        prev = None
        for b in batches:
            b = list(b)
            if prev is not None:
                yield self.encode_audio_batch(prev, sr)
            prev = b
        if prev is not None:
            yield self.encode_audio_batch(prev, sr)


def _worker(rank, world, port, audio, q, lazy=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if lazy:  # each rank loads only its own utterances, through the pipelined iterator
            touched = []

            def load(i):
                touched.append(i)
                return audio[i]
            enc = sharding.DistributedMimiEncoder(encoder=_FakePipelinedEncoder(), batch_size=2)
            out = enc.encode_all(n_items=len(audio), loader=load)
            assert sorted(touched) == sharding.shard_indices(len(audio), world, rank), touched
        else:
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


@pytest.mark.parametrize("lazy", [False, True])
def test_gloo_world2_matches_single_process_per_rank_batches(lazy):
    rng = np.random.RandomState(0)
    audio = [rng.rand(int(n)).astype(np.float32) + 0.01 for n in rng.randint(5, 50, size=9)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, audio, q, lazy)) for r in range(2)]
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


@pytest.mark.gpu
def test_sharded_real_engines_match_single(tmp_path):
    """Two ranks, each with its own HIP engine (both on cuda:0 here), gloo group, DistributedMimiEncoder over the
    real MimiEncoder: the merged codes equal one process encoding the same per-rank batches."""
    import subprocess
    import sys

    import torch
    if torch.cuda.device_count() < 1:
        pytest.skip("no HIP device")
    here = os.path.dirname(os.path.abspath(__file__))
    out = tmp_path / "merged.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", f"--master-port={_free_port()}", os.path.join(here, "shard_worker.py"), str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import shard_worker
    from mimi_hip import synthetic
    from mimi_hip.encoder import MimiEncoder
    from mimi_hip.model import MimiHipModel
    audio = shard_worker.clips()
    model = MimiHipModel(synthetic.make_state_dict(seed=0), device="cuda:0")
    enc = MimiEncoder(device="cuda:0", model=model)
    exp = {}
    for rank in range(2):
        for b in sharding.make_batches(sharding.shard_indices(len(audio), 2, rank), shard_worker.BATCH):
            exp.update(zip(b, enc.encode_audio_batch([audio[i] for i in b], 24000)))
    model.close()
    with np.load(out, allow_pickle=False) as z:
        for i in range(len(audio)):
            assert_codes_in_range(z[f"c{i}"])
            assert np.array_equal(z[f"c{i}"], exp[i]), i


def test_bench_rank_map_rejects_shared_gpus_under_nccl():
    """bench.py's N-GPU line carries each rank's device (host, PCI bus): under nccl two ranks on one device abort the
    run, under the gloo rehearsal they are labelled `sharing`; a process group of another size aborts too."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    r = lambda i, bus: {"rank": i, "host": "h", "pci_bus": bus}  # noqa: E731
    ok = bench.check_rank_places([r(i, f"0000:{0x10 * (i + 1):02x}:00") for i in range(8)], "nccl", 8, 8)
    assert ok == {"backend": "nccl", "world_size": 8, "distinct_devices": 8, "sharing": False}
    shared = [r(0, "0000:75:00"), r(1, "0000:75:00")]
    assert bench.check_rank_places(shared, "gloo", 2, 2)["sharing"] is True
    with pytest.raises(SystemExit, match="share a GPU"):
        bench.check_rank_places(shared, "nccl", 2, 2)
    with pytest.raises(SystemExit, match="process group"):
        bench.check_rank_places(shared[:1], "nccl", 1, 2)
    assert bench.check_rank_places([r(0, "0000:75:00")], "none", 1, 1)["distinct_devices"] == 1
