"""Determinism under contention (diagnostic for GPUTEST_r04's sharded-encode mismatch).

driver:  python tools/det_concurrent.py [iters]
  runs, one after the other: two workers at once (the persistent RVQ chain on), two at once (chain off), one alone
  with dirtied staging memory, and compares every worker's codes of every iteration with the first solo result.
worker:  python tools/det_concurrent.py --worker ROLE ITERS CHAIN DIRTY OUT
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402


def batches():
    import shard_worker
    from mimi_hip import sharding
    audio = shard_worker.clips()
    out = []
    for rank in range(2):
        out += sharding.make_batches(sharding.shard_indices(len(audio), 2, rank), shard_worker.BATCH)
    return audio, out


def worker(role, iters, chain, dirty, path):
    import torch
    from mimi_hip import synthetic
    from mimi_hip.encoder import MimiEncoder
    from mimi_hip.model import MimiHipModel
    if dirty:  # leave NaN / huge garbage in the caching allocators' freed blocks (pinned host and device)
        for n in (1 << 16, 1 << 18, 1 << 20, 1 << 22):
            p = torch.empty(n, dtype=torch.float32, pin_memory=True)
            p.fill_(float("nan") if n & (1 << 18) else 3.0e38)
            d = torch.empty(n, dtype=torch.float32, device="cuda:0")
            d.fill_(float("nan") if n & (1 << 20) else -3.0e38)
            del p, d
        torch.cuda.synchronize()
    model = MimiHipModel(synthetic.make_state_dict(seed=0), device="cuda:0")
    model.set_option("rvq_chain", chain)
    enc = MimiEncoder(device="cuda:0", model=model)
    audio, bl = batches()
    res = {}
    t0 = time.time()
    for it in range(iters):
        for bi, out in enumerate(enc.encode_batches([[audio[i] for i in b] for b in bl], 24000)):
            for i, c in zip(bl[bi], out):
                res[f"p{it}_{i}"] = c
        for bi, b in enumerate(bl):
            for i, c in zip(b, enc.encode_audio_batch([audio[i] for i in b], 24000)):
                res[f"s{it}_{i}"] = c
        if it % 10 == 0:
            print(f"worker {role} chain {chain} it {it} {time.time() - t0:.1f}s", flush=True)
    res["reruns"] = np.array(model.f16_reruns)
    res["chain_reruns"] = np.array(model.rvq_chain_reruns)
    np.savez(path, **res)
    model.close()


def compare(ref, z, tag):
    bad = 0
    for k in z.files:
        if k in ("reruns", "chain_reruns"):
            continue
        i = int(k.split("_")[1])
        if not np.array_equal(z[k], ref[i]):
            d = np.argwhere(z[k] != ref[i])
            print(f"  {tag} {k}: {len(d)} codes differ, first (level, frame) {d[:6].tolist()}", flush=True)
            bad += 1
    print(f"{tag}: {bad} mismatching arrays of {len(z.files) - 2}, f16 reruns {int(z['reruns'])}, chain reruns "
          f"{int(z['chain_reruns'])}", flush=True)
    return bad


def driver(iters):
    out = os.path.join(ROOT, "gpurun_out", "det")
    os.makedirs(out, exist_ok=True)
    me = os.path.abspath(__file__)

    def run(specs):
        procs = [subprocess.Popen([sys.executable, "-u", me, "--worker", str(r), str(iters), str(c), str(d),
                                   os.path.join(out, f"{name}.npz")]) for name, r, c, d in specs]
        rcs = [p.wait(timeout=600) for p in procs]
        assert all(rc == 0 for rc in rcs), rcs

    run([("solo_ref", 0, 0, 0)])
    z = np.load(os.path.join(out, "solo_ref.npz"))
    ref = {int(k.split("_")[1]): z[k] for k in z.files if k.startswith("s0_")}
    total = compare(ref, z, "solo_ref(chain 0)")
    run([("pair_chain_a", 0, 1, 0), ("pair_chain_b", 1, 1, 0)])
    run([("pair_nochain_a", 0, 0, 0), ("pair_nochain_b", 1, 0, 0)])
    run([("solo_dirty", 0, 1, 1)])
    run([("pair_dirty_a", 0, 1, 1), ("pair_dirty_b", 1, 1, 1)])
    for name in ("pair_chain_a", "pair_chain_b", "pair_nochain_a", "pair_nochain_b", "solo_dirty", "pair_dirty_a",
                 "pair_dirty_b"):
        total += compare(ref, np.load(os.path.join(out, f"{name}.npz")), name)
    print("TOTAL mismatching arrays", total, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        worker(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6])
    else:
        driver(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
