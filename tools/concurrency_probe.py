"""Probe: does splitting one B-clip encode into S concurrent sub-batches on S streams (one engine handle per
stream, one host thread each) beat the single-stream encode?  Prints ms per B-clip step for each split.

    python tools/concurrency_probe.py --batch 32 --splits 1 2 4
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--replicas", action="store_true",
                    help="every stream encodes the WHOLE batch (S batches in flight) instead of 1/S of it")
    args = ap.parse_args()
    import torch
    from mimi_hip import synthetic
    from mimi_hip.config import encoded_length
    from mimi_hip.model import MimiHipModel

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K, B = 8, args.batch
    L = int(round(args.seconds * 24000))
    sd = synthetic.make_state_dict(seed=0, num_quantizers=K)
    audio = torch.from_numpy(synthetic.clip_batch(B, L, seed=1000)).to(dev)
    models = [MimiHipModel(sd, device=dev) for _ in range(max(args.splits))]
    streams = [torch.cuda.Stream(dev) for _ in models]
    ref = None
    for S in args.splits:
        nb = B if args.replicas else B // S
        outs = [torch.empty((nb, K, encoded_length(L)), dtype=torch.int32, device=dev) for _ in range(S)]

        def worker(i, n):
            with torch.cuda.stream(streams[i]):
                for _ in range(n):
                    x = audio if args.replicas else audio[i * nb:(i + 1) * nb]
                    models[i].encode_int32(x, K, out=outs[i])
            streams[i].synchronize()

        def run(n):
            ts = [threading.Thread(target=worker, args=(i, n)) for i in range(S)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()

        run(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.steps)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps / (S if args.replicas else 1)
        codes = outs[-1] if args.replicas else torch.cat(outs, 0)
        if ref is None:
            ref = codes.clone()
        same = bool(torch.equal(codes, ref))
        print(f"splits {S}: {dt * 1e3:.3f} ms per {B}-clip step, {B * args.seconds / dt:.0f} audio-s/s, "
              f"codes equal to split-1: {same}", flush=True)


if __name__ == "__main__":
    main()
