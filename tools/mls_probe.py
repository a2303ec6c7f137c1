"""Probe of the MLS-style ragged stream: wall time of MimiEncoder.encode_audio_chunks over N utterances vs the same
ragged encodes back to back on pre-staged device tensors (device-bound rate) -- separates host staging from the
engine.  python tools/mls_probe.py [N] [lo] [hi]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))


def main():
    import numpy as np
    import torch
    from mimi_hip import synthetic
    from mimi_hip.encoder import MimiEncoder
    from mimi_hip.model import MimiHipModel
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 320
    lo = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    hi = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    dev = torch.device("cuda", 0)
    model = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=8), device=dev)
    enc = MimiEncoder(device=dev, model=model, num_quantizers=8)
    lengths = synthetic.random_lengths(n, lo, hi, seed=77)
    clips = [synthetic.speech_like(lengths[i], 77, i) for i in range(n)]
    secs = sum(lengths) / 24000.0
    for _ in range(2):
        enc.encode_audio_chunks(clips, 24000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enc.encode_audio_chunks(clips, 24000)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # device-bound: the same groups (sorted by length, 32 each) pre-staged on the device, encoded back to back
    order = sorted(range(n), key=lambda i: lengths[i])
    groups = [order[i:i + 32] for i in range(0, n, 32)]
    staged = []
    for g in groups:
        L = max(lengths[i] for i in g)
        x = torch.zeros((len(g), L), dtype=torch.float32)
        for r, i in enumerate(g):
            x[r, :lengths[i]] = torch.from_numpy(clips[i])
        staged.append((x.to(dev), [lengths[i] for i in g]))
    for x, ls in staged:
        model.encode_ragged(x, ls, 8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tickets = [model.encode_ragged_async(x, ls, 8) for x, ls in staged[:8]]
    for t in tickets:
        t.wait()
    for x, ls in staged[8:]:
        model.encode_ragged_async(x, ls, 8).wait()
    torch.cuda.synchronize()
    devt = time.perf_counter() - t0
    print(f"utterances {n}: {secs:.0f} audio-s; encode_audio_chunks {wall * 1e3:.1f} ms = {secs / wall:.0f} audio-s/s; "
          f"pre-staged ragged encodes {devt * 1e3:.1f} ms = {secs / devt:.0f} audio-s/s", flush=True)


if __name__ == "__main__":
    main()
