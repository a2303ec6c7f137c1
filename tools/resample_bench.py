"""Throughput of the host-ingest resampler kernel (resample_poly_kernel) on device-resident clips.

    python tools/resample_bench.py [--clips 256 --seconds 20 --rate 16000]

Algorithmic bytes per launch = 4 B per input sample read + 4 B per output sample written; achieved GB/s =
those bytes / the launch's average device time (HIP events on the launch stream), against ~6.3 TB/s
achievable HBM (MI355X_MICROARCH.md).  Also times scipy.signal.resample_poly on one host core for a sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--rate", type=int, default=16000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    from mimi_hip import ingest
    dev = torch.device("cuda", 0)
    n = int(a.seconds * a.rate)
    x = torch.randn(a.clips * n, device=dev) * 0.1      # clips back to back, resident in HBM
    lens = [n] * a.clips
    for _ in range(3):
        out, nfix = ingest.resample_packed(x, lens, a.rate, 24000)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        out, nfix = ingest.resample_packed(x, lens, a.rate, 24000)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    nout = sum(nfix)
    algo = 4 * (a.clips * n + nout)
    from scipy.signal import resample_poly
    xs = x[:n].cpu().numpy()
    import math
    g = math.gcd(a.rate, 24000)
    t0 = time.perf_counter()
    resample_poly(xs, 24000 // g, a.rate // g)
    cpu_s = time.perf_counter() - t0
    print(json.dumps({"kernel": "resample_poly_kernel", "clips": a.clips, "clip_seconds": a.seconds,
                      "rate": a.rate, "ms_per_call": round(ms, 4),
                      "audio_s_per_s": round(a.clips * a.seconds / (ms / 1e3), 1),
                      "algorithmic_bytes": algo, "achieved_GBps": round(algo / (ms / 1e3) / 1e9, 1),
                      "cpu_scipy_one_core_audio_s_per_s": round(a.seconds / cpu_s, 1) if cpu_s else None}))


if __name__ == "__main__":
    main()
