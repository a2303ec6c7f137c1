"""Host -> device copy of one utterance's samples (the per-utterance path's H2D): pageable copy vs staging through
pinned memory with 1 .. 8 host threads.  Prints microseconds per copy (median of 200).

    python tools/h2d_probe.py [seconds_of_audio]
"""
import sys
import threading
import time

import numpy as np
import torch


def med(f, n=200):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return 1e6 * float(np.median(ts))


def main():
    sec = float(sys.argv[1]) if len(sys.argv) > 1 else 15.5
    n = int(sec * 24000)
    a = np.random.default_rng(0).standard_normal(n).astype(np.float32)
    d = torch.empty(n, dtype=torch.float32, device="cuda")
    pin = torch.empty(n, dtype=torch.float32, pin_memory=True)
    pn = pin.numpy()
    s = torch.cuda.current_stream()

    def pageable():
        d.copy_(torch.from_numpy(a), non_blocking=True)
        s.synchronize()

    def staged(k):
        parts = np.array_split(np.arange(n), k)

        def cp(idx):
            pn[idx[0]:idx[-1] + 1] = a[idx[0]:idx[-1] + 1]
        if k == 1:
            pn[:] = a
        else:
            ts = [threading.Thread(target=cp, args=(p,)) for p in parts]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        d.copy_(pin, non_blocking=True)
        s.synchronize()

    def memcpy_only():
        pn[:] = a

    def dma_only():
        d.copy_(pin, non_blocking=True)
        s.synchronize()

    for _ in range(20):
        pageable()
        staged(1)
    print(f"{n * 4 / 1e6:.2f} MB: pageable H2D {med(pageable):.1f} us; pinned memcpy alone {med(memcpy_only):.1f} us; "
          f"pinned DMA alone {med(dma_only):.1f} us")
    for k in (1, 2, 4, 8):
        print(f"  staged through pinned, {k} python threads: {med(lambda: staged(k)):.1f} us")


if __name__ == "__main__":
    main()
