"""Host FLAC decode rate (mimi_flac_decode): LibriSpeech-like 16 kHz 16-bit mono files, one core and a thread pool.
    python tools/flac_bench.py [n_files] [seconds_per_file] [threads]"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tokenize-audio_amd"), os.path.join(ROOT, "tests")]
import flac_writer as fw  # noqa: E402
from mimi_hip import ingest  # noqa: E402

n_files = int(sys.argv[1]) if len(sys.argv) > 1 else 8
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 12.0
threads = int(sys.argv[3]) if len(sys.argv) > 3 else len(os.sched_getaffinity(0))
rng = np.random.default_rng(0)
n = int(secs * 16000)
t = np.arange(n)
files = []
for i in range(n_files):  # speech-like: a few harmonics with an envelope plus noise; LPC 8 / FIXED subframes
    x = sum(np.sin(2 * np.pi * f * t / 16000 + rng.uniform(0, 6)) / (k + 1) for k, f in enumerate([140, 280, 420, 900]))
    x = x * (0.5 + 0.5 * np.sin(2 * np.pi * 3 * t / 16000)) * 0.2 + 0.003 * rng.standard_normal(n)
    pcm = np.clip(np.round(x * 32767), -32768, 32767).astype(np.int64)[None]
    files.append(fw.encode(pcm, 16000, 16, block_sizes=[4096], seed=i, kinds=[("lpc", 8, 12), ("fixed", 2)]))
mb = sum(len(f) for f in files) / 1e6
t0 = time.perf_counter()
for f in files:
    ingest.decode_flac(f)
one = time.perf_counter() - t0
t0 = time.perf_counter()
with ThreadPoolExecutor(threads) as ex:
    list(ex.map(ingest.decode_flac, files * 4))
many = time.perf_counter() - t0
print(f"{n_files} files x {secs} s ({mb:.2f} MB, {mb * 8e6 / (n_files * n):.1f} bits/sample): "
      f"1 thread {n_files * secs / one:.0f} audio-s/s ({n_files * n / one / 1e6:.1f} M samples/s); "
      f"{threads} threads {4 * n_files * secs / many:.0f} audio-s/s")
