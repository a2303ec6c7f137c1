"""Per-utterance loop under a kernel trace: where the ~1.9 ms of each encode_audio_chunk call goes.

    run:      python tools/trace_utt.py run  [n_utts]      (the bench's per_utterance_k32 loop, prints ms per call)
    summary:  python tools/trace_utt.py summary DIR         (rocprofv3 --kernel-trace --memory-copy-trace CSVs)

The summary cuts the trace at the encodes' last kernel (the persistent RVQ chain, or rvq_final), and per utterance
reports: wall from the first dispatch to the last kernel's end, kernel-busy time, idle gaps between dispatches inside
it, and the host time between one utterance's last kernel and the next one's first dispatch (H2D, D2H, host code).
"""
import collections
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))


def run(n):
    import torch
    from mimi_hip import synthetic
    from mimi_hip.encoder import MimiEncoder
    from mimi_hip.model import MimiHipModel
    dev = torch.device("cuda", 0)
    sd = synthetic.make_state_dict(seed=0, num_quantizers=32)
    model = MimiHipModel(sd, device=dev)
    enc = MimiEncoder(device=dev, model=model)
    lens = synthetic.random_lengths(n, 10.0, 20.0, seed=99)
    utts = [synthetic.speech_like(n_, 99, i) for i, n_ in enumerate(lens)]
    for a in utts[:2]:
        enc.encode_audio_chunk(a, 24000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in utts:
        enc.encode_audio_chunk(a, 24000)
    dt = time.perf_counter() - t0
    print(f"{n} utterances, {sum(lens) / 24000:.1f} audio-s: {1e3 * dt / n:.3f} ms per call, "
          f"{sum(lens) / 24000 / dt:.0f} audio-s/s", flush=True)


def summary(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    cps = []
    for g in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        cps += list(csv.DictReader(open(g)))
    ends = [i for i, r in enumerate(rows) if "rvq_chain" in r["Kernel_Name"] or "rvq_final" in r["Kernel_Name"]]
    per = []
    names = collections.defaultdict(float)
    for a, b in zip(ends[-13:-1], ends[-12:]):  # the last 12 utterances
        seg = rows[a + 1:b + 1]
        s0, s1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
        prev_end = int(rows[a]["End_Timestamp"])
        cp = [c for c in cps if prev_end <= int(c["Start_Timestamp"]) < s1]
        cpt = sum(int(c["End_Timestamp"]) - int(c["Start_Timestamp"]) for c in cp)
        per.append(((s1 - s0) / 1e3, busy / 1e3, (s0 - prev_end) / 1e3, len(seg), cpt / 1e3, len(cp)))
        for r in seg:
            names[r["Kernel_Name"].replace("void ", "").split("(")[0][:70]] += \
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("per utterance: wall(first dispatch..last end) us, kernel busy us, host gap before it us, kernels, "
          "copies us (count)")
    for p in per:
        print(f"  {p[0]:8.1f} {p[1]:8.1f} {p[2]:8.1f} {p[3]:4d} {p[4]:8.1f} ({p[5]})")
    n = len(per)
    print(f"mean: wall {sum(p[0] for p in per) / n:.1f}  busy {sum(p[1] for p in per) / n:.1f}  "
          f"host gap {sum(p[2] for p in per) / n:.1f}  copies {sum(p[4] for p in per) / n:.1f}")
    print("kernel time per utterance (us), top 20:")
    for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  {v / n:8.1f}  {k}")




def host_split(n=24):
    """Host-side split of one encode_audio_chunk call: the engine call (mimi_encode_host) vs the Python around it."""
    import torch
    from mimi_hip import synthetic
    from mimi_hip.encoder import MimiEncoder
    from mimi_hip.model import MimiHipModel
    dev = torch.device("cuda", 0)
    model = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=32), device=dev)
    enc = MimiEncoder(device=dev, model=model)
    lens = synthetic.random_lengths(n, 10.0, 20.0, seed=99)
    utts = [synthetic.speech_like(n_, 99, i) for i, n_ in enumerate(lens)]
    for a in utts[:2]:
        enc.encode_audio_chunk(a, 24000)
    orig = model.encode_host
    t_eng = []

    def timed(*a, **k):
        t0 = time.perf_counter()
        r = orig(*a, **k)
        t_eng.append(time.perf_counter() - t0)
        return r
    model.encode_host = timed
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in utts:
        enc.encode_audio_chunk(a, 24000)
    dt = (time.perf_counter() - t0) / n
    print(f"per call {1e6 * dt:.1f} us: engine call {1e6 * sum(t_eng) / n:.1f} us, python around it "
          f"{1e6 * (dt - sum(t_eng) / n):.1f} us", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 24)
    elif sys.argv[1] == "host":
        host_split()
    else:
        summary(sys.argv[2])
