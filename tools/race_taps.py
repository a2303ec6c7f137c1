"""Which stage of engine A's encode varies while engine B loads the GPU?  Taps of a uniform batch (encoder stages,
transformer output, downsample, pre-quantizer) compared run to run against A alone."""
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))
from mimi_hip import synthetic  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sd = synthetic.make_state_dict(seed=0)
A = MimiHipModel(sd, device="cuda:0")
B = A.clone()
xu = torch.from_numpy(synthetic.clip_batch(3, 150000, seed=9)).cuda()
load = torch.from_numpy(synthetic.clip_batch(16, 240000, seed=10)).cuda()
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
A.set_taps(True)
names = None


def run_a():
    global names
    with torch.cuda.stream(sa):
        c = A.encode_int32(xu, 32).cpu().numpy()
    if names is None:
        names = ["conv0", "res0_elu", "down0", "res1_elu", "down1", "res2_elu", "down2", "res3_elu", "down3_elu",
                 "encoder", "xfmr0", "xfmr7", "ds_gemm", "downsample", "proj"]
    return c, {n: A.get_tap(n).copy() for n in names}


ref = run_a()
print("taps compared:", names, {n: ref[1][n].shape for n in names}, flush=True)
stop = threading.Event()


def loader():
    with torch.cuda.stream(sb):
        while not stop.is_set():
            B.encode_int32(load, 32)


def report(tag, rep, c, t):
    diff = {n: int((t[n] != ref[1][n]).sum()) for n in names if not np.array_equal(t[n], ref[1][n])}
    if diff or not np.array_equal(c, ref[0]):
        where = {n: [(i, float(ref[1][n][tuple(i)]), float(t[n][tuple(i)]))
                     for i in np.argwhere(t[n] != ref[1][n])[:4].tolist()] for n in diff}
        print(f"{tag} rep {rep}: codes differ {int((c != ref[0]).sum())}; taps differ {diff}; at {where}", flush=True)


for rep in range(8):
    report("idle", rep, *run_a())
th = threading.Thread(target=loader)
th.start()
for rep in range(reps):
    report("loaded", rep, *run_a())
stop.set()
th.join()
print("done", flush=True)

if len(sys.argv) > 2 and sys.argv[2] == "nocontrols":
    sys.exit(0)
# control: torch's own GEMM under the same load -- bitwise repeatable?
g = torch.Generator(device="cuda").manual_seed(0)
ma = torch.randn(4096, 4096, device="cuda", generator=g)
mb = torch.randn(4096, 4096, device="cuda", generator=g)
with torch.cuda.stream(sa):
    mref = (ma @ mb).cpu()
stop.clear()
th = threading.Thread(target=loader)
th.start()
bad = 0
for rep in range(reps):
    with torch.cuda.stream(sa):
        m = (ma @ mb).cpu()
    if not torch.equal(m, mref):
        bad += 1
        d = (m != mref).nonzero()[:4].tolist()
        print(f"torch matmul rep {rep}: {int((m != mref).sum())} differ at {d}", flush=True)
stop.set()
th.join()
print("torch matmul under load: mismatching reps", bad, "of", reps, flush=True)

# control: D2D copies + an elementwise kernel under load
big = torch.randn(3 * 150000 * 64, device="cuda", generator=g)
with torch.cuda.stream(sa):
    cref = (big * 1.5 + 0.25).cpu()
stop.clear()
th = threading.Thread(target=loader)
th.start()
bad = 0
for rep in range(reps):
    with torch.cuda.stream(sa):
        y = big.clone()
        cc = (y * 1.5 + 0.25).cpu()
    if not torch.equal(cc, cref):
        bad += 1
        d = (cc != cref).nonzero()[:4].flatten().tolist()
        print(f"torch copy rep {rep}: {int((cc != cref).sum())} differ at {d}", flush=True)
stop.set()
th.join()
print("torch copy+axpb under load: mismatching reps", bad, "of", reps, flush=True)
