"""GPU report: end-to-end accuracy and speed of each GEMM precision mode against the golden fixtures.

    python tools/precision_report.py [--out gpurun_out/precision_report.json]

For each mode (f32, bf16x6, bf16x3): pre-quantizer relative error (max|d| / max|ref|) on the golden clips,
per-stage errors on the 0.5 s clip, code exact-match rate (K = 32 and K = 8) against transformers' codes,
the number of mismatches NOT explained as near-ties of the reference's own distances, and device ms per
B = 32 x 10 s encode.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tokenize-audio_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mimi_hip import synthetic  # noqa: E402
from mimi_hip.model import MimiHipModel  # noqa: E402
from test_gpu_parity import margin_audit, rel_err  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "precision_report.json"))
    ap.add_argument("--modes", default="f32,bf16x6,f16x3,bf16x3")
    args = ap.parse_args()
    with np.load(os.path.join(ROOT, "tests", "golden", "golden.npz")) as z:
        g = {k: z[k] for k in z.files}
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_meta.json")))
    sd = synthetic.make_state_dict(seed=0)
    model = MimiHipModel(sd, device="cuda:0")
    clips = {"speech10s": synthetic.speech_like(240000, 7, 6), "speech60s": synthetic.speech_like(1440000, 7, 7),
             "noise5s": synthetic.noise_clip(120000, 7, 0, std=0.1)}
    report = {}
    for mode in args.modes.split(","):
        model.set_precision(mode)
        r = {"clips": {}}
        model.set_taps(True)
        for tag, x in clips.items():
            codes = model.encode(torch.from_numpy(x)[None, None].cuda()).audio_codes[0].cpu().numpy()
            emb = model.get_tap("downsample")[0].T
            ref = g[f"embcodes_{tag}"].astype(np.int64)
            frac, bad = margin_audit(codes, ref, g[f"margins_{tag}"])
            r["clips"][tag] = {"pre_quantizer_rel_err": rel_err(emb, g[f"emb_{tag}"]),
                               "exact_match_k32": frac, "exact_match_k8": float((codes[:8] == ref[:8]).mean()),
                               "mismatches": int((codes != ref).sum()), "codes": int(ref.size),
                               "unexplained": len(bad)}
        x = torch.from_numpy(synthetic.speech_like(12000, meta["audio_seed"], 100))[None, None].cuda()
        model.encode(x, num_quantizers=32)
        stages = {}
        for key, refv in g.items():
            if not key.startswith("stage_"):
                continue
            name, sub = key[len("stage_"):].rsplit("_sub", 1)
            tap = {"res0": "res0_elu", "res1": "res1_elu", "res2": "res2_elu", "res3": "res3_elu",
                   "down3": "down3_elu", "pre_quantizer": "downsample"}.get(name, name)
            t = model.get_tap(tap)[0].T
            if name.startswith(("conv", "res", "down")):
                t = t[:, ::int(sub)]
            rv = refv
            if tap.endswith("_elu"):
                rv = np.where(rv > 0, rv, np.expm1(rv.astype(np.float64))).astype(np.float32)
            if name.startswith("xfmr"):
                t = t.T
            stages[name] = rel_err(t, rv)
        r["stages"] = stages
        model.set_taps(False)
        audio = torch.from_numpy(synthetic.clip_batch(32, 240000, seed=3)).cuda()
        for _ in range(2):
            model.encode_int32(audio, 8)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            model.encode_int32(audio, 8)
        torch.cuda.synchronize()
        r["ms_per_b32x10s"] = (time.perf_counter() - t0) / 5 * 1000
        report[mode] = r
        print(mode, json.dumps(r)[:600], flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
