"""Throughput of the Mimi encode hot path on MI355X: audio-seconds encoded per wall-second (K = 8, 24 kHz).

    python bench.py [--gpus N --steps K --warmup W --batch B --seconds S]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Workload (BASELINE.json configs[1]): one step = one ``mimi_encode`` of a batch of B = 32 synthetic 10 s /
24 kHz clips (speech-like, seeded) already resident in HBM, K = 8 codebooks, weights = the seeded synthetic
kyutai/mimi-shaped checkpoint (random init; throughput does not depend on values).  Multi-GPU: one process
per GPU, each encodes its own batches (utterance round-robin, no data-path collective: SURVEY.md §8e);
per-GPU work is fixed as N grows ("weak").  The timed region is bracketed by barrier + synchronize; the
max over ranks is reported.  Rank 0 prints ONE JSON line.

roofline: per-kernel device time from HIP events recorded by the engine on its launch stream during the
timed steps, aggregated per kernel symbol; the dominant kernel's algorithmic FLOPs / its time vs the MFMA
peak of the arithmetic it runs on (see ``mfma_peak_for``).  cpu_baseline: the oracle (torch CPU restatement of MimiModel.encode) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "tokenize-audio_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: fp32 MFMA/vector peak
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E spec
BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak
F16X3_PEAK_TFLOPS = BF16_PEAK_TFLOPS / 3  # fp32-accurate products as 3 fp16 products


def mfma_peak_for(kernel: str):
    """Peak that bounds a GEMM kernel, in fp32-equivalent TFLOP/s of the algorithmic (fp32) FLOPs it does.

    fp32 kernels run on v_mfma_f32_32x32x2_f32: 157.3 TF.  The split-bf16 kernels compute the same fp32 GEMM
    as P bf16 products per fp32 multiply-add (NS = 3 planes -> 6 products, NS = 2 -> 3) on the dense bf16
    MFMA, so their ceiling is 2.5 PF / P (416.7 TF for bf16x6, 833.3 TF for bf16x3)."""
    if "gemm_bf16x_kernel<" in kernel or "gemm_planes_kernel<" in kernel:
        targs = [t.strip() for t in kernel.split("<", 1)[1].rstrip(">").split(",")]
        ns = int(targs[4])
        products = {3: 6, 2: 3}[ns]
        kind = "fp16" if targs[-1] == "true" else "bf16"
        return BF16_PEAK_TFLOPS / products, (f"{kind} MFMA dense peak (= bf16 rate) / {products} products "
                                             f"(split-{kind}, {ns} planes)")
    if "_h16_kernel" in kernel:  # fp16-plane fused blocks / attention: 3 fp16 products per MAC
        return BF16_PEAK_TFLOPS / 3, "fp16 MFMA dense peak (= bf16 rate) / 3 products (split-fp16, 2 planes)"
    return FP32_PEAK_TFLOPS, "fp32 MFMA peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--num-quantizers", type=int, default=8)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0,
                    help="wall budget of the CPU-baseline sample (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-profile", action="store_true", help="do not record per-stage events")
    ap.add_argument("--precision", default=None, help="GEMM precision mode (default: the engine's)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def cpu_baseline(seconds_budget: float, threads: int, clip_s: float):
    """The oracle on the host cores: whole 10 s clips, batch 1 (config 1 of BASELINE.json), until the budget
    is spent.  Returns the same metric (audio-s / wall-s)."""
    import torch

    from mimi_hip import synthetic
    from oracle import mimi_ref
    threads = max(1, min(threads, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    sd = synthetic.make_state_dict(seed=0, num_quantizers=8)
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    n = int(clip_s * 24000)
    clip = torch.from_numpy(synthetic.speech_like(n, 0, 0))[None, None]
    mimi_ref.encode(clip, sdt, 8)  # warm
    done, t0 = 0, time.perf_counter()
    while True:
        mimi_ref.encode(clip, sdt, 8)
        done += 1
        el = time.perf_counter() - t0
        if el >= seconds_budget or done >= 200:
            break
    try:
        cpu_model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        cpu_model = "unknown"
    return {"value": round(done * clip_s / el, 3), "unit": "audio-sec/sec", "cores": threads, "kind": "port",
            "sample": f"{done} x {clip_s:g} s clips, batch 1, K=8, oracle/mimi_ref.py (torch {torch.__version__} CPU, "
                      f"{threads} threads, {cpu_model})"}


def pmc_lookup(pmc_kernels, name):
    """PMC summary entry of a kernel symbol: the summary keys drop rocprof's 'void ' prefix and, for
    non-template kernels, the parameter list that the engine's names keep."""
    if name in pmc_kernels:
        return pmc_kernels[name]
    bare = name[5:] if name.startswith("void ") else name
    if "(" in bare and not bare.endswith(">"):
        bare = bare[:bare.index("(")]
    return pmc_kernels.get(bare, {})


def north_star_groups(prof, steps, pmc_path):
    """BASELINE.json's reporting asks: HBM GB/s and TFLOP/s of the SEANet conv stack, MFMA utilisation of the
    transformer.  Device ms and algorithmic FLOPs from the engine's events; HBM bytes = the PMC passes'
    FETCH_SIZE x 2 + WRITE_SIZE per launch of each kernel symbol (profiles/pmc_summary.json; a symbol shared
    by several stages carries its average) x that stage's launches."""
    pmc = {}
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f).get("kernels", {})
    groups = {
        "conv_stack": [s for s in prof if s.startswith(("res", "down_s", "final"))],
        "transformer": [s for s in prof if s in ("layernorm", "qkv", "attention", "o_proj", "fc1", "fc2")],
        "quantizer": [s for s in prof if s in ("downsample", "input_proj", "rvq")],
    }
    out = {}
    for g, stages in groups.items():
        if not stages:
            continue
        ms = sum(prof[s]["ms"] for s in stages) / steps
        fl = sum(prof[s]["flops"] for s in stages) / steps
        hbm = [pmc_lookup(pmc, prof[s]["kernel"]).get("traffic_bytes") for s in stages]
        d = {"stages": stages, "ms_per_step": round(ms, 3), "tflops": round(fl / (ms / 1e3) / 1e12, 1),
             "frac_f16x3_peak": round(fl / (ms / 1e3) / 1e12 / F16X3_PEAK_TFLOPS, 4)}
        missing = [prof[s]["kernel"] for s, b in zip(stages, hbm) if b is None]
        if missing:
            d["hbm_unmeasured_kernels"] = sorted(set(missing))
        else:
            by = sum(b * prof[s]["launches"] / steps for b, s in zip(hbm, stages))
            d.update({"hbm_bytes_per_step": round(by), "hbm_GBps": round(by / (ms / 1e3) / 1e9, 1),
                      "frac_hbm_peak": round(by / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)})
        out[g] = d
    return out


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from mimi_hip import synthetic
    from mimi_hip.config import encoded_length
    from mimi_hip.model import MimiHipModel

    K = args.num_quantizers
    B = args.batch
    L = int(round(args.seconds * 24000))
    model = MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=K), device=dev)
    if args.precision:
        model.set_precision(args.precision)
    # this rank's utterances: a distinct seeded slice of the shard (round-robin i -> rank i % N)
    audio = torch.from_numpy(synthetic.clip_batch(B, L, seed=1000 + rank)).to(dev)
    codes = torch.empty((B, K, encoded_length(L)), dtype=torch.int32, device=dev)

    def step():
        model.encode_int32(audio, K, out=codes)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not args.no_profile:
        model.profile_reset()
        model.set_profiling(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = {}
    if not args.no_profile:
        model.set_profiling(False)
        prof = model.profile_read()

    # PCIe-inclusive rate (host f32 in -> device codes -> host): reported beside, never as `value`
    host_audio = audio.cpu().pin_memory()
    torch.cuda.synchronize()
    tp0 = time.perf_counter()
    for _ in range(max(1, min(args.steps, 3))):
        a = host_audio.to(dev, non_blocking=True)
        c = model.encode_int32(a, K)
        c.cpu()
    torch.cuda.synchronize()
    pcie_rate = max(1, min(args.steps, 3)) * B * args.seconds / (time.perf_counter() - tp0)

    total_audio_s = world * B * args.seconds * args.steps
    value = total_audio_s / elapsed
    result = {
        "metric": "audio-sec encoded/sec (Mimi 8-codebook, 24 kHz)",
        "value": round(value, 2),
        "unit": "audio-sec/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded speech-like 24 kHz clips; seeded random-init kyutai/mimi-shaped weights)",
        "config": {"workload": f"LibriTTS-R-style batch encode: batch={B} x {args.seconds:g} s @ 24 kHz, "
                               f"K={K} codebooks, 1 encode per step per GPU",
                   "global_batch": world * B, "clip_seconds": args.seconds, "num_quantizers": K,
                   "parallelism": f"utterance round-robin x{world} (no collective)",
                   "gemm_precision": model.precision},
        "pcie_inclusive_value": round(pcie_rate * world, 2),
    }
    if prof:
        per_kernel = {}
        for stage, st in prof.items():
            k = per_kernel.setdefault(st["kernel"], {"ms": 0.0, "flops": 0.0, "bytes": 0.0, "launches": 0,
                                                      "stages": []})
            k["ms"] += st["ms"]
            k["flops"] += st["flops"]
            k["bytes"] += st["bytes"]
            k["launches"] += st["launches"]
            k["stages"].append(stage)
        dom_name, dom = max(per_kernel.items(), key=lambda kv: kv[1]["ms"])
        t_launch = dom["ms"] / 1000.0 / dom["launches"]
        gemm_like = dom["flops"] > 0
        if gemm_like:
            achieved = dom["flops"] / dom["launches"] / t_launch / 1e12
            peak, peak_note = mfma_peak_for(dom_name)
            roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 4), "peak_basis": peak_note}
        else:
            achieved = dom["bytes"] / dom["launches"] / t_launch / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4)}
        traffic, traffic_src = None, None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                pmc = json.load(f)
            k = pmc_lookup(pmc.get("kernels", {}), dom_name)
            if "traffic_bytes" in k:
                traffic = round(k["traffic_bytes"])
                traffic_src = {"source": f"profiles/{pmc['tag']}_pmc_summary.json", "unit": "bytes per launch",
                               "fetch_bytes": round(k["fetch_bytes"]), "write_bytes": round(k["write_bytes"])}
        roof.update({"traffic": traffic, "traffic_detail": traffic_src, "kernel": dom_name, "stages": dom["stages"],
                     "avg_launch_ms": round(1000 * t_launch, 4), "launches": dom["launches"],
                     "algorithmic_per_launch": dom["flops"] / dom["launches"] if gemm_like
                     else dom["bytes"] / dom["launches"]})
        result["roofline"] = roof
        tot_ms = sum(v["ms"] for v in per_kernel.values())
        tot_fl = sum(v["flops"] for v in per_kernel.values())
        result["whole_encode"] = {"device_ms_per_step": round(tot_ms / args.steps, 3),
                                  "tflops": round(tot_fl / (tot_ms / 1000) / 1e12, 2),
                                  "frac_fp32_peak": round(tot_fl / (tot_ms / 1000) / 1e12 / FP32_PEAK_TFLOPS, 4)}
        result["stages_ms_per_step"] = {s: round(v["ms"] / args.steps, 3) for s, v in prof.items()}
        result["north_star"] = north_star_groups(prof, args.steps, pmc_path)
    if rank == 0 and world == 1 and args.cpu_baseline_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, args.cpu_threads, args.seconds)
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
