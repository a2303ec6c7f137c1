"""Throughput of the Mimi encode hot path on MI355X: audio-seconds encoded per wall-second (K = 8, 24 kHz).

    python bench.py [--gpus N --steps K --warmup W --batch B --seconds S --workload batch|yodas2|mls [--bpe]]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

``--gpus N`` without torchrun's environment launches N ranks itself (``torch.distributed.run`` as a child
process, started before anything touches the GPU) and exits with its status; under torchrun, WORLD_SIZE must
equal ``--gpus``.

Workloads (one "step" each; per-GPU work is fixed as N grows: weak scaling):

* ``batch`` (default, BASELINE.json configs[1], LibriTTS-R-style): one ``mimi_encode`` of B = 32 synthetic
  10 s / 24 kHz clips already resident in HBM (``--batch 64`` = configs[2], Emilia).
* ``yodas2`` (configs[3]): one ``MimiEncoder.encode_audio_batch`` of B mixed-length clips U[1.5, 20] s from
  host memory -- feature extraction (pad to longest), host->device, encode, codes back to host, trim -- the
  reference YODAS2 caller's batch path (``yodas2-mimi/process_shard.py:494-525``).  Clips are this rank's
  round-robin share (``mimi_hip.sharding``).  value counts unpadded audio seconds.
* ``mls`` (configs[4], encode part): B utterances U[10, 20] s, each encoded alone at its own length (the codes
  of ``MimiEncoder.encode_audio_chunk`` per utterance, as ``mls-en-mimi-pretrain/process_shard.py:302-307`` calls it,
  bit for bit) through the ADDED ``MimiEncoder.encode_audio_chunks`` (ragged batches of 32 -- a caller change),
  host->device and back included.

Printed beside the headline (``batch`` workload at B = 32 x 10 s): ``k32`` = the same batch at K = 32 (the drop-in
default: every script builds ``MimiEncoder("kyutai/mimi")`` and encodes all 32 levels), ``b1_k8`` = one 10 s clip per
encode, resident, K = 8, and ``per_utterance_k32`` = the UNCHANGED per-utterance loop -- ``encode_audio_chunk(a,
24000)`` once per U[10, 20] s utterance from host memory at the default K = 32, the way
``librispeech-mimi/process_librispeech_dev-test.py:136-141`` and ``mls-en-mimi-pretrain/process_shard.py:302-307``
run (every length differs, so no hipGraph replay).

Weights: the seeded synthetic kyutai/mimi-shaped checkpoint (random init; throughput does not depend on
values).  The timed region is bracketed by barrier + synchronize; the max over ranks is reported.  Rank 0
prints ONE JSON line.

roofline: per-kernel device time from HIP events recorded by the engine on its launch stream during the timed
steps, aggregated per kernel symbol; the dominant kernel's algorithmic FLOPs / its time vs the MFMA peak of the
arithmetic it runs on (see ``mfma_peak_for``).  cpu_baseline: the oracle (torch CPU restatement of
MimiModel.encode) on a bounded sample of the same workload.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "tokenize-audio_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: fp32 MFMA/vector peak
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E spec
HBM_ACHIEVABLE_GBS = 6300.0  # MI355X_MICROARCH.md §HBM: 8 TB/s spec, ~6.3 TB/s achievable
BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak
F16X3_PEAK_TFLOPS = BF16_PEAK_TFLOPS / 3  # fp32-accurate products as 3 fp16 products
DTYPE_LABEL = {
    "f16x3": "f16x3 (fp32-emulating: 2 fp16 planes per operand, 3 products, fp32 accumulate; RVQ distances fp32)",
    "bf16x6": "bf16x6 (fp32-emulating: 3 bf16 planes, 6 products, fp32 accumulate; RVQ distances fp32)",
    "bf16x3": "bf16x3 (2 bf16 planes, 3 products, fp32 accumulate; RVQ distances fp32)",
    "f32": "f32 (fp32 MFMA throughout)",
}


def mfma_peak_for(kernel: str):
    """Peak that bounds a GEMM kernel, in fp32-equivalent TFLOP/s of the algorithmic (fp32) FLOPs it does.

    fp32 kernels run on v_mfma_f32_32x32x2_f32: 157.3 TF.  The split kernels compute the same fp32 GEMM as P
    16-bit products per fp32 multiply-add (NS = 3 bf16 planes -> 6 products, NS = 2 -> 3) on the dense
    bf16/fp16 MFMA, so their ceiling is 2.5 PF / P (416.7 TF for bf16x6, 833.3 TF for f16x3 / bf16x3)."""
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
    ap.add_argument("--workload", choices=("batch", "yodas2", "mls"), default="batch")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=10.0, help="clip length of the 'batch' workload")
    ap.add_argument("--num-quantizers", type=int, default=8)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0,
                    help="wall budget of the CPU-baseline sample (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: this process's CPU affinity, capped by OMP_NUM_THREADS)")
    ap.add_argument("--concurrency", type=int, default=1,
                    help="host-fed workloads: engines MimiEncoder's pipeline alternates between (batches overlap)")
    ap.add_argument("--bpe", action="store_true",
                    help="mls workload: after the timed encodes, train codec-BPE (GPU merge loop) over the emitted "
                         "codes on rank 0, timed separately (configs[4])")
    ap.add_argument("--bpe-vocab-extra", type=int, default=2000, help="--bpe: learned tokens beyond the codes")
    ap.add_argument("--no-profile", action="store_true", help="do not record per-stage events")
    ap.add_argument("--no-f32-mode", action="store_true", help="skip the fp32-MFMA comparison run")
    ap.add_argument("--precision", default=None, help="GEMM precision mode (default: the engine's)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--ln-fused", type=int, default=None,
                    help="A/B: 0 = LayerNorm launches, 1 = LayerNorm prologue in small-grid q/k/v / fc1 (default)")
    ap.add_argument("--stage0-fused", type=int, default=None,
                    help="kernel variant A/B: 0 = stage-0 block + down conv 0 as two kernels, 1 = fused (default)")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="engine option (mimi_set_option) for A/B runs, e.g. rvq_form=1; repeatable")
    ap.add_argument("--dump-sequence", default=None,
                    help="write the engine's per-encode (stage, kernel) launch sequence here (PMC stage keys)")
    ap.add_argument("--pmc-pass", action="store_true",
                    help="counter pass: the timed steps only (no PCIe / f32 / B=64 extras, no CPU baseline)")
    return ap.parse_args()


def self_launch(args) -> int:
    """--gpus N > 1 outside torchrun: run torch.distributed.run as a child (this process never touched the
    GPU) and return its exit status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cgroup_cpu_quota():
    """CPUs granted by the cgroup's CPU quota (v2 cpu.max / v1 cfs_quota_us), or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_threads(requested: int):
    """(threads, note): the CPUs this process may use -- its affinity, capped by a cgroup CPU quota and by the
    pool's per-GPU CPU share when one is set (OMP_NUM_THREADS on the GPU box: 16 CPUs per GPU; running more threads
    there would take other jobs' cores) -- and the reason for the number."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpu_quota()
    if requested > 0:
        return requested, f"{requested} threads requested (affinity {aff}, cgroup quota {quota or 'none'})"
    n, why = aff, f"all {aff} CPUs of the process affinity"
    if quota is not None and int(quota) < n:
        n, why = max(1, int(quota)), f"cgroup CPU quota {quota:g} CPUs (affinity {aff})"
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and 0 < int(share) < n:
        n, why = int(share), (f"the pool's per-GPU CPU share OMP_NUM_THREADS={share} (process affinity {aff}, "
                              f"cgroup quota {'%g' % quota if quota else 'none'})")
    return max(1, n), why


def cpu_baseline(seconds_budget: float, threads_why, clip_s: float, batch: int):
    """The oracle on the host cores, same metric: whole clips at batch 1 (config 1 of BASELINE.json) and at the
    GPU workload's batch, each on about half the budget.  ``value`` is the rate at the GPU's batch size."""
    import torch

    from mimi_hip import synthetic
    from oracle import mimi_ref
    threads, why = threads_why
    torch.set_num_threads(threads)
    sd = synthetic.make_state_dict(seed=0, num_quantizers=8)
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    n = int(clip_s * 24000)
    rates = {}
    for b in sorted({1, batch}):
        clips = torch.from_numpy(synthetic.clip_batch(b, n, seed=0))[:, None]
        mimi_ref.encode(clips[:1], sdt, 8)  # warm
        done, t0 = 0, time.perf_counter()
        while True:
            mimi_ref.encode(clips, sdt, 8)
            done += 1
            el = time.perf_counter() - t0
            if el >= seconds_budget / 2 or done >= 200:
                break
        rates[b] = (done * b * clip_s / el, done)
    try:
        cpu_model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        cpu_model = "unknown"
    sample = "; ".join(f"batch {b}: {d} encode(s) of {b} x {clip_s:g} s = {r:.1f} audio-s/s"
                       for b, (r, d) in rates.items())
    return {"value": round(rates[batch][0], 3), "unit": "audio-sec/sec", "cores": threads, "kind": "port",
            "sample": f"{sample}; K=8, oracle/mimi_ref.py (torch {torch.__version__} CPU, {threads} threads: {why}; "
                      f"{cpu_model})",
            "batch1_value": round(rates[1][0], 3)}


def pmc_lookup(pmc_kernels, name):
    """PMC summary entry of a kernel symbol: the summary keys drop rocprof's 'void ' prefix and, for
    non-template kernels, the parameter list that the engine's names keep."""
    if name in pmc_kernels:
        return pmc_kernels[name]
    bare = name[5:] if name.startswith("void ") else name
    if "(" in bare and not bare.endswith(">"):
        bare = bare[:bare.index("(")]
    return pmc_kernels.get(bare, {})


def pmc_stage(pmc, stage, kernel):
    """PMC bytes of a stage: the stage-keyed entry (tools/summarize_profile.py aligns the counter rows to the engine's
    launch sequence), else the kernel-symbol entry.  Returns (bytes per launch or None, the measured kernel,
    whether that kernel is this run's)."""
    bare = lambda k: (k or "").replace("void ", "", 1).split("(")[0].strip()  # noqa: E731
    st = pmc.get("stages", {}).get(stage.split("#")[0])
    if st and "traffic_bytes" in st:
        return st["traffic_bytes"], st.get("kernel"), bare(st.get("kernel")) == bare(kernel)
    k = pmc_lookup(pmc.get("kernels", {}), kernel)
    if "traffic_bytes" in k:
        return k["traffic_bytes"], kernel, True
    return None, None, False


def load_pmc(pmc_path, workload):
    """profiles/pmc_summary.json if its PMC passes ran this workload (per-launch bytes are workload-specific: the
    B = 1 or ragged launches of a stage move different bytes from the B = 32 ones), else ({}, why)."""
    if not os.path.exists(pmc_path):
        return {}, "no profiles/pmc_summary.json"
    with open(pmc_path) as f:
        pmc = json.load(f)
    if pmc.get("workload") != workload:
        return {}, f"PMC passes ran workload {pmc.get('workload')}, not this one ({workload})"
    return pmc, None


def north_star_groups(prof, steps, pmc, pmc_note=None):
    """BASELINE.json's reporting asks: HBM GB/s and TFLOP/s of the SEANet conv stack, MFMA utilisation of the
    transformer.  Device ms and algorithmic FLOPs from the engine's events; HBM bytes = the PMC passes'
    FETCH_SIZE x 2 + WRITE_SIZE per launch of each STAGE (profiles/pmc_summary.json, keyed by stage; by kernel
    symbol as a fallback) x that stage's launches."""
    base = lambda s: s.split("#")[0]  # noqa: E731  ("fc2#2": the same stage on a second kernel symbol)
    groups = {
        "conv_stack": [s for s in prof if base(s).startswith(("res", "down_s", "final"))],
        "transformer": [s for s in prof if base(s) in ("layernorm", "qkv", "attention", "qkv_attention", "o_proj", "o_proj_ln", "fc1", "fc2")],
        "quantizer": [s for s in prof if base(s) in ("downsample", "input_proj", "rvq")],
    }
    out = {}
    for g, stages in groups.items():
        if not stages:
            continue
        ms = sum(prof[s]["ms"] for s in stages) / steps
        fl = sum(prof[s]["flops"] for s in stages) / steps
        looked = [pmc_stage(pmc, s, prof[s]["kernel"]) for s in stages]
        d = {"stages": stages, "ms_per_step": round(ms, 3), "tflops": round(fl / (ms / 1e3) / 1e12, 1),
             "frac_f16x3_peak": round(fl / (ms / 1e3) / 1e12 / F16X3_PEAK_TFLOPS, 4)}
        missing = [s for s, (b, _, _) in zip(stages, looked) if b is None]
        stale = [s for s, (b, _, same) in zip(stages, looked) if b is not None and not same]
        if stale:
            d["hbm_measured_on_other_kernel"] = stale
        if missing:
            d["hbm_unmeasured_stages"] = missing
            if pmc_note:
                d["hbm_unmeasured_why"] = pmc_note
        else:
            by = sum(b * prof[s]["launches"] / steps for (b, _, _), s in zip(looked, stages))
            d.update({"hbm_bytes_per_step": round(by), "hbm_GBps": round(by / (ms / 1e3) / 1e9, 1),
                      "frac_hbm_peak": round(by / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)})
        if g == "conv_stack":
            # the north star's HBM-bound layers (k = 1 residual convs of stages 2-3, and the fused stage-1 block that
            # holds stage 1's), each on its own: PMC bytes per launch / its event time, against the 8 TB/s spec and
            # the ~6.3 TB/s MI355X_MICROARCH.md reports achievable
            per = {}
            for s, (b, _, _) in zip(stages, looked):
                if base(s) not in ("res1_s2", "res1_s3", "res_s1") or b is None:
                    continue
                t = prof[s]["ms"] / 1e3 / prof[s]["launches"]
                per[base(s)] = {"kernel": prof[s]["kernel"], "hbm_bytes_per_launch": round(b),
                                "ms_per_launch": round(1e3 * t, 4), "hbm_GBps": round(b / t / 1e9, 1),
                                "frac_hbm_peak": round(b / t / 1e9 / HBM_PEAK_GBS, 4),
                                "frac_hbm_achievable": round(b / t / 1e9 / HBM_ACHIEVABLE_GBS, 4)}
            if per:
                d["hbm_bound_layers"] = per
        out[g] = d
    return out


def roofline_from_profile(prof, steps, pmc, pmc_note=None, lead=None):
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
    timing = "events around every stage of the profiled pass"
    if lead and len(dom["stages"]) == 1 and dom["stages"][0] in lead and lead[dom["stages"][0]]["kernel"] == dom_name:
        # the dominant kernel is each encode's first stage: its duration as the timed region's own events saw it
        ld = lead[dom["stages"][0]]
        t_launch = ld["ms"] / 1000.0 / ld["launches"]
        timing = f"events around it in the timed region ({ld['launches']} launches)"
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
    traffic, traffic_src = None, pmc_note
    if pmc:
        # the dominant kernel's stages, launch-weighted
        looked = [(pmc_stage(pmc, st, dom_name), prof[st]["launches"]) for st in dom["stages"]]
        if all(b is not None for (b, _, _), _ in looked):
            n = sum(l for _, l in looked)
            traffic = round(sum(b * l for (b, _, _), l in looked) / n)
            traffic_src = {"source": f"profiles/{pmc['tag']}_pmc_summary.json", "unit": "bytes per launch",
                           "keyed_by": "stage" if all(st.split("#")[0] in pmc.get("stages", {}) for st in dom["stages"])
                           else "kernel", "measured_kernel_is_this_build": all(same for (_, _, same), _ in looked)}
            ks = [pmc.get("stages", {}).get(st.split("#")[0]) or pmc_lookup(pmc.get("kernels", {}), dom_name)
                  for st in dom["stages"]]
            if all("fetch_bytes" in k and "write_bytes" in k for k in ks):
                traffic_src["fetch_bytes"] = round(sum(k["fetch_bytes"] for k in ks) / len(ks))
                traffic_src["write_bytes"] = round(sum(k["write_bytes"] for k in ks) / len(ks))
    roof.update({"traffic": traffic, "traffic_detail": traffic_src, "kernel": dom_name, "stages": dom["stages"],
                 "avg_launch_ms": round(1000 * t_launch, 4), "launches": dom["launches"], "timing": timing,
                 "algorithmic_per_launch": dom["flops"] / dom["launches"] if gemm_like
                 else dom["bytes"] / dom["launches"]})
    tot_ms = sum(v["ms"] for v in per_kernel.values())
    tot_fl = sum(v["flops"] for v in per_kernel.values())
    whole = {"device_ms_per_step": round(tot_ms / steps, 3),
             "tflops_fp32_equivalent": round(tot_fl / (tot_ms / 1000) / 1e12, 2),
             "frac_f16x3_peak": round(tot_fl / (tot_ms / 1000) / 1e12 / F16X3_PEAK_TFLOPS, 4)}
    # the other heavy kernels against their own ceilings (the dominant one is `roof`): by device time per step
    top = []
    for name, k in sorted(per_kernel.items(), key=lambda kv: -kv[1]["ms"])[:8]:
        t = k["ms"] / 1000.0 / k["launches"]
        e = {"kernel": name, "stages": k["stages"], "ms_per_step": round(k["ms"] / steps, 3),
             "avg_launch_ms": round(1000 * t, 4)}
        if k["flops"] > 0:
            pk, _ = mfma_peak_for(name)
            a = k["flops"] / k["launches"] / t / 1e12
            e.update({"achieved_tflops": round(a, 1), "peak_tflops": round(pk, 1), "frac": round(a / pk, 4)})
        else:
            a = k["bytes"] / k["launches"] / t / 1e9
            e.update({"achieved_GBps": round(a, 1), "frac_hbm_peak": round(a / HBM_PEAK_GBS, 4)})
        top.append(e)
    whole["top_kernels"] = top
    return roof, whole


class Workload:
    """One step of the selected workload on this rank; ``audio_seconds`` = unpadded audio per step."""

    def __init__(self, args, model, dev, world, rank):
        import numpy as np
        import torch

        from mimi_hip import synthetic
        from mimi_hip.config import encoded_length
        from mimi_hip.encoder import MimiEncoder
        from mimi_hip.sharding import make_batches, shard_indices
        self.kind = args.workload
        K = args.num_quantizers
        B = args.batch
        if self.kind == "batch":
            L = int(round(args.seconds * 24000))
            # this rank's utterances: a distinct seeded slice of the shard (round-robin i -> rank i % N)
            self.audio = torch.from_numpy(synthetic.clip_batch(B, L, seed=1000 + rank)).to(dev)
            self.codes = torch.empty((B, K, encoded_length(L)), dtype=torch.int32, device=dev)
            self.codes2 = torch.empty_like(self.codes)
            self.audio_seconds = B * args.seconds
            self.host_audio = self.audio.cpu().pin_memory()
            self.steps_clips = None
            self.pending = None

            def step():
                # each step is one whole encode, waited (its f16x3 overflow check) one step behind: the next encode is
                # enqueued before the host waits for this one, so the GPU never idles on the host's turnaround
                # (the outputs alternate so a fallback re-run of step i cannot land on step i + 1's codes)
                out = self.codes2 if self.pending is not None and self.pending.out is self.codes else self.codes
                t = model.encode_async(self.audio, K, out=out)
                if self.pending is not None:
                    self.pending.wait()
                self.pending = t
            self.step = step
            self.desc = (f"LibriTTS-R-style batch encode (configs[{1 if B <= 32 else 2}]): batch={B} x "
                         f"{args.seconds:g} s @ 24 kHz resident in HBM, K={K} codebooks, 1 encode per step per GPU")
            return
        enc = MimiEncoder(device=dev, model=model, num_quantizers=K, concurrency=max(1, args.concurrency))
        lo, hi = (1.5, 20.0) if self.kind == "yodas2" else (10.0, 20.0)
        n_steps = args.warmup + args.steps
        # the whole shard's utterance list; this rank takes i % world == rank (sharding.py), in batches of B
        n_total = world * B * n_steps
        lengths = synthetic.random_lengths(n_total, lo, hi, seed=77)
        mine = shard_indices(n_total, world, rank)
        batches = make_batches(mine, B)
        self.clips = [[synthetic.speech_like(lengths[i], 77, i) for i in b] for b in batches[:n_steps]]
        self.step_seconds = [sum(len(a) for a in c) / 24000.0 for c in self.clips]
        self.i = 0

        if self.kind == "yodas2":
            def run(first, count):  # the steps' batches through the pipelined iterator (host staging overlapped)
                for _ in enc.encode_batches(self.clips[first:first + count], 24000):
                    pass
            self.desc = (f"YODAS2-style shard (configs[3]): batches of {B} mixed-length clips U[{lo:g}, {hi:g}] s "
                         f"from host memory through MimiEncoder.encode_batches (= encode_audio_batch per batch: "
                         f"pad-to-longest codes, run as a ragged encode at min(Lmax, 1920 ceil(L/1920)) per item; host "
                         f"staging, H2D, encode, D2H, trim -- the next batch staged under the current encode), K={K}, "
                         f"utterance round-robin over {world} GPU(s)")
        else:
            self.emitted = []  # codes of the timed steps, for --bpe

            def run(first, count):  # every utterance of the steps, each encoded alone (ragged batches of 32)
                out = enc.encode_audio_chunks([a for c in self.clips[first:first + count] for a in c], 24000)
                if first >= args.warmup:
                    self.emitted.extend(out)
            self.desc = (f"MLS-style stream (configs[4], encode part): {B} utterances U[{lo:g}, {hi:g}] s per step, "
                         f"each encoded alone at its own length (encode_audio_chunk semantics, bit for bit; H2D + D2H "
                         f"included) through MimiEncoder.encode_audio_chunks = ragged batches of 32 by length, "
                         f"pipelined, K={K}, utterance round-robin over {world} GPU(s)" +
                         ("; then codec-BPE training over the timed steps' codes on rank 0 (`bpe`, `pipeline_value`)"
                          if args.bpe else ""))
        self.run = run

        def step():
            run(self.i, 1)
            self.i += 1
        self.step = step
        self._np = np

    def run_steps(self, first, count):
        """count steps starting at step index first (host-resident workloads pipeline across them)"""
        if self.kind == "batch":
            for _ in range(count):
                self.step()
            if self.pending is not None:  # the last step's wait
                self.pending.wait()
                self.pending = None
        else:
            self.run(first, count)

    def timed_seconds(self, first, count):
        if self.kind == "batch":
            return self.audio_seconds * count
        return sum(self.step_seconds[first:first + count])


def timed_max(fn, n, barrier, reduce_max):
    """n calls of fn between a barrier + synchronize on both sides; the elapsed seconds are the MAX over ranks (the
    headline's method), so a rate world x work / elapsed is the whole job's."""
    import torch
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    barrier()
    return reduce_max(el)


def s8d_rate(model, wl, dev, K, n, barrier, reduce_max):
    """SURVEY.md §8(d)'s metric as defined there: wall clock from the H2D copy of the f32 input through the D2H copy of
    the int codes, steady state.  Host batches (pinned) go up on a copy stream while the previous batch encodes, and
    codes come back on the copy stream behind each encode: double-buffered, as a shard driver would run it."""
    import torch
    B, L = wl.host_audio.shape
    T = wl.codes.shape[2]
    copy = torch.cuda.Stream(device=dev)
    comp = torch.cuda.current_stream(dev)
    din = [torch.empty((B, L), dtype=torch.float32, device=dev) for _ in range(2)]
    dout = [torch.empty((B, K, T), dtype=torch.int32, device=dev) for _ in range(2)]
    hout = [torch.empty((B, K, T), dtype=torch.int32).pin_memory() for _ in range(2)]
    up = [torch.cuda.Event() for _ in range(2)]
    done = [torch.cuda.Event() for _ in range(2)]
    down = [torch.cuda.Event() for _ in range(2)]

    def run(count):
        with torch.cuda.stream(copy):
            din[0].copy_(wl.host_audio, non_blocking=True)
            up[0].record(copy)
        for i in range(count):
            j = i & 1
            if i + 1 < count:  # the next batch's H2D under this encode (its buffer's last encode has finished)
                with torch.cuda.stream(copy):
                    if i >= 1:
                        copy.wait_event(done[j ^ 1])
                    din[j ^ 1].copy_(wl.host_audio, non_blocking=True)
                    up[j ^ 1].record(copy)
            comp.wait_event(up[j])
            if i >= 2:
                comp.wait_event(down[j])  # dout[j]'s previous codes are on the host
            model.encode_int32(din[j], K, out=dout[j])
            done[j].record(comp)
            with torch.cuda.stream(copy):
                copy.wait_event(done[j])
                hout[j].copy_(dout[j], non_blocking=True)
                down[j].record(copy)
        for e in down:
            e.synchronize()

    run(2)
    el = timed_max(lambda: run(n), 1, barrier, reduce_max)
    return el


def drop_in_rates(args, model, wl, dev, world, barrier, reduce_max):
    """The rates the unmodified shard scripts get (VERDICT r3 "missing" 3): K = 32 on the headline batch, batch 1
    resident at K = 8, and the per-utterance loop through MimiEncoder at its default K = 32 (host in / out).  Each
    timed region: barrier + synchronize on both sides, elapsed = max over ranks (timed_max)."""
    import torch

    from mimi_hip import synthetic
    from mimi_hip.config import encoded_length
    from mimi_hip.encoder import MimiEncoder
    out = {}
    # K = 32 on the headline batch
    c32 = torch.empty((wl.audio.shape[0], 32, wl.codes.shape[2]), dtype=torch.int32, device=dev)
    for _ in range(2):
        model.encode_int32(wl.audio, 32, out=c32)
    n = max(1, min(args.steps, 10))
    el = timed_max(lambda: model.encode_int32(wl.audio, 32, out=c32), n, barrier, reduce_max)
    out["k32"] = {"value": round(world * n * wl.audio_seconds / el, 2), "ms_per_step": round(1000 * el / n, 3),
                  "steps": n, "workload": f"the headline batch ({wl.audio.shape[0]} x {args.seconds:g} s resident) at "
                                          f"K=32, the drop-in default (MimiEncoder encodes all 32 levels)"}
    del c32
    # batch 1, resident, K = 8 (hipGraph replays after the 2nd encode of the shape)
    L = 240000
    a1 = torch.from_numpy(synthetic.clip_batch(1, L, seed=3000)).to(dev)
    c1 = torch.empty((1, 8, encoded_length(L)), dtype=torch.int32, device=dev)
    for _ in range(3):
        model.encode_int32(a1, 8, out=c1)
    n = 40
    el = timed_max(lambda: model.encode_int32(a1, 8, out=c1), n, barrier, reduce_max)
    out["b1_k8"] = {"value": round(world * n * 10.0 / el, 2), "ms_per_encode": round(1000 * el / n, 3), "encodes": n,
                    "workload": "batch 1 x 10 s resident in HBM, K=8 (configs[0]'s batch size), each encode waited "
                                "before the next is enqueued"}
    c1b = torch.empty_like(c1)
    held = [None]

    def b1_pipelined():
        t = model.encode_async(a1, 8, out=c1b if held[0] is not None and held[0].out is c1 else c1)
        if held[0] is not None:
            held[0].wait()
        held[0] = t

    def b1_run(count):
        for _ in range(count):
            b1_pipelined()
        held[0].wait()
        held[0] = None
    b1_run(3)
    el = timed_max(lambda: b1_run(n), 1, barrier, reduce_max)
    out["b1_k8_pipelined"] = {"value": round(world * n * 10.0 / el, 2), "ms_per_encode": round(1000 * el / n, 3),
                              "encodes": n,
                              "workload": "the same batch-1 encodes with the next one enqueued before the host waits "
                                          "for the previous (encode_async, one behind): device time per encode without "
                                          "the host's turnaround between them"}
    # the unchanged per-utterance loop: encode_audio_chunk per utterance, default K (32), host numpy in / out
    enc = MimiEncoder(device=dev, model=model)
    lens = synthetic.random_lengths(24, 10.0, 20.0, seed=99)
    utts = [synthetic.speech_like(n_, 99, i) for i, n_ in enumerate(lens)]
    for a in utts[:2]:
        enc.encode_audio_chunk(a, 24000)
    el = timed_max(lambda: [enc.encode_audio_chunk(a, 24000) for a in utts], 1, barrier, reduce_max)
    out["per_utterance_k32"] = {
        "value": round(world * sum(lens) / 24000.0 / el, 2), "utterances": len(utts),
        "ms_per_utterance": round(1000 * el / len(utts), 3),
        "workload": "the unmodified per-utterance loop: MimiEncoder(...).encode_audio_chunk(a, 24000) once per "
                    "U[10, 20] s utterance from host memory (numpy in, int64 [32, T] numpy out), default K=32, every "
                    "length distinct (eager launches) -- librispeech-mimi/process_librispeech_dev-test.py:136-141, "
                    "mls-en-mimi-pretrain/process_shard.py:302-307"}
    return out


def train_bpe_over_codes(args, wl, dist, rank, world, device, encode_s):
    """configs[4]'s second half: codec-BPE over the codes this run emitted (codec-bpe/train_bpe_recipe.txt:18-28:
    30 s chunks, max_token_codebook_ngrams 2), on rank 0 after the ranks' codes are gathered (host objects).
    Reports the training time and the pipeline rate = timed audio-seconds / (encode + train)."""
    from mimi_hip import bpe
    codes = wl.emitted
    if dist is not None:
        parts = [None] * world if rank == 0 else None
        dist.gather_object(codes, parts, dst=0)
        codes = [c for p in parts for c in p] if rank == 0 else []
    out = {}
    if rank == 0:
        K = args.num_quantizers
        tr = bpe.Trainer(K, 2048, codec_framerate=12.5, chunk_size_secs=30,
                         vocab_size=K * 2048 + 1 + args.bpe_vocab_extra, min_frequency=2, pad_token="<pad>",
                         max_token_codebook_ngrams=2, device=device)
        try:  # the one-time transformers import (lazy module) is process start-up, not training
            from transformers import PreTrainedTokenizerFast  # noqa: F401
        except Exception:
            pass
        t0 = time.perf_counter()
        tr.train_codes(codes)
        bpe_s = time.perf_counter() - t0
        audio_s = wl.timed_seconds(args.warmup, args.steps) * world
        out = {"bpe": {"utterances": len(codes), "merges": len(tr.last_merges), "train_s": round(bpe_s, 3),
                       "stats": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in tr.last_stats.items()}},
               "pipeline_value": round(audio_s / (encode_s + bpe_s), 2)}
    if dist is not None:
        dist.barrier()
    return out


def rank_map(dist, backend, world, rank, local, dev, audio_s, elapsed_s):
    """Every rank's device as the driver sees it, so an N-GPU line can show that it ran on N distinct GPUs:
    [{rank, local_rank, host, device, pci_bus, name, audio_s, elapsed_s}] in rank order, plus the process group's own
    world size.  Under nccl (RCCL) two ranks on one PCI device of one host are an error -- a line from ranks sharing a
    GPU must not pass for an N-GPU measurement; the gloo rehearsal (MIMI_BENCH_DIST_BACKEND=gloo, ranks sharing the
    box's GPUs) is allowed and labelled `sharing`.  (One GPU per job is the reference's unit of work:
    yodas2-mimi/submit/job_template.sh:10.)"""
    import socket

    import torch
    p = torch.cuda.get_device_properties(dev)
    bus = "{:04x}:{:02x}:{:02x}".format(getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", -1) & 0xFF,
                                        getattr(p, "pci_device_id", -1) & 0xFF)
    mine = {"rank": rank, "local_rank": local, "host": socket.gethostname(), "device": dev.index, "pci_bus": bus,
            "name": p.name, "audio_s": round(audio_s, 3), "elapsed_s": round(elapsed_s, 6)}
    if dist is None:
        ranks = [mine]
        pg_world = 1
    else:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        pg_world = dist.get_world_size()
    return ranks, check_rank_places(ranks, backend if dist is not None else "none", pg_world, world)


def check_rank_places(ranks, backend, pg_world, world):
    """The `dist` object of the line from the gathered rank map; SystemExit when the map contradicts an N-GPU claim
    (a process group of another size, or two nccl ranks on one device of one host)."""
    places = {(r["host"], r["pci_bus"]) for r in ranks}
    sharing = len(places) < len(ranks)
    if pg_world != world or len(ranks) != world:
        sys.exit(f"bench.py: the process group has {pg_world} ranks ({len(ranks)} reported), WORLD_SIZE says {world}")
    if sharing and backend == "nccl":
        sys.exit("bench.py: ranks share a GPU under nccl: " +
                 ", ".join(f"rank {r['rank']} -> {r['host']} {r['pci_bus']}" for r in ranks))
    return {"backend": backend, "world_size": pg_world, "distinct_devices": len(places), "sharing": sharing}


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(self_launch(args))
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    dist = None
    # one GPU per rank (LOCAL_RANK); MIMI_BENCH_DIST_BACKEND=gloo rehearses the N-rank path on a box with fewer
    # GPUs than ranks (ranks share cuda:(LOCAL_RANK mod devices); barrier and reductions go over gloo on the host)
    backend = os.environ.get("MIMI_BENCH_DIST_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        sys.exit(f"bench.py: MIMI_BENCH_DIST_BACKEND={backend}: expected nccl or gloo")
    ndev = torch.cuda.device_count()
    if ndev == 0:
        sys.exit("bench.py: no HIP device")
    if backend == "nccl" and world > ndev:
        sys.exit(f"bench.py: {world} ranks but {ndev} GPU(s) (MIMI_BENCH_DIST_BACKEND=gloo shares GPUs)")
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    red_dev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from mimi_hip import synthetic
    from mimi_hip.model import MimiHipModel

    K = args.num_quantizers
    # all 32 codebooks, as kyutai/mimi has (the K = 32 lines below; a K-level encode reads only the first K)
    model = MimiHipModel(synthetic.make_state_dict(seed=0), device=dev)
    if args.precision:
        model.set_precision(args.precision)
    if args.stage0_fused is not None:
        model.set_option("stage0_fused", args.stage0_fused)
    if args.ln_fused is not None:
        model.set_option("ln_fused", args.ln_fused)
    for kv in args.option:
        k, v = kv.split("=", 1)
        model.set_option(k, int(v))
    wl = Workload(args, model, dev, world, rank)
    if model.precision == "f16x3":
        model.calibrate()  # (otherwise inside the first encode) -- before the trace marker
    # trace marker (a torch `spin_kernel`): rocprofv3 summaries keep the dispatches after it, i.e. drop the
    # f16x3 calibration encode (tools/summarize_profile.py)
    torch.cuda.synchronize()
    torch.cuda._sleep(100)
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    def reduce_max(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    wl.run_steps(0, args.warmup)
    torch.cuda.synchronize()
    profile = not args.no_profile
    # small batches are launch-bound and replay hipGraphs (engine.cpp graph_encode), which per-stage events
    # would switch off: their timed region runs without events and the stage profile comes from a separate pass;
    # so do the host-fed workloads (their device time per step, beside the wall time, shows what the host costs)
    profile_separately = profile and (args.batch <= 4 or wl.kind != "batch")
    # large uniform batches: the timed region carries the light profile (events around each encode's first stage --
    # the fused stage 0, the dominant kernel -- only); the per-stage table comes from a full pass right after
    lead_only = profile and not profile_separately
    if lead_only:
        model.profile_reset()
        model.set_profiling(2)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wl.run_steps(args.warmup, args.steps)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    audio_s = wl.timed_seconds(args.warmup, args.steps)
    if dist is not None:
        t = torch.tensor([elapsed, audio_s], dtype=torch.float64, device=red_dev)
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, audio_s = float(tmax.item()), float(t[1].item())
    ranks, dist_info = rank_map(dist, backend, world, rank, local, dev, wl.timed_seconds(args.warmup, args.steps),
                                t1 - t0)
    prof, lead = {}, {}
    if lead_only:
        model.set_profiling(False)
        lead = model.profile_read()
    if profile:
        model.profile_reset()
        model.set_profiling(True)
        n_emitted = len(getattr(wl, "emitted", []))
        wl.run_steps(args.warmup, args.steps)
        torch.cuda.synchronize()
        if hasattr(wl, "emitted"):
            del wl.emitted[n_emitted:]  # (the profiled pass re-encodes the timed steps: keep their codes once)
        model.set_profiling(False)
        prof = model.profile_read()
        if args.dump_sequence and rank == 0:
            with open(args.dump_sequence, "w") as f:
                json.dump(model.profile_sequence(), f)

    value = audio_s / elapsed
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
        "dtype": DTYPE_LABEL.get(model.precision, model.precision),
        "data": "synthetic (seeded speech-like 24 kHz clips; seeded random-init kyutai/mimi-shaped weights)",
        "config": {"workload": wl.desc, "global_batch": world * args.batch,
                   "clip_seconds": args.seconds if wl.kind == "batch" else "mixed",
                   "num_quantizers": K, "parallelism": f"utterance round-robin x{world} (no collective)",
                   "gemm_precision": model.precision},
        "ranks": ranks,
        "dist": dist_info,
    }
    if model.precision == "f16x3":
        # fixed activation scales on these weights: overflow fallbacks taken, and the tightest tensor's headroom
        # (2^15 / (scale x max|x|) of the last encode; < 1 = an overflow)
        sc = {k: v for k, v in model.act_scales().items() if v[1] > 0}
        tight = min(sc.items(), key=lambda kv: kv[1][2]) if sc else None
        result["f16x3"] = {"f16_reruns": model.f16_reruns,
                           "min_headroom": round(tight[1][2], 2) if tight else None,
                           "min_headroom_tensor": tight[0] if tight else None}
    if wl.kind == "batch" and not args.pmc_pass:
        # SURVEY.md §8(d)'s metric as it defines the wall clock (H2D of the f32 input through D2H of the codes),
        # reported beside `value` (the HBM-resident rate, the contract's definition), never as it
        n = max(2, min(args.steps, 20))
        el = s8d_rate(model, wl, dev, K, n, barrier, reduce_max)
        result["s8d_h2d_to_d2h"] = {
            "value": round(world * n * wl.audio_seconds / el, 2), "ms_per_step": round(1000 * el / n, 3), "steps": n,
            "definition": "SURVEY.md 8(d): audio-s per wall-s from the H2D copy of each step's pinned f32 batch "
                          "through the D2H copy of its int32 codes, steady state, double-buffered (the next batch's "
                          "H2D and the previous codes' D2H on a copy stream under the encode)"}
        result["pcie_inclusive_value"] = result["s8d_h2d_to_d2h"]["value"]
        if not args.no_f32_mode and model.precision != "f32":
            # the same workload on true fp32 MFMA arithmetic, for comparison with the split-precision number
            prev = model.precision
            model.set_precision("f32")
            wl.step()
            torch.cuda.synchronize()
            n32 = max(1, min(args.steps, 5))
            tf0 = time.perf_counter()
            for _ in range(n32):
                wl.step()
            torch.cuda.synchronize()
            result["f32_mode_value"] = round(world * n32 * wl.audio_seconds / (time.perf_counter() - tf0), 2)
            model.set_precision(prev)
        if args.batch == 32 and args.seconds == 10.0:
            # BASELINE configs[2] (Emilia, batch 64 x 10 s), the largest single-GPU config, beside the headline
            import numpy as np  # noqa: F401
            from mimi_hip import synthetic
            from mimi_hip.config import encoded_length
            L = 240000
            a64 = torch.from_numpy(synthetic.clip_batch(64, L, seed=2000 + rank)).to(dev)
            c64 = torch.empty((64, K, encoded_length(L)), dtype=torch.int32, device=dev)
            for _ in range(2):
                model.encode_int32(a64, K, out=c64)
            n64 = max(1, min(args.steps, 10))
            el64 = timed_max(lambda: model.encode_int32(a64, K, out=c64), n64, barrier, reduce_max)
            result["configs2_b64"] = {"value": round(world * n64 * 64 * 10.0 / el64, 2),
                                      "ms_per_step": round(1000 * el64 / n64, 3), "steps": n64,
                                      "workload": "Emilia-style batch (configs[2]): 64 x 10 s resident in HBM, K=8"}
            del a64, c64
            result.update(drop_in_rates(args, model, wl, dev, world, barrier, reduce_max))
    if profile_separately:
        result["stages_source"] = "a separate profiled pass of the same steps (timed region: hipGraph replays)"
    elif lead_only:
        result["stages_source"] = ("a profiled pass of the same steps right after the timed region; the timed region "
                                   "carries events around each encode's first stage only (roofline.timing)")
    result["graph_replays"] = model.graph_replays
    if prof:
        pmc, pmc_note = load_pmc(os.path.join(ROOT, "profiles", "pmc_summary.json"),
                                 {"kind": wl.kind, "batch": args.batch, "seconds": args.seconds})
        roof, whole = roofline_from_profile(prof, args.steps, pmc, pmc_note, lead)
        result["roofline"] = roof
        result["whole_encode"] = whole
        stages, sflops = {}, {}
        for s_, v in prof.items():  # per stage, summed over the kernel symbols that run it
            stages[s_.split("#")[0]] = stages.get(s_.split("#")[0], 0.0) + v["ms"] / args.steps
            sflops[s_.split("#")[0]] = sflops.get(s_.split("#")[0], 0.0) + v["flops"] / args.steps
        result["stages_ms_per_step"] = {s_: round(v, 3) for s_, v in stages.items()}
        result["stages_tflops"] = {s_: round(sflops[s_] / (v / 1e3) / 1e12, 1) for s_, v in stages.items()
                                   if sflops[s_] > 0 and v > 0}
        result["north_star"] = north_star_groups(prof, args.steps, pmc, pmc_note)
    if args.bpe and wl.kind == "mls":
        result.update(train_bpe_over_codes(args, wl, dist, rank, world, dev.index, elapsed))
    if rank == 0 and world == 1 and args.cpu_baseline_seconds > 0 and not args.pmc_pass:
        cb_batch = args.batch if wl.kind == "batch" else 1
        result["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, cpu_threads(args.cpu_threads),
                                              args.seconds if wl.kind == "batch" else 15.0, cb_batch)
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
