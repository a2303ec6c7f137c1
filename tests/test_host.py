"""CPU: host logic (codes serialisation, wrapper semantics) and the C-ABI library surface."""
import ctypes
import json
import os
import re

import numpy as np
import pytest
import torch

from mimi_hip import synthetic
from mimi_hip.codes import chars_to_codes, codes_to_chars
from mimi_hip.config import encoded_length

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_codes_to_chars_golden():
    with open(os.path.join(ROOT, "tests", "golden", "codes_to_chars.json")) as f:
        g = json.load(f)
    codes = np.array(g["codes"], dtype=np.int64)
    s = codes_to_chars(codes, codebook_size=2048)
    assert [ord(c) for c in s] == g["chars_utf32"]
    assert chars_to_codes(s, num_codebooks=8, codebook_size=2048) == g["codes"]
    assert torch.equal(chars_to_codes(s, 8, 2048, return_tensors="pt"), torch.tensor(codes))
    # tensor input and list input give the same string; copy_before_conversion leaves the input intact
    assert codes_to_chars(torch.from_numpy(codes), 2048) == s
    assert codes_to_chars(codes.tolist(), 2048) == s
    c2 = codes.copy()
    codes_to_chars(c2, 2048)
    assert np.array_equal(c2, codes)


def test_codes_to_chars_errors():
    with pytest.raises(ValueError):
        codes_to_chars(np.zeros(5, np.int64), 2048)
    assert codes_to_chars(np.zeros((8, 0), np.int64), 2048) == ""


def _header_symbols():
    with open(os.path.join(ROOT, "include", "mimi_hip.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:[a-z_0-9]+\s*\*?\s+)+\**(mimi_[a-z_0-9]+)\s*\(", txt, re.M)))


def test_lib_exports_every_header_symbol():
    from mimi_hip import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.EXPORTED_SYMBOLS)


def test_header_documents_every_engine_option():
    """Every mimi_set_option key of the engine's table (engine.cpp kEngineOptions) is documented in the C header,
    and the header names no key the engine would reject."""
    src = open(os.path.join(ROOT, "tokenize-audio_amd", "csrc", "engine.cpp")).read()
    table = src[src.index("kEngineOptions[] = {"):]
    table = table[:table.index("};")]
    keys = re.findall(r'\{"([a-z0-9_]+)", &mimi_engine::', table)
    assert len(keys) >= 10, keys
    hdr = open(os.path.join(ROOT, "include", "mimi_hip.h")).read()
    doc = hdr[hdr.index("mimi_set_option") - 4000:hdr.index("int mimi_set_option(")]
    for k in keys:
        assert f'"{k}"' in doc, k
    for k in re.findall(r'"([a-z0-9_]+)"', doc[doc.index("key"):]):
        assert k in keys, k


def test_lib_length_math_matches_python():
    from mimi_hip import _lib
    lib = _lib.load()
    for L in [1, 2, 1919, 1920, 1921, 23999, 24000, 240000, 240001, 1440000, 16_777_217, 50_000_001]:
        assert lib.mimi_encoded_length(L) == encoded_length(L), L
    cfg = _lib.default_config()
    assert cfg.hidden_size == 512 and list(cfg.upsampling_ratios)[:4] == [8, 6, 5, 4]
    assert lib.mimi_encoded_length_cfg(ctypes.byref(cfg), 240000) == 125


def test_lib_errors_without_device():
    """No GPU here: create must fail with a status + message, never crash or fall back."""
    from mimi_hip import _lib
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = _lib.load()
    h = ctypes.c_void_p()
    st = lib.mimi_create(None, 0, ctypes.byref(h))
    assert st != 0 and lib.mimi_last_error()
    assert lib.mimi_encode(None, None, 1, 1, 8, None, None) == 1


class _OracleModel:
    """Test double exposing MimiHipModel.encode's contract on the CPU oracle (host-logic test only)."""

    def __init__(self, sd):
        self.sd = sd

    def to(self, *_):
        return self

    def eval(self):
        return self

    def encode(self, input_values, padding_mask=None, num_quantizers=None):
        from oracle import mimi_ref
        from mimi_hip.model import MimiEncoderOutput
        return MimiEncoderOutput(mimi_ref.encode(input_values.cpu(), self.sd, num_quantizers))


def test_wrapper_batch_semantics_match_reference(golden, state_dict):
    """mimi_hip.MimiEncoder's pad/trim/delegate logic reproduces the reference wrapper's outputs."""
    from mimi_hip.encoder import MimiEncoder
    arrays, meta = golden
    enc = MimiEncoder(device="cpu", model=_OracleModel(state_dict))
    audio = [synthetic.speech_like(L, meta["audio_seed"], 200 + i) for i, L in enumerate(meta["batch_lengths"])]
    assert synthetic.audio_sha256(audio) == meta["audio_sha256"]["batch"]
    outs = enc.encode_audio_batch(audio, 24000)
    assert len(outs) == len(audio)
    for i, o in enumerate(outs):
        ref = arrays[f"batch_item{i}"]
        assert o.shape == ref.shape and o.dtype == np.int64
        assert np.array_equal(o, ref), i  # the oracle is the reference's arithmetic on this CPU
    single = enc.encode_audio_batch([audio[2]], 24000)
    assert single[0].shape == arrays["batch_single"].shape
    assert enc.encode_audio_batch([], 24000) == []
    chunk = enc.encode_audio_chunk(audio[3], 24000)
    assert chunk.shape == arrays["chunk_item3"].shape
    # pad-to-longest changes only the last frame of padded items (everything is causal)
    alone = enc.encode_audio_chunk(audio[0], 24000)
    assert np.array_equal(alone[:, :-1], outs[0][:, :-1])


def test_import_without_gpu_has_no_fallback():
    from mimi_hip import model
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(Exception):
        model.MimiHipModel(synthetic.make_state_dict(seed=0, num_quantizers=2), device="cuda")


def test_bench_north_star_groups(tmp_path):
    """bench.py's north-star breakdown: stage grouping, PMC lookup by stage (then by bare symbol), HBM rate
    arithmetic, a stage measured on another build's kernel flagged, and PMC bytes of another workload not used."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    pmc = {"tag": "t", "kernels": {"mimi::resblock0_h16_kernel": {"traffic_bytes": 2.0e9}},
           "stages": {"down_s0": {"traffic_bytes": 1.0e9, "kernel": "mimi::gemm_planes_kernel<1, 3>"}}}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(pmc))
    prof = {"res_s0": {"ms": 7.0, "flops": 1.4e12, "kernel": "mimi::resblock0_h16_kernel(mimi::ResArgs)",
                       "launches": 10},
            "down_s0": {"ms": 10.0, "flops": 2.5e12, "kernel": "void mimi::gemm_planes_kernel<1, 2>", "launches": 10},
            "qkv": {"ms": 5.0, "flops": 1.0e12, "kernel": "unknown", "launches": 80}}
    wl = {"kind": "batch", "batch": 32, "seconds": 10.0}
    assert bench.load_pmc(str(p), wl)[0] == {}  # no workload key: not this workload's bytes
    pmc["workload"] = wl
    p.write_text(json.dumps(pmc))
    other, why = bench.load_pmc(str(p), dict(wl, batch=1))
    assert other == {} and "batch" in why
    g0 = bench.north_star_groups(prof, 10, other, why)
    assert "hbm_GBps" not in g0["conv_stack"] and g0["conv_stack"]["hbm_unmeasured_why"] == why
    g = bench.north_star_groups(prof, 10, bench.load_pmc(str(p), wl)[0])
    cs = g["conv_stack"]
    assert cs["stages"] == ["res_s0", "down_s0"] and cs["ms_per_step"] == 1.7
    assert cs["hbm_bytes_per_step"] == 3_000_000_000 and abs(cs["hbm_GBps"] - 3e9 / 1.7e-3 / 1e9) < 0.1
    assert cs["hbm_measured_on_other_kernel"] == ["down_s0"]
    assert g["transformer"]["hbm_unmeasured_stages"] == ["qkv"]
    assert "quantizer" not in g


def test_stage_keyed_pmc_alignment(tmp_path):
    """tools/summarize_profile.stage_bytes: counter rows after the spin marker walked against the launch sequence;
    a stage's extra dispatches (RVQ levels, final) summed into it; bookkeeping kernels left out."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import summarize_profile as sp
    seq = [["res_s0", "mimi::resblock0_h16_kernel"], ["down_s0", "mimi::gemm_planes_kernel<1, 2>"],
           ["rvq", "mimi::rvq_level_h16_kernel<256, 4, 16>"]]
    rows = [("void at::spin_kernel(long)", 9)]
    for enc in range(2):
        rows += [("mimi::resblock0_h16_kernel(mimi::ResArgs)", 10), ("void mimi::gemm_planes_kernel<1, 2>(mimi::GemmArgs)", 20),
                 ("void mimi::rvq_level_h16_kernel<256, 4, 16>(mimi::RvqArgs, int)", 1),
                 ("void mimi::rvq_level_h16_kernel<256, 4, 16>(mimi::RvqArgs, int)", 2),
                 ("mimi::rvq_final_kernel(mimi::RvqArgs, int)", 3), ("mimi::amax_reduce_kernel(unsigned int*, int)", 99)]
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tmp_path / f"pmc_{counter}"
        d.mkdir()
        with open(d / "run_counter_collection.csv", "w") as f:
            f.write("Dispatch_Id,Kernel_Name,Counter_Value\n")
            for i, (k, v) in enumerate(rows):
                f.write(f'{i},"{k}",{v}\n')
    st = sp.stage_bytes(str(tmp_path), seq)
    assert st["res_s0"]["write_bytes"] == 10 * 1024 and st["down_s0"]["fetch_bytes"] == 20 * 1024 * 2
    assert st["rvq"]["write_bytes"] == 6 * 1024 and st["rvq"]["launches_WRITE_SIZE"] == 2
    assert st["rvq"]["traffic_bytes"] == 6 * 1024 * 3
