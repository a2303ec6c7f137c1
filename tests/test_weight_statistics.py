"""GPU: the f16x3 arithmetic on weights whose statistics differ from the seeded synthetic checkpoint's (VERDICT r5
weak #3: the kyutai/mimi weights are not available offline, so the activation scales' headroom was only ever measured
on one weight distribution).  The fixed activation scales are calibrated at mimi_finalize on the LOADED weights
(DESIGN.md §3.2), so they must follow any weight statistics.  Three perturbed checkpoints -- the early SEANet convs
8x louder and the late ones quieter, heavy-tailed (Student-t, 3 degrees of freedom) weights of the same spread, and
transformer layer scales 5x larger -- each encode a speech-like clip and a full-scale noise clip and must keep the
north-star bars against the CPU oracle: pre-quantizer relative error < 1e-4, the quantizer bit-exact on the oracle's
embedding, and no overflow fallback on these signals."""
import numpy as np
import pytest
import torch

from mimi_hip import synthetic

pytestmark = pytest.mark.gpu


def _perturb(sd, kind):
    sd = {k: v.copy() for k, v in sd.items()}
    rng = np.random.default_rng(17)
    if kind == "loud_early":
        for k in sd:
            if k.startswith("encoder.layers.") and k.endswith(".weight"):
                layer = int(k.split(".")[2])
                sd[k] *= np.float32(8.0 if layer < 4 else (0.5 if layer > 10 else 1.0))
    elif kind == "heavy_tailed":
        for k in sd:
            if (k.startswith("encoder.layers.") or "mlp.fc" in k or "self_attn." in k) and k.endswith(".weight"):
                t = rng.standard_t(3, size=sd[k].shape)
                sd[k] = (t / np.sqrt(3.0) * sd[k].std()).astype(np.float32)  # (t_3 has variance 3)
    elif kind == "large_layer_scale":
        for k in sd:
            if k.endswith("layer_scale.scale"):
                sd[k] *= np.float32(5.0)
    return sd


@pytest.mark.parametrize("kind", ["loud_early", "heavy_tailed", "large_layer_scale"])
def test_f16x3_follows_weight_statistics(kind):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mimi_hip.model import MimiHipModel
    from oracle import mimi_ref
    sd = _perturb(synthetic.make_state_dict(seed=0, num_quantizers=8), kind)
    model = MimiHipModel(sd, device="cuda:0")
    L = 36000
    speech = synthetic.speech_like(L, 21, 0)
    noise = np.random.default_rng(22).uniform(-1, 1, L).astype(np.float32)
    x = torch.from_numpy(np.stack([speech, noise]))[:, None]
    model.set_taps(True)
    try:
        codes = model.encode(x.cuda(), num_quantizers=8).audio_codes.cpu()
        emb = torch.from_numpy(model.get_tap("downsample")).permute(0, 2, 1)
    finally:
        model.set_taps(False)
    taps = {}
    ref_codes = mimi_ref.encode(x, sd, 8, taps=taps)
    ref = taps["pre_quantizer"]
    err = float((emb - ref).abs().max() / ref.abs().max())
    assert err < 1e-4, (kind, err)
    assert torch.equal(model.quantize(ref.cuda(), 8).cpu(), ref_codes), kind
    assert model.f16_reruns == 0, kind
    assert codes.shape == ref_codes.shape and float((codes == ref_codes).float().mean()) > 0.99, kind
