"""Near-tie audit shared by the CPU and GPU parity tests.

Bit-exact codes from an fp32 network are only possible up to near-ties: any other summation order (a GPU
kernel, another host's BLAS) moves activations by ~1e-6 relative and can flip a code whose best and
second-best distances are that close (SURVEY.md §7 'Hard parts').  A mismatch is accepted only where the
reference's own relative top-2 margin m = (d2 - d1) / d2 at the FIRST diverging level of the frame's chain is
below the near-tie threshold; later levels of the same chain follow from the different residual and are not
audited separately.

The threshold is DERIVED from the measured perturbation (``perturbation_near_tie``) wherever the test has both
embeddings: the engine's RVQ is bit-exact with the reference's given the same residual
(test_quantizer_bit_exact_on_reference_embedding), so up to the first diverging level the only difference is the
pre-quantizer error e = emb - emb_ref, projected by the chain's input_proj W: r' = r + W e.  Every distance moves
by at most |W e| (triangle inequality), so the reference's best code a can lose to b only if d_b - d_a <= 2 |W e|,
i.e. m <= 2 |W e| / d2, plus the fp32 rounding of the two mm-form distance chains (FP32_DIST_SLACK relative).
NEAR_TIE (fixed) remains only for the CPU oracle-vs-fixture tests, where no second embedding exists.
"""
import numpy as np

NEAR_TIE = 2e-4
FP32_DIST_SLACK = 8e-6  # two fp32 mm-form distance chains of 256 terms: ~sqrt(256) ulps of |r|^2 + |e|^2 each


def margin_audit(codes, ref_codes, margins, near_tie=NEAR_TIE):
    """codes / ref_codes / margins: [K, T] (semantic level 0, acoustic levels 1.. chained); near_tie a scalar or a
    [K, T] array (perturbation_near_tie).  Returns (exact-match fraction, list of unexplained (frame, level,
    margin, threshold))."""
    codes = np.asarray(codes)
    ref_codes = np.asarray(ref_codes)
    margins = np.asarray(margins, dtype=np.float64)
    assert codes.shape == ref_codes.shape == margins.shape, (codes.shape, ref_codes.shape, margins.shape)
    thr = np.broadcast_to(np.asarray(near_tie, dtype=np.float64), margins.shape)
    K, T = ref_codes.shape
    bad = []
    for t in range(T):
        diff = np.nonzero(codes[:, t] != ref_codes[:, t])[0]
        if len(diff) == 0:
            continue
        for chain in ([0], list(range(1, K))):
            d = [k for k in diff if k in chain]
            if d and margins[d[0], t] > thr[d[0], t]:
                bad.append((t, int(d[0]), float(margins[d[0], t]), float(thr[d[0], t])))
    return float((codes == ref_codes).mean()), bad


def first_flip_margins(codes, ref_codes, margins):
    """The reference margins at each frame-chain's first diverging level (the flips the audit judges)."""
    codes, ref_codes = np.asarray(codes), np.asarray(ref_codes)
    margins = np.asarray(margins, dtype=np.float64)
    out = []
    K, T = ref_codes.shape
    for t in range(T):
        diff = np.nonzero(codes[:, t] != ref_codes[:, t])[0]
        for chain in ([0], list(range(1, K))):
            d = [k for k in diff if k in chain]
            if d:
                out.append(float(margins[d[0], t]))
    return out


def perturbation_near_tie(emb, emb_ref, sd, seconds, num_semantic=1):
    """Per-code audit thresholds [B, K, T] from the measured pre-quantizer error (module docstring).

    emb, emb_ref: [B, 512, T] (ours, the reference's); seconds: the reference's second-best distance d2 per code
    [B, K, T] (oracle rvq_from_embedding(return_second=True)); sd: the state dict (input_proj weights)."""
    e = np.asarray(emb, np.float64) - np.asarray(emb_ref, np.float64)
    d2 = np.asarray(seconds, np.float64)
    B, K, T = d2.shape
    thr = np.empty_like(d2)
    for which, levels in (("semantic", range(0, num_semantic)), ("acoustic", range(num_semantic, K))):
        W = np.asarray(sd[f"quantizer.{which}_residual_vector_quantizer.input_proj.weight"], np.float64)[:, :, 0]
        pe = np.linalg.norm(np.einsum("oc,bct->bot", W, e[:, :, :T]), axis=1)  # [B, T]
        for lv in levels:
            thr[:, lv] = 2.0 * pe * (1.0 + 1e-9) / np.maximum(d2[:, lv], 1e-30) + FP32_DIST_SLACK
    return thr
