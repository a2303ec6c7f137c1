"""Near-tie audit shared by the CPU and GPU parity tests.

Bit-exact codes from an fp32 network are only possible up to near-ties: any other summation order (a GPU
kernel, another host's BLAS) moves activations by ~1e-6 relative and can flip a code whose best and
second-best distances are that close (SURVEY.md §7 'Hard parts').  A mismatch is accepted only where the
reference's own relative top-2 margin at the FIRST diverging level of the frame's chain is below NEAR_TIE;
later levels of the same chain follow from the different residual and are not audited separately.
"""
import numpy as np

NEAR_TIE = 2e-4


def margin_audit(codes, ref_codes, margins, near_tie=NEAR_TIE):
    """codes / ref_codes / margins: [K, T] (semantic level 0, acoustic levels 1.. chained).
    Returns (exact-match fraction, list of unexplained (frame, level, margin))."""
    codes = np.asarray(codes)
    ref_codes = np.asarray(ref_codes)
    margins = np.asarray(margins, dtype=np.float64)
    assert codes.shape == ref_codes.shape == margins.shape, (codes.shape, ref_codes.shape, margins.shape)
    K, T = ref_codes.shape
    bad = []
    for t in range(T):
        diff = np.nonzero(codes[:, t] != ref_codes[:, t])[0]
        if len(diff) == 0:
            continue
        for chain in ([0], list(range(1, K))):
            d = [k for k in diff if k in chain]
            if d and margins[d[0], t] > near_tie:
                bad.append((t, int(d[0]), float(margins[d[0], t])))
    return float((codes == ref_codes).mean()), bad
