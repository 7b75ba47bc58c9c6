"""Per-iteration band for BiCGSTAB residual histories (test helper, no tests).

BiCGSTAB's residual history against the reference's, per iteration, over the WHOLE
history.  Its recurrence amplifies any reduction-order
difference: the reference against ITSELF (1 vs 8 OpenMP threads, the same binary;
tests/golden/reference_runs.json "*_hist" and "*_hist_t8") differs by 1e-13 at
iteration 10, 1e-10 at 20 and O(1) past ~80 at 256^2.  The band per iteration k is
that measured spread, S_k = max over i <= k of |r8_i - r1_i| / r1_i (floor 1e-15),
widened BAND_F times: |ln(h_k / r1_k)| <= ln(1 + BAND_F S_k).  Measured on the
device (r06c, tools/sr_hist_dump.py): the fused passes' deviation from the 1-thread
run peaks at 53 S_k (256^2 identity), 23 (128^2), 11 / 8 (cbpr2), 2-4 at 4096^2.
"""
import numpy as np

BAND_F = 100.0


def bicgstab_band(h, r1, r8):
    k = min(len(h), len(r1), len(r8))
    h, r1, r8 = (np.asarray(v[:k], dtype=float) for v in (h, r1, r8))
    S = np.maximum.accumulate(np.maximum(np.abs(r8 - r1) / r1, 1e-15))
    lhs, rhs = np.abs(np.log(h / r1)), np.log1p(BAND_F * S)
    return bool(np.all(lhs <= rhs)), float(np.max(lhs / rhs))
