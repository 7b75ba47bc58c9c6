"""The look-ahead blocked MGS-R schedule (tests/lookahead_model.py, the host model
of k_mgs_bla) against strict MGS-R: every block subtracted once, in the blocked
step's order, each all-gather collected one pass after it was published, and
the same H column and V(:, j+1) as gmres_mgsr.f90:341-363 up to rounding."""
import numpy as np
import pytest

from tests import lookahead_model as lm


@pytest.mark.parametrize("S", [2])
@pytest.mark.parametrize("j", list(range(1, 41)) + [63, 94, 95])
def test_schedule_invariants(j, S):
    seq = lm.blocks(j, S)
    sch = lm.schedule(j, S)
    n = len(seq) // 2
    subs = [s for s, _ in sch if s >= 0]
    assert subs == list(range(len(seq)))                  # every block once, in order
    assert sch[-1] == (len(seq) - 1, lm.NORM)              # the norm after the last AXPY
    dotted = {d: pi for pi, (_, d) in enumerate(sch) if d >= 0}
    assert sorted(dotted) == list(range(1, len(seq)))      # every block but the first dotted
    for pi, (sub, _) in enumerate(sch):
        if pi >= 2 and sub >= 0:
            assert dotted[sub] == pi - 2                   # cache rotation: A <- B <- C
    for b, pi in dotted.items():
        # everything before b-1 subtracted by the dot; b-1 at most one pass later, and
        # then in the same sweep (the Gram correction never crosses the sweeps)
        subbed = {s for s, _ in sch[:pi + 1] if s >= 0}
        assert set(range(b - 1)) <= subbed
        if b - 1 not in subbed:
            assert sch[pi + 1][0] == b - 1 and (b - 1 < n) == (b < n)
    # passes: the blocks plus two dummies
    assert len(sch) == len(seq) + 2


@pytest.mark.parametrize("j", [1, 2, 3, 4, 5, 8, 17, 30, 47, 95])
def test_lookahead_matches_strict_mgs(j):
    rng = np.random.default_rng(1000 + j)
    n = 400
    V, _ = np.linalg.qr(rng.standard_normal((n, j)))
    # a w with large components along the basis (as A v_j has in GMRES) plus a small rest
    w = V @ rng.standard_normal(j) * 10.0 + rng.standard_normal(n) * 1e-3
    H, v, _ = lm.lookahead_step(V, w, j, 2)
    Hs, vs = lm.strict_step(V, w, j)
    assert np.allclose(H, Hs, rtol=1e-10, atol=1e-12 * np.abs(Hs).max()), np.abs(H - Hs).max()
    assert np.abs(v - vs).max() < 1e-8
    # and the new column is orthogonal to the basis as well as strict MGS-R makes it
    assert np.abs(V.T @ v).max() < 10 * max(np.abs(V.T @ vs).max(), 1e-15)
