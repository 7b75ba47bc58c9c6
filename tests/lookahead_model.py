"""Host model of a look-ahead blocked MGS-R step: the pass schedule and the h
recurrence, in numpy, checked against strict MGS-R (gmres_mgsr.f90:341-360) on
the CPU (tests/test_lookahead_model.py).  Round 5 built it as a kernel
(k_mgs_bla) on this model -- parity green against the reference's histories --
and removed it: every build measured slower than the plain blocked step
(profiles/r05/ab_lookahead_r05mnop.txt, ab_lookahead_r05qr.txt).
The model stays as the tested specification for a next attempt.

The blocked step dots block b in the pass that subtracts block
b-1 and all-gathers right after it; the look-ahead step dots block b one pass
EARLIER -- in the pass that subtracts b-2 -- and collects that all-gather one pass
later, so every all-gather overlaps a whole pass.  The block subtracted in between
(b-1) enters h(b) as a Gram correction:

  z_t = <w after subtracting b-2, V_t>
  h_t = z_t - sum_{s in b-1} h_s <V_s, V_t> - sum_{s < t in b} h_s <V_s, V_t>

with the Gram terms taken in the same pass as z (the block b-1 is cached on chip,
block b streams), so no table is needed.  Pass pi dots dot(pi) and subtracts
sub(pi) = dot(pi - 2) (the cache rotates A <- B <- C), DUMMY (h = 0) where that is
not a block.  Dots by pass: sweep 1: pi = i - 1 for block i = 1..n-1; one pass
without a dot (pi = n - 1) so that sweep 2's first block is dotted after sweep 1
is fully subtracted; sweep 2: pi = i for i = n..2n-1; pass 2n without a dot; pass
2n + 1 subtracts the last block and takes ||w||^2.
"""
from __future__ import annotations

import numpy as np

NONE, NORM, DUMMY = -1, -2, -3


def blocks(j: int, S: int) -> list[list[int]]:
    """The blocked step's block sequence of step j (0-based columns): sweep 1
    {0}, {1..S}, {S+1..2S}, ...; sweep 2 the same blocks in reverse
    (GK_BLK_REV2)."""
    b1 = [[0]] + [list(range(lo, min(lo + S, j))) for lo in range(1, j, S)]
    return b1 + b1[::-1]


def schedule(j: int, S: int) -> list[tuple[int, int]]:
    """(sub, dot) per pass: indices into blocks(j, S), or DUMMY / NONE / NORM."""
    seq = blocks(j, S)
    P = len(seq)
    n = P // 2
    dot = []
    for i in range(1, n):
        dot.append(i)          # sweep 1: pass i - 1 dots block i
    dot.append(NONE)           # pass n - 1: sweep 2's first block waits for sweep 1
    for i in range(n, P):
        dot.append(i)          # sweep 2: pass i dots block i
    dot.append(NONE)           # pass P: the last block is subtracted next
    dot.append(NORM)           # pass P + 1: subtract the last block, ||w||^2
    out = []
    for pi, d in enumerate(dot):
        if pi == 0:
            sub = 0
        elif pi == 1:
            sub = DUMMY
        else:
            sub = dot[pi - 2] if dot[pi - 2] >= 0 else DUMMY
        out.append((sub, d))
    return out


def lookahead_step(V: np.ndarray, w: np.ndarray, j: int, S: int):
    """Run the schedule on w (n,) against V (n, >= j): returns (H column of
    length j + 1, w / ||w||, the schedule).  Arithmetic in numpy float64; dots
    are plain np.dot (the order differs from the device's, which only matters
    at rounding level)."""
    seq = blocks(j, S)
    sch = schedule(j, S)
    w = w.copy()
    H = np.zeros(j + 1)
    h_known = {0: np.array([V[:, 0] @ w])}  # block 0 of sweep 1: the first dot (pin)
    pending = None  # (block index, z, Gram B x C, Gram C x C, h of the block subtracted in between)
    n = len(seq) // 2
    for pi, (sub, d) in enumerate(sch):
        # the pass: subtract `sub` with its known h (DUMMY: nothing), then dot `d`
        if sub >= 0:
            hs = h_known.pop(sub)
            for s, c in enumerate(seq[sub]):
                w -= hs[s] * V[:, c]
                H[c] = (H[c] if sub >= n else 0.0) + hs[s]
            h_between = (sub, hs)
        else:
            h_between = None
        if d == NORM:
            hn = np.sqrt(w @ w)
            H[j] = hn
            return H, w / hn, sch
        new = None
        if d >= 0:
            cols = seq[d]
            z = np.array([w @ V[:, c] for c in cols])
            prev = seq[sch[pi + 1][0]] if pi + 1 < len(sch) and sch[pi + 1][0] >= 0 else []
            gbc = np.array([[V[:, b] @ V[:, c] for c in cols] for b in prev]).reshape(len(prev), len(cols))
            gcc = np.array([[V[:, a] @ V[:, c] for c in cols] for a in cols])
            new = (d, z, gbc, gcc)
        # collect the all-gather published one pass earlier: h of that block, corrected
        # for the block this pass subtracted (its h: h_between)
        if pending is not None:
            bd, z, gbc, gcc = pending
            h = z.copy()
            if h_between is not None and gbc.size:
                h -= h_between[1] @ gbc
            for t in range(len(h)):
                for s in range(t):
                    h[t] -= h[s] * gcc[s, t]
            h_known[bd] = h
        pending = new
    raise AssertionError("schedule without a norm pass")


def strict_step(V: np.ndarray, w: np.ndarray, j: int):
    """Strict MGS-R (gmres_mgsr.f90:341-363): two sweeps of j projections."""
    w = w.copy()
    H = np.zeros(j + 1)
    for sweep in range(2):
        for i in range(j):
            h = w @ V[:, i]
            H[i] = (H[i] if sweep else 0.0) + h
            w -= h * V[:, i]
    hn = np.sqrt(w @ w)
    H[j] = hn
    return H, w / hn
