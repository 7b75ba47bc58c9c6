"""Host evaluation of the reference's orthogonality diagnostics on a basis
copied off the device (test infrastructure for tests/test_gpu_solver.py).

  mgs_verr      gmres_mgsr.f90:414-420  (cumulative v_err(1:n_out+1))
  hh_verr       gmres_hh.f90:568-593    calculate_verr: V_i = P_1..P_i e_i
                rebuilt from the reflectors, then v_err(i) = sum_{j<i} 2 (V_i.V_j)^2
  hh_verr_of_basis   the second half of calculate_verr on an already rebuilt V

`dot` is either the reference's sequential dot_product (oracle.dot at one
thread, ref_dot) or an extended-precision dot (exact_dot, x87 long double
accumulation of the rounded products -- about 11 more bits than the values).
"""
from __future__ import annotations

import numpy as np


def ref_dot(oracle):
    oracle.set_threads(1)
    return oracle.dot


def exact_dot(a, b):
    return float(np.dot(np.asarray(a, dtype=np.longdouble), np.asarray(b, dtype=np.longdouble)))


def mgs_verr(V, n_out, dot):
    v = np.zeros(n_out + 2)
    for j in range(1, n_out + 1):
        s = 0.0
        for i in range(1, j + 1):
            d = dot(V[i - 1], V[j])
            s = s + 2.0 * (d * d)
        dd = dot(V[j], V[j]) - 1.0
        s = s + dd * dd
        v[j] = np.sqrt(v[j - 1] * v[j - 1] + s)
    return v


def hh_verr_of_basis(Vb, n_iter, dot):
    v = np.zeros(n_iter + 1)
    for i in range(1, n_iter):
        s = 0.0
        for j in range(i):
            d = dot(Vb[i], Vb[j])
            s = s + 2.0 * (d * d)
        v[i] = s
    return v


def hh_rebuild(P, n_iter, dot):
    """calculate_verr's V(:,i) = P_1..P_i e_i (gmres_hh.f90:581-585)."""
    n = P[0].size
    Vb = []
    for i in range(n_iter):
        vi = np.zeros(n)
        vi[i] = 1.0
        for j in range(i, -1, -1):
            d = dot(vi, P[j])
            vi = vi - (2.0 * P[j]) * d
        Vb.append(vi)
    return Vb


def hh_verr(P, n_iter, dot):
    return hh_verr_of_basis(hh_rebuild(P, n_iter, dot), n_iter, dot)
