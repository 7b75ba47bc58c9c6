"""Distributed restatement of the multi-GPU protocol of libgmres_hip
(gmres_amd/csrc/gk_api.hip), in numpy over torch.distributed (gloo), for the
CPU multi-process tests.  TEST INFRASTRUCTURE: it checks the decomposition
(row-block slabs of grid lines, one-line halo exchange before every stencil,
all-reduced partial dots, the Householder pivot owned by rank 0 and
broadcast), not the kernels.

Per rank it runs exactly the C-ABI's message pattern:
  halo(v)        : send first line to rank-1 / last line to rank+1, receive
                   the neighbours' lines into halo_lo / halo_hi
  allreduce(p)   : sum of the per-rank partials (one value per projection)
  bcast(hb, 0)   : w(1:j+1) from the owner of the first global indices
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


class Slab:
    def __init__(self, N: int, line0: int, nlines: int, rank: int, world: int):
        self.N, self.line0, self.nlines, self.rank, self.world = N, line0, nlines, rank, world
        self.n = N * nlines
        self.g0 = N * line0

    # -- communication ------------------------------------------------------
    def halo(self, v: np.ndarray):
        N = self.N
        lo = np.zeros(N) if self.rank > 0 else None
        hi = np.zeros(N) if self.rank < self.world - 1 else None
        reqs = []
        if self.rank > 0:
            reqs.append(dist.isend(torch.from_numpy(v[:N].copy()), self.rank - 1))
            t_lo = torch.zeros(N, dtype=torch.float64)
            reqs.append(dist.irecv(t_lo, self.rank - 1))
        if self.rank < self.world - 1:
            reqs.append(dist.isend(torch.from_numpy(v[-N:].copy()), self.rank + 1))
            t_hi = torch.zeros(N, dtype=torch.float64)
            reqs.append(dist.irecv(t_hi, self.rank + 1))
        for r in reqs:
            r.wait()
        if lo is not None:
            lo = t_lo.numpy()
        if hi is not None:
            hi = t_hi.numpy()
        return lo, hi

    def allreduce(self, x: float) -> float:
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t)
        return float(t.item())

    def bcast(self, a: np.ndarray, root: int = 0) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64).copy())
        dist.broadcast(t, root)
        return t.numpy()

    # -- operators -----------------------------------------------------------
    def stencil(self, x: np.ndarray, div: float = 1.0) -> np.ndarray:
        """y = A (x/div) on the slab, sum order ((W+E)+S)+N, zeros outside."""
        N, L = self.N, self.nlines
        lo, hi = self.halo(x)
        X = np.zeros((L + 2, N + 2))
        X[1:L + 1, 1:N + 1] = x.reshape(L, N) / div
        if lo is not None:
            X[0, 1:N + 1] = lo / div
        if hi is not None:
            X[L + 1, 1:N + 1] = hi / div
        C = X[1:L + 1, 1:N + 1]
        s = ((X[1:L + 1, 0:N] + X[1:L + 1, 2:N + 2]) + X[2:L + 2, 1:N + 1]) + X[0:L, 1:N + 1]
        return (4.0 * C - 1.0 * s).reshape(-1)

    def precond(self, kind: str, r: np.ndarray, params=(8.2, 0.2), degree=8) -> np.ndarray:
        if kind == "identity":
            return r.copy()
        if kind == "cbpr2":
            em, eM = params
            c = (eM - em) / 2.0
            d = (eM + em) / 2.0
            alpha = 1.0 / d
            beta = (c * alpha / 2.0) ** 2
            alpha = 1.0 / (d - beta)
            zp = r / d
            aux = self.stencil(r, d)
            return zp + alpha * (r - aux)
        theta = (params[0] + params[1]) / 2.0
        delta = abs(params[1] - params[0]) / 2.0
        sigma, rho0 = theta / delta, delta / theta
        res, dv = r.copy(), r / theta
        z = dv.copy()
        for _ in range(degree):
            rho1 = 1.0 / (2.0 * sigma - rho0)
            ad = self.stencil(dv)
            res = res - ad
            dv = (rho1 * rho0) * dv + (2.0 * rho1 / delta) * res
            z = z + dv
            rho0 = rho1
        return z

    def dot(self, a, b) -> float:
        return self.allreduce(float(np.dot(a, b)))


def givens(H, cs, sn, g, j):
    for i in range(j):
        tmp = H[i, j]
        H[i, j] = cs[i] * tmp + sn[i] * H[i + 1, j]
        H[i + 1, j] = -sn[i] * tmp + cs[i] * H[i + 1, j]
    ds = np.hypot(H[j + 1, j], H[j, j])
    cs[j] = H[j, j] / ds
    sn[j] = H[j + 1, j] / ds
    H[j, j] = cs[j] * H[j, j] + sn[j] * H[j + 1, j]
    H[j + 1, j] = 0.0
    tmp = g[j]
    g[j] = cs[j] * tmp + sn[j] * g[j + 1]
    g[j + 1] = -sn[j] * tmp + cs[j] * g[j + 1]


def back_solve(H, g, n_out):
    y = np.zeros(n_out)
    y[n_out - 1] = g[n_out - 1] / H[n_out - 1, n_out - 1]
    for i in range(n_out - 2, -1, -1):
        y[i] = (g[i] - np.dot(H[i, i + 1:n_out], y[i + 1:n_out])) / H[i, i]
    return y


def mgsr(S: Slab, b, m, tol=1e-15, prec="identity", max_cycles=1000):
    """gmres_mgsr_omp semantics on the slab; returns (x_local, hist_res, iterations)."""
    n = S.n
    x = np.zeros(n)
    beta0 = np.sqrt(S.dot(b, b))
    V = np.zeros((m + 1, n))
    hist = []
    converged, n_out, h_val = False, 0, 0.0
    cs, sn = np.zeros(m), np.zeros(m)
    for st in range(1, max_cycles + 1):
        H = np.zeros((m + 1, m))
        g = np.zeros(m + 1)
        w = S.precond(prec, b - S.stencil(x))
        beta = np.sqrt(S.dot(w, w))
        g[0] = beta
        V[0] = w / beta
        for j in range(m):
            if converged:
                break
            n_out = j + 1
            w = S.precond(prec, S.stencil(V[j]))
            for _ in range(2):
                for i in range(j + 1):
                    h = S.dot(w, V[i])
                    H[i, j] += h
                    w = w - h * V[i]
            h_val = np.sqrt(S.dot(w, w))
            H[j + 1, j] = h_val
            givens(H, cs, sn, g, j)
            fe = abs(g[j + 1]) / beta0
            V[j + 1] = w / h_val
            if fe < tol:
                converged = True
        y = back_solve(H, g, n_out)
        x = x + y @ V[:n_out]
        r = b - S.stencil(x)
        hist.append(np.sqrt(S.dot(r, r)) / beta0)
        if h_val < tol or fe < tol:
            return x, hist, (st - 1) * m + n_out
    return x, hist, (max_cycles - 1) * m + n_out


def hh(S: Slab, b, m, tol=1e-15, prec="identity", midcycle_exit=False, max_cycles=1000):
    """gmres_hh_omp / gmres_hh_prec_omp on the slab; rank 0 owns global 0..m."""
    n = S.n
    gidx = S.g0 + np.arange(n)
    x = np.zeros(n)
    beta0 = np.sqrt(S.dot(b, b))
    hist = []
    converged, n_out = False, 0
    cs, sn = np.zeros(m), np.zeros(m)
    for k in range(1, max_cycles + 1):
        P = np.zeros((m + 1, n))
        H = np.zeros((m + 1, m))
        g = np.zeros(m + 1)
        w = b - S.stencil(x)
        if midcycle_exit:
            w = S.precond(prec, w)
        beta = np.sqrt(S.dot(w, w))
        w1 = S.bcast(w[:1] if S.rank == 0 else np.zeros(1))[0]
        g[0] = -np.copysign(abs(beta), w1)
        if S.rank == 0:
            w[0] = np.copysign(abs(beta), w1) + w[0]
        P[0] = w / np.sqrt(S.dot(w, w))
        for j in range(m):
            if converged:
                break
            n_out = j + 1
            v = (gidx == j).astype(np.float64)
            for i in range(j, -1, -1):
                v = v - 2.0 * P[i] * S.dot(v, P[i])
            w = S.stencil(v)
            if midcycle_exit:
                w = S.precond(prec, w)
            for i in range(j + 1):
                w = w - 2.0 * P[i] * S.dot(w, P[i])
            hb = S.bcast(w[:j + 2] if S.rank == 0 else np.zeros(j + 2))
            tail = w * (gidx >= j + 1)
            tmp = np.sqrt(S.dot(tail, tail))
            H[:j + 1, j] = hb[:j + 1]
            H[j + 1, j] = -tmp if hb[j + 1] > 0 else tmp
            w = np.where(gidx < j + 1, 0.0, w)
            w = np.where(gidx == j + 1, w - H[j + 1, j], w)
            P[j + 1] = w / np.sqrt(S.dot(w, w))
            givens(H, cs, sn, g, j)
            fe = abs(g[j + 1]) / beta0
            if midcycle_exit and fe < tol:
                converged = True
        y = back_solve(H, g, n_out)
        w = np.zeros(n)
        own = gidx < n_out
        w[own] = y[gidx[own]]
        for i in range(n_out - 1, -1, -1):
            w = w - 2.0 * P[i] * S.dot(w, P[i])
        x = x + w
        r = b - S.stencil(x)
        hist.append(np.sqrt(S.dot(r, r)) / beta0)
        if fe < tol:
            return x, hist, (k - 1) * m + n_out
    return x, hist, (max_cycles - 1) * m + n_out
