"""Per-collective cost of the multi-rank paths on ONE GPU (tiny grid, so the
kernels themselves are negligible): time one GMRES(95) cycle of the
N=128 grid split over R in-process ranks, with the host-side local group
(host barrier + events, RCCL's message pattern) and with the device exchange,
against the single-context cycle.  A cycle issues ~m(m+2) = 9,215 slab
all-reduces and 95-190 halo exchanges."""
import json
import sys
import threading
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import gmres_amd as ga  # noqa: E402

N, m, CYC = 128, 95, 3


def single():
    with ga.Context(N, m) as c:
        c.set_rhs_ones()
        ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)
        t = time.perf_counter()
        ga.gmres_mgsr(c, 1e-15, max_cycles=CYC, want_verr=False)
        return (time.perf_counter() - t) / CYC


def group(R, xgmi):
    parts = ga.slab_partition(N, R)
    ml = max(nl for _, nl in parts)
    g = ga.LocalGroup(R)
    ctxs = [ga.Context(N, m, line0=l0, nlines=nl) for l0, nl in parts]
    for r, c in enumerate(ctxs):
        c.comm_init_local(g, r, ml)
    if xgmi:
        for c in ctxs:
            c.xchg_local()
    bar = threading.Barrier(R)
    out = [0.0] * R

    def work(r):
        c = ctxs[r]
        c.set_rhs_ones()
        ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)
        bar.wait()
        t = time.perf_counter()
        ga.gmres_mgsr(c, 1e-15, max_cycles=CYC, want_verr=False)
        c.sync()
        out[r] = (time.perf_counter() - t) / CYC

    th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in ctxs:
        c.close()
    g.close()
    return max(out)


if __name__ == "__main__":
    res = {"grid": N, "m": m, "single_ms_per_cycle": round(single() * 1e3, 2)}
    for R in (2, 3):
        for xg in (False, True):
            res[f"R{R}_{'xgmi' if xg else 'host_group'}_ms_per_cycle"] = round(group(R, xg) * 1e3, 2)
    nred = m * (m + 2)
    for k in list(res):
        if k.startswith("R"):
            res[k.replace("ms_per_cycle", "extra_us_per_allreduce")] = round(
                (res[k] - res["single_ms_per_cycle"]) * 1e3 / nred, 2)
    print(json.dumps(res), flush=True)
