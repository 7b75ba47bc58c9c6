"""Config 4 (8192^2, m = 95, MGS-R, 8 row-block ranks) on ONE GPU: one
restart cycle of a single-context 8192^2 run, then the same cycle as 8 slab
contexts joined by one of the two multi-rank transports:

  local  the in-process communicator (RCCL's message pattern: host barrier +
         device copies and sums; tests/test_gpu_configs.py runs it in-process)
  xchg   the device exchange (gk_xchg_local: tagged granules in every peer's
         receive region, k_xchg / k_xhalo spin-waiting on the device -- the
         transport of the 8-GPU bench).  Eight contexts of one process then
         spin on each other's granules from eight streams, which must run
         concurrently: test_gpu_configs.py starts this module as a child
         process with GPU_MAX_HW_QUEUES=16 (HIP's default of 4 hardware
         queues would serialise streams that share a queue).
  xchg-res  the device exchange with the resident step forced on
         (GK_TUNE_RES 1, GK_TUNE_RES_SHARE 8: 32 workgroups per rank): every
         Arnoldi step is ONE launch per rank whose 2j projections sum the 8
         rank totals inside the launch -- the in-launch cross-rank path the
         8-GPU run takes (there with 256 workgroups per rank).
  xchg-res-blk2  the same with the opt-in blocked-projection step (GK_TUNE_RES_BLOCK 2:
         one in-launch all-gather, and so one rank-total hop, per block of 2
         projections; exact-arithmetic MGS, pinned to the same reference cycle).

Prints one JSON line: the single run's and rank 0's residual / final_err,
whether every rank took identical decisions, and the largest deviations.
  python tests/config4_run.py local|xchg|xchg-res|xchg-res-blk2
"""
from __future__ import annotations

import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

N, M, R = 8192, 95, 8
CYCLES = 2  # the reference's own 8192^2 run is recorded for two cycles (tests/golden/make_ref_8192.py)


def run(transport: str, cycles: int = CYCLES) -> dict:
    import gmres_amd as ga
    from gmres_amd import _native as nat

    with ga.Context(N, M) as c:
        c.set_rhs_ones()
        ref = ga.gmres_mgsr(c, 1e-15, max_cycles=cycles, want_verr=False, want_hist=True)
        xref = c.get_x()
    parts = ga.slab_partition(N, R)
    g = ga.LocalGroup(R)
    ctxs = [ga.Context(N, M, device=0, line0=l0, nlines=nl) for l0, nl in parts]
    out, err = [None] * R, []
    try:
        ml = max(nl for _, nl in parts)
        for r, c in enumerate(ctxs):
            c.comm_init_local(g, r, ml)
        if transport.startswith("xchg"):
            for c in ctxs:
                c.xchg_local()
                c.tune(nat.GK_TUNE_XCHG_TIMEOUT_MS, 20000)
        if transport.startswith("xchg-res"):
            for c in ctxs:
                if transport == "xchg-res-blk2":
                    c.tune(nat.GK_TUNE_RES_BLOCK, 2)
                c.tune(nat.GK_TUNE_RES, 1)
                c.tune(nat.GK_TUNE_RES_SHARE, R)
                c.tune(nat.GK_TUNE_RES_TIMEOUT_MS, 20000)
        kinds = {c.comm_info()["kind"] for c in ctxs}
        plans = {c.res_info()["variant"] for c in ctxs}
        gs = {c.res_info()["G"] for c in ctxs}

        def work(r):
            try:
                ctxs[r].set_rhs_ones()
                ctxs[r].profile(True)
                ctxs[r].profile_reset()
                out[r] = (ga.gmres_mgsr(ctxs[r], 1e-15, max_cycles=cycles, want_verr=False, want_hist=True),
                          ctxs[r].profile_read())
            except Exception as e:  # reported below
                err.append(repr(e))

        th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        if err or any(o is None for o in out):
            return {"ok": False, "error": err or "a rank did not finish"}
        res = [o[0] for o in out]
        x = np.concatenate([o.x for o in res])
        return {
            "ok": True, "transport": transport, "comm_kinds": sorted(map(str, kinds)), "res_variants": sorted(map(str, plans)),
            "res_G": sorted(gs),
            "comm_launches": int(min(o[1]["comm"][1] for o in out)),
            "comm_launches_max": int(max(o[1]["comm"][1] for o in out)),
            "res_launches_min": int(min(o[1]["res"][1] for o in out)),
            "proj_launches_max": int(max(o[1]["proj"][1] for o in out)),
            "same_decisions": len({(o.n_out, o.cycles_out, o.n_cycles) for o in res}) == 1
            and all(np.array_equal(o.hist_res, res[0].hist_res) for o in res)
            and all(np.array_equal(o.final_err, res[0].final_err) for o in res),
            "n_out": res[0].n_out, "hist_res0": float(res[0].hist_res[0]), "ref_hist_res0": float(ref.hist_res[0]),
            "hist_res": [float(v) for v in res[0].hist_res], "ref_hist_res": [float(v) for v in ref.hist_res],
            "final_err_max_rel": float(np.max(np.abs(res[0].final_err[:M] - ref.final_err[:M]) / ref.final_err[:M])),
            "x_max_dev": float(np.max(np.abs(x - xref) / (1e-12 + 1e-9 * np.abs(xref)))),
        }
    finally:
        for c in ctxs:
            c.close()
        g.close()


if __name__ == "__main__":
    print(json.dumps(run(sys.argv[1] if len(sys.argv) > 1 else "local")), flush=True)
