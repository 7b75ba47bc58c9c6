#!/usr/bin/env python3
"""bench.py -- Arnoldi iterations/s and HBM GB/s of the MI355X GMRES(m) inner
cycle on the north-star workload (BASELINE.json): 4096^2 Poisson-2D fp64,
GMRES-MGSR, m = 95, b = A*1, x0 = 0.

One "step" = one full GMRES(m) restart cycle (cycle start + m Arnoldi steps +
back-solve + x update), run by the Fortran host over the HIP C-ABI exactly as
a solve does; K timed steps are K consecutive cycles of one solve.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 4096] [--m 95]
                  [--prec identity|cbpr2|cheb] [--method mgsr|hh] [--no-cpu]

N > 1 is launched by torch.distributed.run (one rank per GPU): the grid is
split into row-block slabs of grid lines; dot-product slabs are RCCL
all-reduced and halo lines exchanged inside libgmres_hip (one RCCL
communicator owned by the C-ABI context); torch.distributed (gloo) is used only
for bootstrapping the RCCL id, the barriers and the max-over-ranks timing.
Scaling is strong: the global grid is fixed as N grows.

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "Arnoldi iters/sec + HBM GB/s, 4096² Poisson-2D fp64, GMRES(m=95)"


def alg_bytes_cycle(n: int, m: int, prec: str, degree: int, steps: int | None = None) -> float:
    """SURVEY 8(d) byte model: the reference's op sequence as written, every
    vector operand read once and every result written once (fp64).
    per MGS-R step j: (40 + 80 j) n  [stencil 16n + 2j (dot 16n + AXPY 24n) + norm 8n + scale 16n];
    cycle start: (16 + 24 + 8 + 16) n; x update: 8 (m + 2) n;
    cbpr2 as written: +64 n per application; Chebyshev(k): 48 n per sweep
    (read d, r, z; write r, d, z) + 16 n stencil on entry, counted the same way."""
    s = m if steps is None else steps
    b = sum(40 + 80 * j for j in range(1, s + 1)) * n
    b += 64 * n + 8 * (m + 2) * n
    if prec == "cbpr2":
        b += 64 * n * (s + 1)
    elif prec == "cheb":
        b += (16 + 48 * degree) * n * (s + 1)
    return float(b)


def proj_alg_bytes(n: int, steps_js: list[int]) -> float:
    """Algorithmic bytes of the launches of the dominant kernel (fused
    projection): per step j, 2j launches; 2j-1 carry AXPY (24n) + dot (16n),
    the last AXPY (24n) + norm (8n)."""
    return float(sum((2 * j - 1) * 40 * n + 32 * n for j in steps_js))


def res_alg_bytes(n: int, j: int) -> float:
    """Algorithmic bytes of one resident-step launch (step j): the reference's
    MGS-R cascade as written, 2j x (dot 16n + AXPY 24n), + norm 8n + scale 16n
    (SURVEY 8(d) per-step model without the 16n stencil, which is its own launch)."""
    return float((80 * j + 24) * n)


def cpu_baseline(N: int, m: int, prec: str, degree: int, sample_steps: int, threads: int) -> dict:
    """Reference CPU path (the oracle, a loop-for-loop restatement of
    gmres_mgsr_omp) on this host: the first `sample_steps` Arnoldi steps of
    cycle 1 of the same workload; converted to full-cycle it/s through the
    same byte model (its per-step cost grows with j like the GPU's)."""
    from oracle import oracle as orc

    orc.build()
    b = orc.rhs_ones(N)
    kind = {"identity": orc.PREC_IDENTITY, "cbpr2": orc.PREC_CBPR2, "cheb": orc.PREC_CHEB}[prec]
    t0 = time.perf_counter()
    r = orc.gmres_mgsr(b, N, m, prec=kind, degree=degree, variant=orc.MGSR_OMP, max_cycles=1,
                       step_limit=sample_steps, threads=threads)
    t1 = time.perf_counter()
    st = r.step_times
    # per-step times from the oracle's own omp_get_wtime stamps
    dt = np.diff(st)
    steps_timed = list(range(2, sample_steps + 1))
    n = N * N
    bytes_timed = sum((40 + 80 * j) * n for j in steps_timed)
    if prec == "cbpr2":
        bytes_timed += 64 * n * len(steps_timed)
    elif prec == "cheb":
        bytes_timed += (16 + 48 * degree) * n * len(steps_timed)
    gbps = bytes_timed / dt.sum() / 1e9
    it_s = gbps * 1e9 / (alg_bytes_cycle(n, m, prec, degree) / m)
    return {"value": round(it_s, 4), "unit": "Arnoldi it/s", "cores": threads, "kind": "port",
            "gbps_alg": round(gbps, 2),
            "sample": f"oracle/gmres_oracle.c (gmres_mgsr_omp restatement, OpenMP {threads} threads) on "
                      f"{N}^2 m={m} prec={prec}: Arnoldi steps 2..{sample_steps} of cycle 1 "
                      f"({t1 - t0:.1f} s wall incl. setup), {gbps:.1f} GB/s algorithmic, scaled to a full "
                      f"cycle by the SURVEY 8(d) byte model"}


def setup_xgmi(ctx, dist, world: int, rank: int, required: bool):
    """Map every rank's exchange region (IPC handles over the gloo control
    plane) and run the collective self-test; every rank must pass, else all
    ranks fall back to RCCL (or fail when --collective xgmi was asked for)."""
    import torch

    ok = 1
    hs = [None] * world
    try:
        h = ctx.xchg_handle()
        dist.all_gather_object(hs, h)
        ctx.xchg_open(hs)
    except Exception as e:  # noqa: BLE001 - reported, then the self-test decides
        print(f"rank {rank}: device exchange unavailable: {e}", file=sys.stderr)
        ok = 0
    if ok:
        ok = int(ctx.xchg_selftest(5000))
        if not ok:
            print(f"rank {rank}: {getattr(ctx, 'xchg_error', '')}", file=sys.stderr)
    t = torch.tensor([ok], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if int(t.item()) == 1:
        return "xgmi-device-exchange"
    if required:
        raise RuntimeError("--collective xgmi: device exchange self-test failed")
    if ok:
        ctx.xchg_enable(False)
    return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--m", type=int, default=95)
    ap.add_argument("--prec", default="identity", choices=["identity", "cbpr2", "cheb"])
    ap.add_argument("--degree", type=int, default=8)
    ap.add_argument("--method", default="mgsr", choices=["mgsr", "hh"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=90)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-prof", action="store_true", help="no HIP-event kernel timing in the timed region")
    ap.add_argument("--collective", default="auto", choices=["auto", "rccl", "xgmi"],
                    help="N>1: RCCL calls, or the device exchange over xGMI (auto: device exchange if its "
                         "self-test passes on every rank, else RCCL)")
    ap.add_argument("--prof-every", type=int, default=16,
                    help="HIP events around the launches of every S-th Arnoldi step (1 = all)")
    args = ap.parse_args()

    import torch  # device plumbing + gloo control plane only

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")

    import gmres_amd as ga

    N, m = args.grid, args.m
    parts = ga.slab_partition(N, world)
    line0, nlines = parts[rank]
    ctx = ga.Context(N, m, device=local, line0=line0, nlines=nlines)
    ml = max(p[1] for p in parts)
    collective = None
    if world > 1 and args.collective == "xgmi":
        ctx.comm_init_xgmi(world, rank, ml)
    elif world > 1 or os.environ.get("GK_FORCE_RCCL") == "1":  # 1-rank RCCL: exercises the comm path
        obj = [ga.Context.unique_id() if rank == 0 else None]
        if dist is not None:
            dist.broadcast_object_list(obj, src=0)
        ctx.comm_init(world, rank, ml, obj[0])
        collective = "rccl"
    if world > 1 and args.collective in ("auto", "xgmi"):
        collective = setup_xgmi(ctx, dist, world, rank, required=args.collective == "xgmi") or "rccl"
    ctx.set_precond(args.prec, (8.2, 0.2), args.degree)
    ctx.set_rhs_ones()

    def run(cycles: int):
        if args.method == "mgsr":
            return ga.gmres_mgsr(ctx, 1e-15, max_cycles=cycles, want_verr=False)
        return ga.gmres_hh(ctx, 1e-15, precondition=(args.prec != "identity"), max_cycles=cycles,
                           want_verr=False)

    def barrier():
        ctx.sync()
        torch.cuda.synchronize(local)
        if dist is not None:
            dist.barrier()

    def guarded_warmup() -> bool:
        ok = 1
        try:
            if args.warmup > 0:
                run(args.warmup)
        except Exception as e:  # noqa: BLE001 - every rank reports, then all agree below
            print(f"rank {rank}: warmup failed: {e}", file=sys.stderr)
            ok = 0
        if dist is not None:
            t = torch.tensor([ok], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = int(t.item())
        return ok == 1

    if not guarded_warmup():
        # Fallback, decided by all ranks together: the launch-per-projection path
        # (and RCCL instead of the device exchange when that was in use).
        if collective == "xgmi-device-exchange" and args.collective == "auto":
            ctx.xchg_enable(False)
            collective = "rccl (device exchange failed in warmup)"
        ctx.tune(8, 0)  # GK_TUNE_RES off
        if not guarded_warmup():
            raise RuntimeError("warmup failed on the fallback path too")
    if not args.no_prof:
        ctx.profile(1 if args.method == "hh" else max(1, args.prof_every))
        ctx.profile_reset()
    barrier()
    t0 = time.perf_counter()
    res = run(args.steps)
    barrier()
    t1 = time.perf_counter()
    prof = ctx.profile_read() if not args.no_prof else {}
    resid = ctx.true_residual()  # outside the timed region; same value at any N
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    cycles = res.n_cycles
    iters = (cycles - 1) * m + res.n_out if cycles > 0 else 0

    if rank == 0:
        n = N * N
        nloc = ctx.nloc
        it_s = iters / elapsed
        bytes_cycle = alg_bytes_cycle(n, m, args.prec, args.degree)
        gbps_alg = bytes_cycle * cycles / elapsed / 1e9 if cycles == args.steps else None
        roof = None
        if prof and prof.get("res", (0.0, 0))[1] > 0:
            # resident MGS-R step: one launch = the 2j projections + norm + scale of step j
            ms, launches = prof["res"]
            if args.method == "hh":
                # every launch sampled (profile(1)): per step j a RES_HH_DOWN chain (v_j = P_1..P_j e_j)
                # and a RES_HH_UP chain (w = P_j..P_1 A v_j), j reflections of 40n each
                # (gmres_hh.f90:269-304); per cycle one more chain of n_out = m (x update, :361-373)
                steps_js = list(range(1, m + 1)) * cycles
                palg = float(sum(2 * j * 40 * nloc for j in steps_js) + cycles * m * 40 * nloc)
                nproj = sum(2 * j for j in steps_js) + cycles * m
                kname = ("gk::k_mgs_res / k_mgs_wres in reflection mode (RES_HH_DOWN / RES_HH_UP: a chain of j "
                         "Householder reflections, one persistent launch per chain)")
                timing = "HIP events on the context stream around every resident launch of the timed cycles"
            else:
                S = max(1, args.prof_every)
                steps_js = [j for j in range(1, m + 1) if j % S == 0] * cycles
                palg = float(sum(res_alg_bytes(nloc, j) for j in steps_js))
                nproj = sum(2 * j + 1 for j in steps_js)
                kname = ("gk::k_mgs_res (resident MGS-R step: 2j fused projections + norm + scale, one "
                         "persistent launch per Arnoldi step)")
                timing = (f"HIP events on the context stream around the step launch of steps j % {S} == 0 "
                          f"of the timed cycles")
            achieved = palg / (ms / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                    "kernel": kname,
                    "launches": launches, "avg_launch_us": round(ms * 1e3 / launches, 2),
                    "alg_bytes_per_launch": round(palg / launches),
                    "per_projection_us": round(ms * 1e3 / nproj, 2),
                    "timing": timing,
                    "per_kernel_ms_sampled": {k: round(v[0], 3) for k, v in prof.items()}}
            tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            key = f"{N}_{m}_{args.prec}_{args.method}_{world}_res"
            if os.path.exists(tf):
                pm = json.load(open(tf))
                if key in pm:
                    # PMC bytes per launch are linear in the projection count: a + b 2j
                    a0, b0 = pm[key]["bytes_fixed"], pm[key]["bytes_per_projection"]
                    tb = sum(a0 + b0 * 2 * j for j in steps_js) / len(steps_js)
                    roof["traffic"] = round(tb)
                    roof["traffic_source"] = pm[key]["source"]
                    roof["physical"] = {"fabric_GBps": round(tb * launches / (ms / 1e3) / 1e9, 1),
                                        "bytes_per_projection": round(b0)}
        elif prof and prof["proj"][1] > 0:
            ms, launches = prof["proj"]
            S = 1 if args.method == "hh" else max(1, args.prof_every)
            steps_js = [j for j in range(1, m + 1) if j % S == 0] * cycles
            if args.method == "hh":
                # HH: 2j reflections/step (j on v_j incl. a leading dot, j on w), 40n each
                palg = float(sum(2 * j * 40 * nloc for j in steps_js))
            else:
                palg = proj_alg_bytes(nloc, steps_js)
            achieved = palg / (ms / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                    "kernel": "gk::k_proj (fused MGS-R AXPY_i + dot_{i+1})", "launches": launches,
                    "avg_launch_us": round(ms * 1e3 / launches, 2),
                    "alg_bytes_per_launch": round(palg / launches),
                    "timing": f"HIP events on the context stream around every launch of steps j % {S} == 0 "
                              f"of the timed cycles (launch cost is independent of j)",
                    "per_kernel_ms_sampled": {k: round(v[0], 3) for k, v in prof.items()}}
            tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(tf):
                try:
                    pm = json.load(open(tf))
                    key = f"{N}_{m}_{args.prec}_{args.method}_{world}"
                    if key in pm:
                        tb = pm[key]["hbm_bytes_per_launch"]
                        roof["traffic"] = round(tb)
                        roof["traffic_source"] = pm[key]["source"]
                        avg_s = ms / 1e3 / launches
                        roof["physical"] = {
                            "fabric_GBps": round(tb / avg_s / 1e9, 1),
                            "fabric_frac_of_hbm_peak": round(tb / avg_s / 1e9 / HBM_PEAK_GBPS, 4),
                            "note": "frac > 1 is algorithmic: the reference's op sequence moves 40 B/unknown per "
                                    "dot+AXPY pair, the fused kernel moves 32 B/unknown (traffic), and w "
                                    "(128 MiB at 4096^2) is re-read from the 256 MiB Infinity Cache"}
                except Exception:
                    pass
        cpu = None
        if not args.no_cpu and world == 1:
            thr = args.cpu_threads or min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(N, m, args.prec, args.degree, args.cpu_steps, thr)
        prec_name = {"identity": "no precond", "cbpr2": "cbpr2", "cheb": f"Chebyshev({args.degree})"}[args.prec]
        out = {
            "metric": METRIC,
            "value": round(it_s, 4),
            "unit": "Arnoldi it/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(cycles, 1) * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: b = A*1 (the reference drivers' manufactured RHS), x0 = 0, tol 1e-15",
            "config": {"workload": f"{N}x{N} Poisson-2D fp64, GMRES-{args.method.upper()} m={m}, {prec_name}",
                       "grid": N, "m": m, "precond": args.prec, "method": args.method,
                       "step": "one GMRES(m) restart cycle", "parallelism": f"row-block slabs x{world}",
                       "collective": collective, "arnoldi_iters": iters},
            "check": {"true_rel_residual_after_timed_cycles": resid},
            "hbm_gbps_alg": round(gbps_alg, 1) if gbps_alg else None,
            "cycle_roofline_frac": round(gbps_alg / HBM_PEAK_GBPS, 4) if gbps_alg else None,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
