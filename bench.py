#!/usr/bin/env python3
"""bench.py -- Arnoldi iterations/s and HBM GB/s of the MI355X GMRES(m) inner
cycle on the north-star workload (BASELINE.json): 4096^2 Poisson-2D fp64,
GMRES-MGSR, m = 95, b = A*1, x0 = 0.

One "step" = one full GMRES(m) restart cycle (cycle start + m Arnoldi steps +
back-solve + x update), run by the Fortran host over the HIP C-ABI exactly as
a solve does; K timed steps are K consecutive cycles of one solve.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 4096] [--m 95]
                  [--prec identity|cbpr2|cheb] [--method mgsr|hh] [--no-cpu]
                  [--plan-only]

--gpus N > 1: one rank per GPU.  Launched under torch.distributed.run (the
driver's way) the ranks read RANK/LOCAL_RANK/WORLD_SIZE; launched directly
(WORLD_SIZE unset) bench.py starts torch.distributed.run itself as a child
process -- before anything touches a GPU -- and exits with its status; it
refuses (exit 2) when fewer than N GPUs are visible.  --plan-only prints that
launch plan as JSON and exits.  The grid is split into row-block slabs of grid
lines (strong scaling: the global grid is fixed as N grows); per projection
the dot products are all-reduced inside libgmres_hip (device exchange over
xGMI, or RCCL), halo lines exchanged point to point; a small TCP control
plane on the loopback interface (gmres_amd/ctl.py) only bootstraps the
communicator and times max-over-ranks.  No rank imports torch: the library
runs on the HIP runtime and RCCL it was built against (config.runtime).

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; ~6.3 TB/s achievable)
FABRIC_REF_GBPS = 8600.0  # Infinity-Cache-resident reads chip-wide (MI355X_MICROARCH.md, indexed-rows table)
METRIC = "Arnoldi iters/sec + HBM GB/s, 4096² Poisson-2D fp64, GMRES(m=95)"


# ------------------------------------------------------------- byte models ---
# Two models per launch / per cycle:
#  * as written: the reference's op sequence, every BLAS-1 op
#    reading its operands and writing its result once -- dot 16n, AXPY 24n,
#    norm 8n, scale 16n.  A fused kernel beats it, so its "fraction" can
#    exceed 1: reported as alg_as_written_*, never as roofline.frac.
#  * fused minimum: what the fused schedule must move at least with w held on
#    chip -- per MGS projection (AXPY_i fused with dot_{i+1}) the two Krylov
#    columns it touches, 16n; per resident step launch (32j + 16) n (2j
#    projections + reading w once + writing V(:,j+1)).  roofline.frac uses it.

def mgs_step_bytes(n: int, j: int, model: str) -> float:
    """One resident MGS-R step launch (cascade + norm + scale); the stencil is
    its own launch."""
    if model == "as_written":
        return float((80 * j + 24) * n)
    return float((32 * j + 16) * n)


def res_regions(plan: dict, nloc: int) -> dict:
    """How a resident launch holds the slab (gk_res_info): unknowns whose w AND
    running Krylov column sit on chip ("pairs": the pairs / prefetch variants,
    and the w+column variant's cached chunks), unknowns whose w alone is on chip
    (registers of the w-only variant, or LDS), and the streamed rest.  Chunks of
    DT double2: 256 (w-only, w+column), 448 (prefetch, one control wave), 512
    (pairs); w+column: the plan's "wt" (512 since round 4's two-wave build)."""
    n2 = nloc // 2
    var = plan["variant"]
    if var == "blocked":  # k_mgs_blk: the w-only build (no block cache) or a block-cache build
        # (the one-wave S = 4 build also runs 256 threads, with its whole block cached)
        var = "w-only" if int(plan["r2"]) + int(plan["l2"]) == 0 else "w+column"
    dt = 256 if var in ("w-only", "w+column") else (448 if plan.get("cw") else 512)
    if var in ("w-only", "w+column") and plan.get("wt"):
        dt = int(plan["wt"])  # threads per workgroup = double2 per chunk
    nres2 = min(int(plan["nres2"]), n2)
    nreg2 = min(nres2, int(plan["G"]) * int(plan["r2e"]) * dt)
    if var == "w-only":
        return {"pairs": 0, "w_on_chip": 2 * nres2, "streamed": 2 * (n2 - nres2) + (nloc & 1)}
    if var == "w+column":  # w in registers; the column (blocked: each block slot) of r2 + l2 chunks cached
        cached = min(nres2, int(plan["G"]) * min(int(plan["r2e"]), int(plan["r2"]) + int(plan["l2"])) * dt)
        return {"pairs": 2 * cached, "w_on_chip": 2 * (nres2 - cached), "streamed": 2 * (n2 - nres2) + (nloc & 1)}
    return {"pairs": 2 * nreg2, "w_on_chip": 2 * (nres2 - nreg2), "streamed": 2 * (n2 - nres2) + (nloc & 1)}


def res_launch_bytes(plan: dict, nloc: int, P: int, mgs: bool = True) -> float:
    """Compulsory bytes of ONE resident launch of the selected variant running P
    passes (an MGS-R step: P = 2j, the last one closing with ||w||; a Householder
    chain: P = L reflections), per unknown of each region (res_regions):
      pairs       w in 8, one Krylov column per pass (the AXPY partner of pass
                  p+1 is pass p's dot partner, still in registers): 8P, out 8
                  -> 8P + 16
      w on chip   w in 8, both columns of every pass but the last (no dot
                  partner) 16P - 8, out 8 -> 16P + 8
      streamed    w read + written, both columns, every pass: 32P - 8; the MGS
                  step then reads w once more and writes V(:,j+1): +16"""
    r = res_regions(plan, nloc)
    b = r["pairs"] * (8 * P + 16) + r["w_on_chip"] * (16 * P + 8) + r["streamed"] * (32 * P - 8 + (16 if mgs else 0))
    return float(b)


def hh_chain_bytes(n: int, L: int, model: str) -> float:
    """One resident Householder chain of L reflections w -= 2<w,P_i>P_i."""
    return float(40 * L * n if model == "as_written" else (16 * L + 16) * n)


def prec_bytes(n: int, prec: str, degree: int, model: str, cheb_sten: bool = True) -> float:
    """One preconditioner application after the stencil (z = A v already made).
    cheb_sten: the Arnoldi step's Chebyshev pass forms z = A v in its own stage
    0 (gk_res_info "cheb_sten"; off with GK_TUNE_CHEB_STEN 0, N < 128, k > 8,
    or a slab thinner than k + 1 lines)."""
    if prec == "identity":
        return 0.0
    if prec == "cbpr2":
        return float(64 * n if model == "as_written" else 16 * n)
    # Chebyshev(k): 48n per sweep as written; fused, k <= 8 sweeps are ONE
    # temporal-blocked pass.  With the stencil as its stage 0 it reads v, writes
    # the result and reads the dot partner -- the 24n the stencil term already
    # counts, so +0; after a stencil launch it reads z and writes the result
    # (+16n).  Each further pass of up to 8 hands over (d, r, z): +48n.
    passes = (degree + 7) // 8
    if model == "as_written":
        return float(48 * degree * n)
    return float(((0 if (passes == 1 and cheb_sten) else 16) + 48 * (passes - 1)) * n)


def cycle_bytes(n: int, m: int, prec: str, degree: int, method: str, model: str, cheb_sten: bool = True) -> float:
    """One full restart cycle of m Arnoldi steps."""
    if model == "as_written":  # per step (40 + 80 j) n, cycle start 64n, update 8(m+2)n
        if method == "hh":
            b = sum((64 + 80 * j) * n for j in range(1, m + 1)) + 64 * n + 8 * (m + 2) * n + 40 * m * n
        else:
            b = sum((40 + 80 * j) * n for j in range(1, m + 1)) + 64 * n + 8 * (m + 2) * n
        return float(b + (m + 1) * prec_bytes(n, prec, degree, model))
    st = 24 * n  # stencil fused with the first dot: read V_j and V_1, write w
    if method == "hh":
        b = sum(hh_chain_bytes(n, j, model) * 2 + st + 40 * n for j in range(1, m + 1))
        b += hh_chain_bytes(n, m, model) + 24 * n + 40 * n
    else:
        b = sum(mgs_step_bytes(n, j, model) + st for j in range(1, m + 1))
        b += 40 * n + 8 * (m + 2) * n  # cycle start (b - A x, norm, V_1) + x update
    # the cycle start's application runs after a stencil launch (never stage-0 fused)
    return float(b + m * prec_bytes(n, prec, degree, model, cheb_sten) + prec_bytes(n, prec, degree, model, False))


# ------------------------------------------------------------- CPU baseline ---
def cpu_info() -> dict:
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    share = min(aff, int(omp)) if omp.isdigit() and int(omp) > 0 else aff
    return {"nproc": os.cpu_count(), "affinity": aff, "OMP_NUM_THREADS": omp or None, "cpu_model": model,
            "omp_threads": share,
            "omp_threads_note": "the CPU share this process is granted: min(affinity mask, OMP_NUM_THREADS); on "
                                "the GPU box OMP_NUM_THREADS=16 is the harness's per-GPU CPU share of a larger "
                                "host, so the sweep stops there (nproc / affinity show the whole machine)"}


def _extrapolate(step_t: dict, c0: float, m: int) -> tuple[float, str]:
    """Cycle time from step stamps of a cut run: step durations d_j = t_{j+1}
    - t_j are linear in j (2j dot+AXPY pairs); least-squares a + b j over the
    sampled steps, summed over j = 1..m, plus the cycle start as measured and
    the x update priced at (m+2)/10 of one (dot+AXPY pair) increment b."""
    js = sorted(step_t)
    d = {j: step_t[j + 1] - step_t[j] for j in js if j + 1 in step_t}
    xs = np.array(sorted(d), dtype=float)
    ys = np.array([d[int(j)] for j in xs])
    if len(xs) >= 3:
        b, a = np.polyfit(xs[1:], ys[1:], 1)  # step 1 pays first touches
    else:
        b, a = 0.0, float(ys.mean())
    start = step_t[js[0]] - c0
    t = start + sum(a + b * j for j in range(1, m + 1)) + max(b, 0.0) * (m + 2) / 10.0
    return float(t), f"steps 1..{int(xs[-1]) + 1} timed, step cost fitted a + b j (a={a:.4g} s, b={b:.4g} s)"


def sweep_threads(share: int) -> list[int]:
    """The reference's strong-scaling pattern (tests/strong_scaling.f90:44-55:
    1, 2, 4, 8, 16 threads), capped at this process's CPU share, which is
    always the last point."""
    ts = [t for t in (1, 2, 4, 8, 16) if t < share]
    return ts + [share]


def cpu_baseline(N: int, m: int, prec: str, degree: int, method: str, cap_full: float, steps: int) -> dict:
    """The reference CPU path timed on this host (rank 0, N = 1 only):
    oracle/_ref/ref_driver = the reference's own gmres_mgsr_omp / gmres_hh_omp
    (kind "reference"); Chebyshev(k) does not exist in the reference, so that
    config times the restatement (kind "port").  Thread sweep in the
    reference's own strong-scaling pattern (1, 2, 4, 8, 16 threads, capped at
    the process's OpenMP share; OMP_PROC_BIND=close, OMP_PLACES=cores).  Every
    leg, the share included, times the SAME window -- Arnoldi steps 1..`steps`
    of cycle 1 from x0 = 0, stamped by omp_get_wtime -- and prices the cycle
    identically: step cost fitted a + b j over steps 2..`steps` (step 1 pays the
    solve's first touches), summed over j = 1..m.  `value` is the fastest leg.
    The share also runs one full cycle when it fits cap_full seconds: a check
    of the fit (`full_cycle_check`), not the value."""
    from oracle import refrun

    info = cpu_info()
    env = {"OMP_PROC_BIND": "close", "OMP_PLACES": "cores"}
    legs = []
    use_ref = refrun.available() and prec in ("identity", "cbpr2")
    solver = ("hh_omp" if prec == "identity" else "hh_prec_omp") if method == "hh" else "mgsr_omp"
    share = info["omp_threads"]

    def leg(thr: int, step_limit: int):
        if use_ref:
            r = refrun.run(solver, N, m, prec, threads=thr, max_cycles=1, step_limit=step_limit, env=env,
                           timeout=900)
            return r.step_t, r.cycle_t, r.threads
        from oracle import oracle as orc

        kind = {"identity": orc.PREC_IDENTITY, "cbpr2": orc.PREC_CBPR2, "cheb": orc.PREC_CHEB}[prec]
        rr = orc.gmres_mgsr(orc.rhs_ones(N), N, m, prec=kind, degree=degree, variant=orc.MGSR_OMP,
                            max_cycles=1, step_limit=step_limit or m, threads=thr)
        st = {j + 1: float(t) for j, t in enumerate(rr.step_times) if t > 0}
        return st, [0.0], thr

    for thr in sweep_threads(share):
        t0 = time.perf_counter()
        step_t, cycle_t, thr_used = leg(thr, steps)
        t_cyc, how = _extrapolate(step_t, cycle_t[0], m)
        legs.append({"threads": thr_used, "cycle_s": round(t_cyc, 3), "it_s": round(m / t_cyc, 4), "how": how,
                     "wall_s": round(time.perf_counter() - t0, 1)})
    best = max(legs, key=lambda d: d["it_s"])
    check = None
    if use_ref and cap_full > 0 and legs[-1]["cycle_s"] <= cap_full:
        t0 = time.perf_counter()
        r = refrun.run(solver, N, m, prec, threads=share, max_cycles=1, env=env, timeout=cap_full + 600)
        if len(r.cycle_t) >= 2:
            full = r.cycle_t[1] - r.cycle_t[0]
            check = {"threads": r.threads, "cycle_s": round(full, 3), "it_s": round(m / full, 4),
                     "fit_over_full": round(legs[-1]["cycle_s"] / full, 4),
                     "how": "one full cycle (omp_get_wtime stamps of cycles 1 and 2)",
                     "wall_s": round(time.perf_counter() - t0, 1)}
    # value: the measured full cycle when it ran (the fit understated
    # the reference by 10.7 %); the a + b j fit of the fastest sweep leg otherwise
    if check is not None and check["it_s"] >= best["it_s"] * 0.5:
        value, cores, how = check["it_s"], check["threads"], "full_cycle_check (one measured cycle)"
    else:
        value, cores, how = best["it_s"], best["threads"], f"fit of the fastest sweep leg ({best['threads']} threads)"
    return {"value": value, "unit": "Arnoldi it/s", "cores": cores, "value_from": how,
            "kind": "reference" if use_ref else "port",
            "sample": (f"{'oracle/_ref/ref_driver (the reference src/*.f90 built by oracle/Makefile.ref)' if use_ref else 'oracle/gmres_oracle.c (restatement; Chebyshev(k) is not in the reference)'} "
                       f"{solver} on {N}^2 m={m} prec={prec}, b = A*1, x0 = 0; thread sweep "
                       f"{[d['threads'] for d in legs]} (the reference's strong-scaling pattern, capped at the "
                       f"process's OpenMP share of {share}); every leg times Arnoldi steps 1..{steps} of cycle 1 "
                       f"and prices the cycle by the same a + b j fit; value = one measured full cycle at the "
                       f"share when it fits the cap, else the fastest leg's fit"),
            "sweep": legs, "full_cycle_check": check,
            "hbm_gbps_alg_as_written": round(cycle_bytes(N * N, m, prec, degree, method, "as_written")
                                             * value / m / 1e9, 1),
            "host": info, "calibration": "profiles/r02/cpu_calibration.json"}


# ------------------------------------------------------------- launcher -----
def _free_port() -> int:
    """A port for the self-launched rendezvous, below the kernel's ephemeral range
    (32768-60999 by default): an ephemeral port that probed free can be taken by
    a client connection (or sit in TIME_WAIT after the previous run's ranks) by
    the time torch.distributed.run's store binds it (EADDRINUSE, seen r04t)."""
    import random

    rng = random.Random(os.getpid() ^ int(time.time() * 1e6))
    for _ in range(200):
        port = rng.randrange(20000, 32000)
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus: int, argv: list[str]) -> dict:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
    cmd += [a for a in argv if a != "--plan-only"]
    return {"launcher": "torch.distributed.run", "ranks": gpus, "cmd": cmd,
            "env": {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}}


def visible_gpus() -> int:
    """GPUs this process can open, counted WITHOUT the HIP runtime (the
    launcher touches nothing GPU-side before its ranks start): the KFD topology
    nodes with a non-zero gpu_id whose DRM render node /dev/dri/renderD<minor>
    exists and is readable + writable here (a container sees the host's whole
    topology in sysfs but only its own render nodes), capped by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        nodes = os.listdir(base)
    except OSError:
        nodes = []
    for d in nodes:
        try:
            if int(open(os.path.join(base, d, "gpu_id")).read().strip() or "0") == 0:
                continue
            minor = None
            for line in open(os.path.join(base, d, "properties")):
                k, _, v = line.partition(" ")
                if k == "drm_render_minor":
                    minor = int(v)
            dev = f"/dev/dri/renderD{minor}" if minor is not None else None
            if dev is None or os.access(dev, os.R_OK | os.W_OK):
                n += 1
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def maybe_self_launch(args, argv: list[str]) -> None:
    """N > 1 without a launcher: start one rank per GPU as child processes
    (never exec from a process that may have touched the GPU) and exit with
    their status."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        if args.plan_only:
            print(json.dumps({"launcher": None, "ranks": int(os.environ.get("WORLD_SIZE", "1"))}))
            sys.exit(0)
        return
    plan = launch_plan(args.gpus, argv)
    if args.plan_only:
        print(json.dumps(plan))
        sys.exit(0)
    vis = visible_gpus()
    if vis < args.gpus and os.environ.get("GK_BENCH_SAME_DEVICE") != "1":
        print(f"bench.py: --gpus {args.gpus} but only {vis} GPU(s) visible", file=sys.stderr)
        sys.exit(2)
    p = subprocess.run(plan["cmd"], env=rank_env(os.environ, plan["env"]))
    sys.exit(p.returncode)


def rank_env(environ, plan_env: dict) -> dict:
    """The rank processes' environment.  The N-rank rehearsal on ONE device
    (GK_BENCH_SAME_DEVICE=1) gets one hardware queue per rank process, so the N
    processes' queues do not oversubscribe the device's scheduler (8 x the default
    4 hung the 8-process rehearsal in round 4 and ran its warmup 50x slow in r05y;
    8 x 1 runs, resident steps too: profiles/r05/reh8_same_device_r05_note.txt).
    It overrides an inherited GPU_MAX_HW_QUEUES (the GPU box exports 4);
    GK_BENCH_SAME_DEVICE_QUEUES picks another count."""
    env = dict(environ, **plan_env)
    if environ.get("GK_BENCH_SAME_DEVICE") == "1":
        env["GPU_MAX_HW_QUEUES"] = environ.get("GK_BENCH_SAME_DEVICE_QUEUES", "1")
    return env


# ------------------------------------------------------------- first contact
def first_contact_record(ctx, ctl, rank: int, world: int, device: int) -> dict:
    """N > 1: what every rank saw of the others before the
    timed region -- per ordered rank pair, hipDeviceCanAccessPeer and
    hipExtGetLinkTypeAndHopCount between their devices; per rank, the device
    exchange self-test's wall time (every rank's granules through every peer's
    region: a round trip to each peer) and its outcome; gathered on rank 0."""
    import gmres_amd as ga

    devs = ctl.allgather(device)
    pairs = []
    for q, d in enumerate(devs):
        if q == rank:
            continue
        try:
            pi = ga.peer_info(device, d)
            pairs.append([rank, q, device, d, int(pi["can_access_peer"]), pi["link_type"], pi["hops"]])
        except Exception as e:  # noqa: BLE001 - recorded, never fatal
            pairs.append([rank, q, device, d, None, repr(e)[:80], None])
    mine = {"rank": rank, "device": device, "selftest_ms": getattr(ctx, "selftest_ms", None),
            "selftest_error": getattr(ctx, "xchg_error", None), "pairs": pairs}
    allr = ctl.allgather(mine)
    return {"pairs_columns": ["rank", "peer_rank", "device", "peer_device", "can_access_peer", "link_type", "hops"],
            "pairs": [p for r in allr for p in r["pairs"]],
            "selftest_ms": [r["selftest_ms"] for r in allr],
            "selftest_errors": [r["selftest_error"] for r in allr],
            "same_device_rehearsal": len(set(devs)) == 1}


def comm_ranks_note(comm: dict, world: int, collective) -> str | None:
    """comm_ranks_seen must equal N; when it does not, the line says why."""
    seen = comm.get("nranks")
    if seen == world:
        return None
    if world == 1:
        return "single rank: no communicator" if not seen else None
    return (f"the communicator reports {seen} rank(s) for a {world}-rank launch (collective {collective!r}): the "
            f"collective was not set up on every rank -- this line is not an N-GPU measurement")


# ------------------------------------------------------------- device exchange
def setup_xgmi(ctx, ctl, rank: int, required: bool):
    """Map every rank's exchange region (IPC handles over the control plane,
    gmres_amd/ctl.py) and run the collective self-test; every rank must pass,
    else all ranks fall back to RCCL (or fail when --collective xgmi was asked
    for, or when there is no RCCL communicator to fall back to)."""
    ok = 1
    try:
        hs = ctl.allgather(ctx.xchg_handle())
        ctx.xchg_open(hs)
    except Exception as e:  # noqa: BLE001 - reported, then the self-test decides
        print(f"rank {rank}: device exchange unavailable: {e}", file=sys.stderr)
        ok = 0
    if ok:
        t0 = time.perf_counter()
        ok = int(ctx.xchg_selftest(5000))
        ctx.selftest_ms = round((time.perf_counter() - t0) * 1e3, 3)  # the bench line's first-contact record
        if not ok:
            print(f"rank {rank}: {getattr(ctx, 'xchg_error', '')}", file=sys.stderr)
    if ctl.allreduce(ok, "min") == 1:
        return "xgmi-device-exchange"
    if required:
        raise RuntimeError("device exchange self-test failed on some rank (and no RCCL fallback: --collective xgmi, "
                           "or the RCCL communicator failed too)")
    if ok:
        ctx.xchg_enable(False)
    return None


def roofline_entry(prof: dict, args, nloc: int, cycles: int, world: int, plan: dict | None = None) -> dict | None:
    """Dominant kernel: its compulsory bytes per launch over its average launch
    time from HIP events on the context stream.  `plan` = gk_res_info of the
    timed context (the resident variant the launches ran: its bytes are
    res_launch_bytes)."""
    m = args.m
    on_res = bool(prof) and prof.get("res", (0.0, 0))[1] > 0 and plan is not None and plan.get("variant")
    if not on_res:
        if not prof or (prof["proj"][1] == 0 and prof.get("graph", (0.0, 0))[1] == 0):
            return None
        # launch-per-projection path (RCCL multi-rank, or after a fallback)
        S = 1 if args.method == "hh" else max(1, args.prof_every)
        steps_js = [j for j in range(1, m + 1) if j % S == 0] * cycles
        nproj = sum(2 * j for j in steps_js)
        fused, written = 32.0 * nloc * nproj, 40.0 * nloc * nproj
        if prof.get("graph", (0.0, 0))[1] > 0 and args.method == "mgsr":  # the step replayed as a hipGraph
            ms, launches = prof["graph"]
            fused += sum(16.0 * nloc for _ in steps_js)  # + the normalisation (w in, V(:,j+1) out)
            kname = ("hipGraph of a launch-path MGS-R step (2j gk::k_proj launches with their 2j + 1 all-reduces "
                     "and k_scale, captured once per j, GK_TUNE_GRAPH)")
            timing = f"HIP events around every replayed step graph of steps j % {S} == 0 of the timed cycles"
        else:
            ms, launches = prof["proj"]
            kname = "gk::k_proj (AXPY_i fused with dot_{i+1}, one launch per projection)"
            timing = f"HIP events around every projection launch of steps j % {S} == 0 of the timed cycles"
        per_proj = ms * 1e3 / nproj
        variant, regions, bound, peak = "launch-per-projection", None, "hbm", HBM_PEAK_GBPS
        model = "32 B per unknown per projection (w read + written, both Krylov columns)"
    else:
        ms, launches = prof["res"]
        variant = plan["variant"]
        regions = res_regions(plan, nloc)
        if args.method == "hh":
            steps_js = list(range(1, m + 1)) * cycles
            chains = [j for j in steps_js for _ in (0, 1)] + [m] * cycles
            fused = sum(res_launch_bytes(plan, nloc, L, mgs=False) for L in chains)
            written = sum(hh_chain_bytes(nloc, L, "as_written") for L in chains)
            nproj = sum(chains)
            kname = ("gk::k_mgs_wres / k_mgs_res in reflection mode (RES_HH_DOWN / RES_HH_UP: a chain of j "
                     "Householder reflections per persistent launch)")
            timing = "HIP events on the context stream around every resident launch of the timed cycles"
        else:
            S = max(1, args.prof_every)
            steps_js = [j for j in range(1, m + 1) if j % S == 0] * cycles
            fused = sum(res_launch_bytes(plan, nloc, 2 * j, mgs=True) for j in steps_js)
            written = sum(mgs_step_bytes(nloc, j, "as_written") for j in steps_js)
            nproj = sum(2 * j for j in steps_js)
            kname = ("gk::k_mgs_wres / k_mgs_wpc / k_mgs_res (resident MGS-R step: 2j fused projections + norm + "
                     "scale, one persistent launch per Arnoldi step)")
            if variant == "blocked":
                kname = (f"gk::k_mgs_blk (blocked-projection MGS-R step, GK_TUNE_RES_BLOCK {plan.get('blk')}: the 2j "
                         f"projections in blocks of {plan.get('blk')}, one in-launch all-gather per block; one "
                         "persistent launch per Arnoldi step)")
            timing = f"HIP events on the context stream around the step launch of steps j % {S} == 0 of the timed cycles"
        per_proj = ms * 1e3 / nproj
        model = ("compulsory bytes of the selected resident variant (bench.res_launch_bytes, DESIGN.md §3): per "
                 "pass 8 B per unknown whose w and running column sit in registers, 16 B per unknown whose w alone "
                 "is on chip, 32 B per streamed unknown; plus w in and V(:,j+1) out")
        # Which memory ceiling binds.  The w-only variant reads each pass's dot column
        # V_q with the default policy so that it is still in the 256 MiB Infinity
        # Cache when the next pass reads it as V_i: its bytes cross the L2 <-> fabric
        # boundary (Infinity-Cache hits included), about half of them from DRAM --
        # the fabric read rate binds.  The other variants load their columns
        # non-temporally or hold the reused column in registers: every byte is DRAM.
        if variant == "w-only":
            bound, peak = "fabric", FABRIC_REF_GBPS
        else:
            bound, peak = "hbm", HBM_PEAK_GBPS
    secs = ms / 1e3
    ach = fused / secs / 1e9
    roof = {"bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": "GB/s",
            "frac": round(ach / peak, 4), "traffic": None, "model": model, "variant": variant,
            "regions_unknowns": regions,
            "hbm_spec_frac": round(ach / HBM_PEAK_GBPS, 4),
            "kernel": kname, "launches": launches, "avg_launch_us": round(ms * 1e3 / launches, 2),
            "alg_bytes_per_launch": round(fused / launches), "per_projection_us": round(per_proj, 2),
            "alg_as_written_bytes_per_launch": round(written / launches),
            "alg_as_written_frac": round(written / secs / 1e9 / HBM_PEAK_GBPS, 4),
            "timing": timing, "per_kernel_ms_sampled": {k: round(v[0], 3) for k, v in prof.items()}}
    if bound == "fabric":
        roof["peak_source"] = ("MI355X_MICROARCH.md: Infinity-Cache-resident reads 8.6 TB/s chip-wide (the rate "
                               "the L2 <-> fabric boundary sustains when lines come from the Infinity Cache)")
        # DRAM side: each pass's dot column from HBM, its AXPY column from the
        # Infinity Cache; w in, V(:,j+1) out.  A/B evidence (V_q non-temporal, so V_i
        # must come from HBM): 41.07 -> 45.06 us per projection, 5.96 TB/s of HBM
        # traffic = the achievable HBM rate (profiles/r03/ab_qnt_r03d.jsonl).
        if args.method == "hh":
            dram = sum((8.0 * L + 16.0) * nloc for L in chains)
        else:
            dram = sum((16.0 * j + 16.0) * nloc for j in steps_js)
        roof["ceiling"] = ("fabric: L2 <-> Infinity Fabric read rate (Infinity-Cache hits included); the DRAM "
                           "side carries about half of these bytes")
        roof["hbm"] = {"bytes_per_launch_est": round(dram / launches), "achieved": round(dram / secs / 1e9, 1),
                       "peak": HBM_PEAK_GBPS, "frac": round(dram / secs / 1e9 / HBM_PEAK_GBPS, 4),
                       "model": "each pass's dot column from HBM, its AXPY column from the Infinity Cache; w in, "
                                "the output column out",
                       "evidence": "profiles/r03/ab_qnt_r03d.jsonl (V_q non-temporal: +9.7 % per projection)"}
    else:
        roof["ceiling"] = "hbm: every compulsory byte is a DRAM byte (non-temporal column loads / register reuse)"
    roof_guard(roof)
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf) and on_res and args.method == "mgsr":
        pvar = f"blocked{(plan or {}).get('blk')}" if variant == "blocked" else variant  # bytes depend on S
        key, scale = pmc_lookup(json.load(open(tf)), pvar, nloc, m, args.prec, args.method,
                                int((plan or {}).get("G", 256)))
        pm = json.load(open(tf)).get(key) if key else None
        if pm and "per_step" in pm:
            per_step = {int(k): v * scale for k, v in pm["per_step"].items()}
            if all(j in per_step for j in set(steps_js)):
                tb = sum(per_step[j] for j in steps_js) / len(steps_js)
                roof["traffic"] = round(tb)
                roof["traffic_source"] = pm["source"] + (f" (scaled x{scale:.5f} from the {pm.get('nloc')}-unknown "
                                                         f"slab it was measured on)" if scale != 1.0 else "")
                roof["traffic_key"] = key
                roof["physical"] = {"fabric_GBps": round(tb * launches / secs / 1e9, 1),
                                    "traffic_over_alg": round(tb * launches / fused, 3),
                                    "note": "FETCH_SIZE (x2, gfx950) + WRITE_SIZE at the same steps j: L2<->fabric "
                                            "bytes, Infinity-Cache hits included"}
    return roof


def pmc_lookup(db: dict, variant: str, nloc: int, m: int, prec: str, method: str,
               G: int = 256) -> tuple[str | None, float]:
    """The PMC entry of this kernel: the exact slab on the same workgroup count,
    else the same variant whose per-workgroup load (unknowns / workgroups) is
    within 2 % of this one -- 4096^2 / 2 and 8192^2 / 8 have 8,388,608 unknowns
    per GPU, the single-GPU stand-in 2896^2 has 8,386,816; a same-device
    rehearsal rank holds half of 2896^2 on 128 workgroups -- its bytes scaled by
    the unknown count.  Entries without "G" were measured on 256 workgroups."""
    key = pmc_key(variant, nloc, m, prec, method)
    if key in db and int(db[key].get("G", 256)) == G:
        return key, 1.0
    load = nloc / max(1, G)
    best, bdev = None, None
    for k, v in db.items():
        if not (k.startswith(f"res_{variant}_") and k.endswith(f"_{m}_{prec}_{method}") and v.get("nloc")):
            continue
        dev = abs(v["nloc"] / int(v.get("G", 256)) - load)
        if dev <= 0.02 * load and (best is None or dev < bdev):
            best, bdev = k, dev
    return (best, nloc / db[best]["nloc"]) if best else (None, 1.0)


def pmc_key(variant: str, nloc: int, m: int, prec: str, method: str) -> str:
    """profiles/pmc_traffic.json key of a resident kernel's per-step PMC bytes:
    the variant and the slab it ran on (the same kernel at the same load gives
    the same bytes on 1 GPU and on every GPU of an N-rank split)."""
    return f"res_{variant}_{nloc}_{m}_{prec}_{method}"


def rhs_ones_host(N: int, line0: int, nlines: int) -> np.ndarray:
    """b = A*1 on the slab's lines, on the host: 4 minus the neighbours present."""
    i = np.arange(N)
    j = np.arange(line0, line0 + nlines)[:, None]
    b = 4.0 - (i > 0) - (i < N - 1) - (j > 0).astype(float) - (j < N - 1).astype(float)
    return np.ascontiguousarray(b.reshape(-1))


def pcie_inclusive(ctx, args, run, ctl, line0: int, nlines: int, cycles: int = 2) -> dict:
    """After the timed region: the drop-in's host-buffer flow -- b uploaded from
    host memory, `cycles` restart cycles, x downloaded into host memory (the
    solve's own final gk_get_x) -- timed as one, max over ranks.  Not `value`."""
    bh = rhs_ones_host(args.grid, line0, nlines)
    ctx.sync()
    ctl.barrier()
    t0 = time.perf_counter()
    ctx.set_rhs(bh)
    r = run(cycles)
    ctx.sync()
    el = ctl.allreduce(time.perf_counter() - t0, "max")
    iters = (r.n_cycles - 1) * args.m + r.n_out
    return {"cycles": r.n_cycles, "it_s": round(iters / el, 3), "wall_ms": round(el * 1e3, 2),
            "bytes_over_pcie": 16 * args.grid * args.grid,
            "note": "b host -> device before the cycles, x device -> host after (the Fortran drop-in's interface); "
                    "value keeps b, V and x resident (x is read back after the timed region)"}


def diagnostics(ctx, args, run, ctl, world: int) -> dict:
    """After the timed region (not part of `value`): one more cycle with the
    in-kernel clock split on -- per projection / reflection, the time a
    resident launch spends streaming its pass vs waiting in the in-launch
    all-gather (on N ranks that wait includes the cross-device rank totals) --
    and on N ranks the collective's own latency (gk_comm_latency).  Max over
    ranks, so the 8-GPU line carries the cross-device price beside it."""
    m = args.m
    if args.method == "mgsr":
        kinds = [(0, "mgs_step", m * (m + 1))]
    else:
        kinds = [(1, "hh_up", m * (m + 1) // 2), (2, "hh_down", m * (m + 1) // 2 + m)]
    ctx.res_split(1)
    run(1)
    ctx.sync()
    vals = []
    for which, _, nproj in kinds:
        r = ctx.res_split(-1, which)
        ok = r["launches"] > 0
        vals += [r["pass_ms"] * 1e3 / nproj if ok else -1.0, r["wait_ms"] * 1e3 / nproj if ok else -1.0]
    ctx.res_split(0)
    lat = [-1.0, -1.0]
    if world > 1:
        c = ctx.comm_latency(200)
        lat = [c["allreduce_us"], c["halo_us"]]
    allv = ctl.allgather(vals + lat)
    v = [round(float(max(col)), 3) for col in zip(*allv)]
    split = {}
    for k, (_, name, _) in enumerate(kinds):
        if v[2 * k] >= 0:
            split[name] = {"pass_us": v[2 * k], "wait_us": v[2 * k + 1]}
    return {"resident_split_per_unit_us": split or None,
            "collective_latency_us": ({"allreduce": v[-2], "halo": v[-1]} if world > 1 else None),
            "note": "one extra cycle after the timed region, max over ranks; pass = streaming, wait = in-launch "
                    "all-gather (tools/res_split.py); collective = one partial-slab all-reduce / one halo exchange"}


def blocked_leg_block(grid: int, world: int) -> int:
    """The projection block of the N-rank blocked leg: per GPU load, the S that measured
    fastest on one GPU at that load (tools/predict_scaling.py POINTS_BLOCKED):
    4 at the 4096^2 / 8 load (1448^2) and below, 2 above."""
    return 4 if grid * grid // world <= 1448 * 1448 * 11 // 10 else 2


def blocked_leg(ctx, args, run, ctl, world: int, cycles: int = 2, key: int = 23, S: int | None = None) -> dict:
    """After the timed region, N > 1 only (not `value`, which stays the reference's strict
    MGS-R on the default kernels): the same N-rank workload on an opt-in step -- by default
    the blocked-projection step (GK_TUNE_RES_BLOCK, one in-launch all-gather -- and one
    cross-GPU rank hop -- per block of S projections), or (key 27, GK_TUNE_RES_PF) the strict
    step on the prefetching blocked kernel -- so a multi-GPU run measures what DESIGN.md 6.1
    predicts for it: a 1-cycle solve from x0 = 0 checked against the reference's history,
    then `cycles` timed cycles, max over ranks, and the in-launch split."""
    S = blocked_leg_block(args.grid, world) if S is None else S
    ok, why, out = 1, "", {}
    try:
        ctx.tune(key, S)  # GK_TUNE_RES_BLOCK / GK_TUNE_RES_PF (re-plans, drops captured graphs)
        ctx.zero_x()
        chk = run(1, hist=True)
        ctx.sync()
        ctl.barrier()
        t0 = time.perf_counter()
        r = run(cycles, want_x=False)
        ctx.sync()
        el = time.perf_counter() - t0
        out = {"res": r, "chk": chk, "el": el, "plan": ctx.res_info()}
    except Exception as e:  # noqa: BLE001 - every rank reports, then all agree below
        ok, why = 0, str(e)
    if ctl.allreduce(ok, "min") != 1:
        ctx.tune(key, 1 if key == 23 else 0)  #  back to the default step on the error path too
        return {"projection_block": S, "error": why[:300] or "a peer rank failed the blocked leg"}
    el = ctl.allreduce(out["el"], "max")
    try:
        split = diagnostics(ctx, args, run, ctl, world).get("resident_split_per_unit_us")
    finally:
        ctx.tune(key, 1 if key == 23 else 0)
    r = out["res"]
    iters = (r.n_cycles - 1) * args.m + r.n_out
    check = history_vs_golden(out["chk"].hist_res, *GOLDEN_OF.get((args.grid, args.m, args.prec, args.method),
                                                                   (None, None)))
    what = ("opt-in blocked-projection MGS-R step (GK_TUNE_RES_BLOCK)" if key == 23 else
            "strict MGS-R on the prefetching blocked kernel, blocks of 1 (GK_TUNE_RES_PF)")
    return {"projection_block": S if key == 23 else 1, "it_s": round(iters / el, 3),
            "ms_per_cycle": round(el / max(r.n_cycles, 1) * 1e3, 3),
            "cycles": r.n_cycles, "resident_variant": out["plan"].get("variant"),
            "resident_split_per_unit_us": split, "check": check,
            "note": f"{what} on the same ranks after the timed region; value is the strict step on the default kernels"}


# ------------------------------------------------------- BASELINE configs ---
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")
# cycle-1 true residual of each workload from x0 = 0: the reference's own run
# (tests/golden/reference_runs.json, the reference built from its sources) or,
# for Chebyshev(8) which the reference does not have, the restatement's
GOLDEN_OF = {
    (4096, 95, "identity", "mgsr"): ("reference_runs.json", "mgsr_omp_identity_4096_m95_2cyc_t8"),
    (1024, 95, "identity", "mgsr"): ("reference_runs.json", "mgsr_omp_identity_1024_m95_12cyc_t8"),
    (4096, 95, "cheb", "mgsr"): ("oracle_4096.json", "mgsr_cheb8"),
    (4096, 95, "cbpr2", "mgsr"): ("reference_runs.json", "mgsr_omp_cbpr2_4096_m95_2cyc_t8"),
    (4096, 95, "identity", "hh"): ("reference_runs.json", "hh_omp_identity_4096_m95_2cyc_t8"),
}
# older fixtures (cycle 1 only / 3 cycles) where a longer history is not recorded
GOLDEN_FALLBACK = {
    "mgsr_omp_identity_4096_m95_2cyc_t8": "mgsr_omp_identity_4096_m95_1cyc_t8",
    "mgsr_omp_identity_1024_m95_12cyc_t8": "mgsr_omp_identity_1024_m95_3cyc_t8",
    "mgsr_omp_cbpr2_4096_m95_2cyc_t8": "mgsr_omp_cbpr2_4096_m95_1cyc_t8",
    "hh_omp_identity_4096_m95_2cyc_t8": "hh_omp_identity_4096_m95_1cyc_t8",
}
# (BASELINE configs[] index, grid, precond, degree, method, timed cycles, MGS projection block)
# -- block > 1: the same config on the opt-in blocked-projection step (GK_TUNE_RES_BLOCK;
# the reference's strict MGS-R stays the default everywhere else)
CONFIG_LEGS = [(1, 1024, "identity", 1, "mgsr", 3, 1), (1, 1024, "identity", 1, "mgsr", 3, 4),
               (2, 4096, "cheb", 8, "mgsr", 2, 1), (4, 4096, "identity", 1, "hh", 2, 1)]


def history_vs_golden(hist, gfile: str | None, gkey: str | None, tol: float = 1e-9, floor: float = 1e-6) -> dict:
    """The per-cycle true relative residuals of a run from x0 = 0 against the
    golden run's (the reference's own, or for Chebyshev(8) the restatement's):
    every common cycle within `tol` relative while the residual is above
    `floor` (below it the history is chaotic)."""
    hist = [float(h) for h in hist]
    if gfile is None or not hist:
        return {"cycle1_true_rel_residual": hist[0] if hist else None}
    runs = json.load(open(os.path.join(GOLDEN_DIR, gfile)))
    if gkey not in runs:
        gkey = GOLDEN_FALLBACK.get(gkey, gkey)
    g = runs[gkey]["hist_res"]
    k = min(len(hist), len(g))
    devs = [abs(hist[i] - g[i]) / g[i] for i in range(k)]
    checked = [d for i, d in enumerate(devs) if g[i] > floor]
    return {"cycle1_true_rel_residual": hist[0], "golden": g[0], "golden_source": f"tests/golden/{gfile}:{gkey}",
            "rel_dev": devs[0], "cycles_compared": k, "history": hist[:k], "history_rel_dev": devs,
            "tol": tol, "pass": bool(checked and max(checked) <= tol)}


def config_legs(ga, prof_every: int) -> list[dict]:
    """After the headline (not part of `value`): short timed legs of the other
    single-GPU BASELINE configs, each on a fresh context -- a 1-cycle solve from
    x0 = 0 (warmup; its cycle-1 true residual checked against the golden run),
    then K timed cycles of a new solve with HIP events on the dominant kernels."""
    out = []
    for idx, N, prec, degree, method, K, block in CONFIG_LEGS:
        m = 95
        ns = argparse.Namespace(m=m, method=method, prof_every=prof_every, grid=N, prec=prec, degree=degree)
        with ga.Context(N, m) as c:
            if block > 1:
                c.tune(23, block)  # GK_TUNE_RES_BLOCK
            c.set_precond(prec, (8.2, 0.2), degree)
            c.set_rhs_ones()

            def run(k, hist=False, want_x=True):
                if method == "mgsr":
                    return ga.gmres_mgsr(c, 1e-15, max_cycles=k, want_verr=False, want_hist=hist, want_x=want_x)
                return ga.gmres_hh(c, 1e-15, precondition=prec != "identity", max_cycles=k, want_verr=False,
                                   want_hist=hist, want_x=want_x)

            chk = run(K, hist=True)  # from x0 = 0: the K cycles' residual history vs the golden run
            c.profile(1 if method == "hh" else max(1, prof_every))
            c.profile_reset()
            c.sync()
            t0 = time.perf_counter()
            r = run(K, want_x=False)
            c.sync()
            t1 = time.perf_counter()
            prof = c.profile_read()
            plan = c.res_info(hh=method == "hh")
            roof = roofline_entry(prof, ns, c.nloc, r.n_cycles, 1, plan) or {}
        iters = (r.n_cycles - 1) * m + r.n_out
        pname = {"identity": "no precond", "cbpr2": "cbpr2", "cheb": f"Chebyshev({degree})"}[prec]
        blk = f", blocked projections S={block} (opt-in GK_TUNE_RES_BLOCK)" if block > 1 else ""
        leg = {"baseline_config": idx,
               "workload": f"{N}x{N} Poisson-2D fp64, GMRES-{method.upper()} m={m}, {pname}{blk}",
               "projection_block": block,
               "it_s": round(iters / (t1 - t0), 3), "ms_per_cycle": round((t1 - t0) / r.n_cycles * 1e3, 3),
               "cycles": r.n_cycles,
               "dominant": {k: roof.get(k) for k in ("kernel", "variant", "avg_launch_us", "per_projection_us",
                                                     "achieved", "bound", "peak", "frac", "hbm_spec_frac")},
               "check": history_vs_golden(chk.hist_res, *GOLDEN_OF[(N, m, prec, method)])}
        if prof.get("prec", (0, 0))[1] > 0:  # the temporal-blocked Chebyshev pass (k_cheb_fused)
            us = prof["prec"][0] * 1e3 / prof["prec"][1]
            leg["chebyshev_pass"] = {"avg_launch_us": round(us, 2), "launches_sampled": prof["prec"][1],
                                     "fused_bytes_per_launch": 24 * N * N,
                                     "GBps": round(24 * N * N / us / 1e3, 1)}
        out.append(leg)
    return out


# ------------------------------------------- short-recurrence legs (8f-3) ---
# Fused bytes per unknown of every gk_sr pass: operand inputs of
# a line march read once (their neighbour lines are L1/L2 hits), outputs written once.
SR_PASS_BYTES = {"sr_cg_p": 24, "sr_cg_x": 40, "sr_cg_z": 16, "sr_bi_p": 48, "sr_bi_pc": 40, "sr_bi_s": 32,
                 "sr_bi_sc": 32, "sr_st1": 24, "sr_st2": 24, "sr_bi_x": 64, "sr_bi_pe": 32, "sr_bi_se": 24,
                 "sr_dot": 16, "sr_cg_xz": 48, "sr_bi_pz": 56, "sr_bi_sz": 40}
# per iteration: the fused passes, and the reference's loops as written (each loop's
# operands read once, results written once; the identity preconditioner is a copy)
SR_ITER_BYTES = {("pcg", "identity"): (64, 152), ("pcg", "cbpr2"): (72, 200),
                 ("pbicgstab", "identity"): (136, 240), ("pbicgstab", "cbpr2"): (160, 336)}
# (cbpr2: the two-level marches, GK_TUNE_SR_TWO_LEVEL 1 -- one-level passes 80 / 184; a leg
# takes its fused figure from the passes that actually ran, sr_legs)
SR_LEGS = [("pcg", "identity"), ("pcg", "cbpr2"), ("pbicgstab", "identity"), ("pbicgstab", "cbpr2")]


def roof_guard(entry: dict) -> dict:
    """A byte model whose algorithmic bytes / kernel time exceed the peak it is
    priced against cannot be right (a cache the model ignores, or bytes it
    double-counts): flag it and withhold the fraction."""
    if entry and entry.get("frac") is not None and entry["frac"] > 1.0:
        entry["model_error"] = True
        entry["frac_claimed"] = entry["frac"]
        entry["frac"] = None
    return entry


def sr_cpu_baseline(solver: str, N: int, prec: str, k1: int = 4, k2: int = 0, budget_s: float = 12.0) -> dict | None:
    """The reference's own pcg_omp / pbicgstab_omp (oracle/_ref/ref_driver, src/cg.f90 /
    src/bicgstab.f90 built from the reference sources) on this host's OpenMP share:
    two truncated solves from x0 = 0 (max_iter = k1, k2); the rate is
    (k2 - k1) / (TIME_k2 - TIME_k1), which removes the allocation and first touch
    both runs pay.  k2 is sized from the k1 run to about budget_s seconds."""
    from oracle import refrun

    if not refrun.available():
        return None
    info = cpu_info()
    thr = info["omp_threads"]
    env = {"OMP_PROC_BIND": "close", "OMP_PLACES": "cores"}
    r1 = refrun.run(f"{solver}_omp", N, k1, prec, threads=thr, env=env, timeout=600)
    if not k2:
        per = max(r1.time / k1, 1e-4)
        k2 = int(min(2000, max(k1 + 8, budget_s / per)))
    r2 = refrun.run(f"{solver}_omp", N, k2, prec, threads=thr, env=env, timeout=900)
    rate = (k2 - k1) / max(r2.time - r1.time, 1e-9)
    return {"value": round(rate, 3), "unit": "iterations/s", "cores": r2.threads, "kind": "reference",
            "sample": f"oracle/_ref/ref_driver {solver}_omp on {N}^2 prec={prec}, b = A*1, x0 = 0, max_iter {k1} and "
                      f"{k2} (TIME = omp_get_wtime around the solver call); rate = ({k2} - {k1}) / (t{k2} - t{k1})",
            "t_s": [round(r1.time, 3), round(r2.time, 3)], "host": {k: info[k] for k in ("cpu_model", "nproc",
                                                                                       "omp_threads")}}


def sr_pmc_traffic(name: str, prec: str, n: int) -> dict:
    """The committed PMC measurement of a short-recurrence pass at 4096^2
    (profiles/r06/pmc_sr_traffic_r06as.json: FETCH_SIZE x 2 + WRITE_SIZE per
    unknown, median over the dispatches of `bench.py --sr-only`): `traffic` in
    bytes per launch, or null where the pass was not measured."""
    path = os.path.join(ROOT, "profiles", "r06", "pmc_sr_traffic_r06as.json")
    try:
        db = json.load(open(path))
    except (OSError, ValueError):
        return {"traffic": None}
    key = name[3:] if name.startswith("sr_") else name
    if key == "bi_x":
        key = "bi_x_identity" if prec == "identity" else "bi_x_cbpr2"
    e = db.get(key)
    if not e or n != 4096 * 4096:
        return {"traffic": None}
    per = e["fetch_B_per_unknown_x2"] + e["write_B_per_unknown"]
    return {"traffic": round(per * n), "traffic_per_unknown": round(per, 3),
            "traffic_source": f"profiles/r06/pmc_sr_traffic_r06as.json:{key} (FETCH_SIZE x2 + WRITE_SIZE)"}


def sr_legs(ga, iters: int = 400, with_cpu: bool = True, tune: list[str] | None = None,
            legs: list[tuple[str, str]] | None = None) -> list[dict]:
    """SURVEY 8f rank 3 at the bench's 4096^2: pcg_omp / pbicgstab_omp on the fused
    device passes (gk_sr_*).  Per leg, on a fresh context: the first 50 iterations
    from x0 = 0 against the reference's own truncated run (tests/golden
    reference_runs.json *_4096_hist50); `iters` timed iterations (tol 0: no early
    exit; graphs of 16 iterations, one status read at the end); one more run with
    HIP events on every pass (eager launches) for the per-pass roofline; the same
    workload as the reference sequences it (one device call per BLAS-1 operation,
    scalars on the host: fused=False) for the A/B; and the reference itself on
    this host's cores."""
    out = []
    N = 4096
    n = N * N
    runs = json.load(open(os.path.join(GOLDEN_DIR, "reference_runs.json")))
    for solver, prec in legs or SR_LEGS:
        leg = {"baseline_config": None, "kind": "short-recurrence solver (SURVEY 8f rank 3)",
               "workload": f"{N}x{N} Poisson-2D fp64, {solver}_omp ({'no precond' if prec == 'identity' else prec}), "
                           f"fused device passes", "solver": solver, "precond": prec}
        with ga.Context(N, 8) as c:
            for kv in tune or []:
                k, v = kv.split("=")
                c.tune(int(k), int(v))
            c.set_precond(prec, (8.2, 0.2), 1)
            c.set_rhs_ones()
            g = runs.get(f"{solver}_omp_{prec}_{N}_hist50")
            K = len(g["hist_res"]) if g else 50
            s = ga.SrSolve(c, solver, 0.0, K)
            s.iterate(K)
            ex, _, _ = s.status()
            h = s.history(ex)
            if g:
                dev = np.abs(h - np.asarray(g["hist_res"])) / np.asarray(g["hist_res"])
                leg["check"] = {"golden_source": f"tests/golden/reference_runs.json:{solver}_omp_{prec}_{N}_hist50",
                                "iterations_compared": int(len(h)), "max_rel_dev": float(dev.max()), "tol": 1e-9,
                                "pass": bool(dev.max() <= 1e-9)}
                g8 = runs.get(f"{solver}_omp_{prec}_{N}_hist50_t8")
                if solver == "pbicgstab" and g8:  # chaotic recurrence: the reference's own spread sets the band
                    from tests.sr_band import BAND_F, bicgstab_band

                    ok, worst = bicgstab_band(h, g["hist_res"], g8["hist_res"])
                    leg["check"].update({"tol": f"band: |ln(h/r)| <= ln(1 + {BAND_F:g} S_k), S_k = the reference's own "
                                                "1-vs-8-thread spread (tests/sr_band.py)",
                                         "band_worst": round(worst, 4), "pass": ok})
            s = ga.SrSolve(c, solver, 0.0, iters)  # timed: graphs, no events
            c.sync()
            t0 = time.perf_counter()
            s.iterate(iters)
            ex, _, res = s.status()
            t1 = time.perf_counter()
            el = t1 - t0
            fb, wb = SR_ITER_BYTES[(solver, prec)]
            leg.update({"iterations": ex, "it_s": round(ex / el, 2), "ms_per_iteration": round(el / ex * 1e3, 4),
                        "hbm_gbps_fused": round(fb * n * ex / el / 1e9, 1),
                        "fused_bytes_per_unknown_iteration": fb, "as_written_bytes_per_unknown_iteration": wb,
                        "hbm_gbps_alg_as_written": round(wb * n * ex / el / 1e9, 1)})
            # per-pass HIP events (eager launches)
            kp = 64
            c.profile(1)
            c.profile_reset()
            s = ga.SrSolve(c, solver, 0.0, kp)
            s.iterate(kp)
            s.status()
            prof = c.profile_read()
            c.profile(0)
            passes = {}
            for name, byt in SR_PASS_BYTES.items():
                ms, nl = prof.get(name, (0.0, 0))
                if nl == 0 or name == "sr_dot":
                    continue
                if name == "sr_bi_x" and prec == "identity":
                    byt = 56  # z2 = s: one read serves two operands
                us = ms * 1e3 / nl
                passes[name] = {"avg_launch_us": round(us, 2), "launches": nl, "bytes_per_unknown": byt,
                                "GBps": round(byt * n / us / 1e3, 1), "frac": round(byt * n / us / 1e3 / HBM_PEAK_GBPS, 4),
                                "share_of_pass_time": None}
            tot = sum(p["avg_launch_us"] * p["launches"] for p in passes.values())
            for p in passes.values():
                p["share_of_pass_time"] = round(p["avg_launch_us"] * p["launches"] / tot, 4)
            dom = max(passes, key=lambda k: passes[k]["avg_launch_us"] * passes[k]["launches"])
            d = passes[dom]
            leg["passes"] = passes
            # the fused bytes of the passes that ran (per iteration; the start's passes are < 2 %)
            fb_run = int(round(sum(p["bytes_per_unknown"] * p["launches"] for p in passes.values()) / kp))
            if fb_run != fb:
                leg.update({"fused_bytes_per_unknown_iteration": fb_run,
                            "hbm_gbps_fused": round(fb_run * n * ex / el / 1e9, 1)})
            leg["gap_us_per_iteration"] = round(el / ex * 1e6 - tot / kp, 2)
            leg["dominant"] = roof_guard({"kernel": f"gk::k_sr_march / k_sr_march2 / k_sr_vec pass {dom}",
                                          "bound": "hbm",
                                          "avg_launch_us": d["avg_launch_us"], "achieved": d["GBps"],
                                          "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": d["frac"],
                                          "bytes_per_launch": d["bytes_per_unknown"] * n,
                                          "timing": f"HIP events around every pass of {kp} eager iterations",
                                          **sr_pmc_traffic(dom, prec, n)})
            # A/B: the reference's operation sequence on the same device
            ka = 60 if solver == "pcg" else 40
            c.sync()
            t0 = time.perf_counter()
            getattr(ga, solver)(c, 0.0, ka, fused=False)
            t1 = time.perf_counter()
            leg["as_written_sequence"] = {"iterations": ka, "it_s": round(ka / (t1 - t0), 2),
                                          "note": "one device call per BLAS-1 operation of the reference, each dot "
                                                  "a host round trip (pcg_drive_seq / bicgstab_drive_seq); includes "
                                                  "the start and the final x download"}
        if with_cpu:
            leg["cpu_baseline"] = sr_cpu_baseline(solver, N, prec)
            if leg["cpu_baseline"]:
                leg["gpu_over_cpu"] = round(leg["it_s"] / leg["cpu_baseline"]["value"], 1)
        out.append(leg)
    return out


# ------------------------------------------------------------------- main ---
def kfd_queues(pid: int | None = None):
    """User-mode queues the KFD has created for this process (one per HIP hardware
    queue in use: the context stream, the null stream, RCCL's, blit queues ...), from
    /sys/class/kfd/kfd/proc/<pid>/queues; None where that is not readable."""
    d = f"/sys/class/kfd/kfd/proc/{pid or os.getpid()}/queues"
    try:
        return len(os.listdir(d))
    except OSError:
        return None


def kfd_sched_info() -> dict:
    """The amdgpu scheduler limits that decide how many processes' queues the
    hardware runs at once (readable module parameters only)."""
    out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
    for k in ("hws_max_conc_proc", "sched_policy", "mes", "cwsr_enable"):
        try:
            out[k] = open(f"/sys/module/amdgpu/parameters/{k}").read().strip()
        except OSError:
            pass
    return out


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
    ap.add_argument("--cpu-cap", type=float, default=45.0,
                    help="seconds: the share's leg also runs one full cycle (a check of the fit) if the fit says it "
                         "finishes within this")
    ap.add_argument("--cpu-steps", type=int, default=24,
                    help="Arnoldi steps of cycle 1 every thread-sweep leg times (the same window for every leg)")
    ap.add_argument("--no-configs", action="store_true",
                    help="N=1: skip the short timed legs of BASELINE configs 2, 3 and 5 after the headline")
    ap.add_argument("--no-prof", action="store_true", help="no HIP-event kernel timing in the timed region")
    ap.add_argument("--collective", default="auto", choices=["auto", "rccl", "xgmi"],
                    help="N>1: RCCL calls, or the device exchange over xGMI (auto: device exchange if its "
                         "self-test passes on every rank, else RCCL)")
    ap.add_argument("--prof-every", type=int, default=16,
                    help="HIP events around the launches of every S-th Arnoldi step (1 = all)")
    ap.add_argument("--plan-only", action="store_true", help="print the multi-GPU launch plan and exit")
    ap.add_argument("--no-diag", action="store_true", help="skip the post-timing diagnostic cycle")
    ap.add_argument("--sr-only", action="store_true",
                    help="run only the short-recurrence legs (pcg / pbicgstab at 4096^2) and print them as JSON")
    ap.add_argument("--no-sr", action="store_true", help="N=1: skip the short-recurrence legs after the headline")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="A/B runs: gk_set_tuning(KEY, VALUE) on the bench context (include/gmres_hip.h GK_TUNE_*)")
    args = ap.parse_args()
    if args.sr_only:
        import gmres_amd as ga

        print(json.dumps({"sr_legs": sr_legs(ga, with_cpu=not args.no_cpu, tune=args.tune), "tune": args.tune}),
              flush=True)
        return
    maybe_self_launch(args, sys.argv[1:])

    # No torch in this process: the library runs on the HIP runtime and RCCL it
    # was built against (gmres_amd._native; the line's config.runtime says which).
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the N-rank flow on a 1-GPU box (tests only, never a bench
    # line): every rank on device 0, resident launches sharing its CUs.
    same_dev = os.environ.get("GK_BENCH_SAME_DEVICE") == "1"
    if same_dev:
        local = 0
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    from gmres_amd.ctl import Ctl

    t_start = time.perf_counter()

    def log(stage: str) -> None:  # progress on stderr: a long multi-rank run is never silent
        print(f"[bench rank {rank}/{world} +{time.perf_counter() - t_start:.1f}s] {stage}", file=sys.stderr,
              flush=True)

    ctl = Ctl(rank, world)  # out-of-band control plane (TCP on loopback); a no-op for one rank
    log("control plane up")
    if rank == 0 and world > 1:
        log(f"kfd scheduler: {kfd_sched_info()}")

    import gmres_amd as ga

    N, m = args.grid, args.m
    parts = ga.slab_partition(N, world)
    line0, nlines = parts[rank]
    ctx = ga.Context(N, m, device=local, line0=line0, nlines=nlines)
    if same_dev and world > 1:
        ctx.tune(10, world)  # GK_TUNE_RES_SHARE: 256 / N workgroups per rank
        ctx.tune(8, 1)  # GK_TUNE_RES: resident steps on (auto mode assumes one context per device)
    ml = max(p[1] for p in parts)
    collective = None
    rccl_failed = None  # RCCL init failed on some rank; the device exchange carries every collective
    if world > 1 and args.collective == "xgmi":
        ctx.comm_init_xgmi(world, rank, ml)
    elif world > 1 or os.environ.get("GK_FORCE_RCCL") == "1":  # 1-rank RCCL: exercises the comm path
        uid = ctl.bcast(ga.Context.unique_id() if rank == 0 else None)
        ok, why = 1, ""
        try:
            ctx.comm_init(world, rank, ml, uid)
        except ga.GkError as e:
            ok, why = 0, str(e)
            print(f"rank {rank}: RCCL communicator failed: {e}", file=sys.stderr)
        ok = ctl.allreduce(ok, "min")
        if ok:
            collective = "rccl"
        elif world > 1 and args.collective == "auto":
            # every rank together: the slab decomposition without RCCL, collectives
            # by the device exchange only (setup_xgmi below must then succeed)
            rccl_failed = why[:300] or "a peer rank's RCCL init failed"
            ctx.comm_init_xgmi(world, rank, ml)
        else:
            raise RuntimeError(f"RCCL communicator: {why or 'a peer rank failed'}")
    if world > 1 and args.collective in ("auto", "xgmi"):
        collective = setup_xgmi(ctx, ctl, rank,
                                required=args.collective == "xgmi" or rccl_failed is not None) or "rccl"
    log(f"collective: {collective or 'none'}; kfd user queues of this process: {kfd_queues()}")
    first_contact = first_contact_record(ctx, ctl, rank, world, local) if world > 1 else None
    if first_contact is not None and rank == 0:
        log(f"first contact: {json.dumps(first_contact)}")
    for kv in args.tune:
        k, v = kv.split("=")
        ctx.tune(int(k), int(v))
    ctx.set_precond(args.prec, (8.2, 0.2), args.degree)
    ctx.set_rhs_ones()

    def run(cycles: int, hist: bool = False, want_x: bool = True):
        if args.method == "mgsr":
            return ga.gmres_mgsr(ctx, 1e-15, max_cycles=cycles, want_verr=False, want_hist=hist, want_x=want_x)
        return ga.gmres_hh(ctx, 1e-15, precondition=(args.prec != "identity"), max_cycles=cycles,
                           want_verr=False, want_hist=hist, want_x=want_x)

    def barrier():
        ctx.sync()  # this rank's stream drained (every kernel of the solve is on it)
        ctl.barrier()

    warm = {}

    def guarded_warmup() -> tuple[bool, str]:
        ok, why = 1, ""
        try:
            if args.warmup > 0:  # from x0 = 0: its cycle 1 is checked against the reference below
                warm["res"] = run(args.warmup, hist=True)
        except Exception as e:  # noqa: BLE001 - every rank reports, then all agree below
            why = str(e)
            print(f"rank {rank}: warmup failed: {e}", file=sys.stderr)
            ok = 0
        return ctl.allreduce(ok, "min") == 1, why

    fallback = None
    ok, why = guarded_warmup()
    log(f"warmup {'done' if ok else 'FAILED'}; kfd user queues of this process: {kfd_queues()}")
    if not ok:
        # Fallback, decided by all ranks together and REPORTED in the JSON line:
        # the launch-per-projection path, and RCCL instead of the device exchange
        # where an RCCL communicator exists.  A device exchange that missed a
        # deadline is retired (its sequence numbers may differ across ranks), so
        # without RCCL there is nothing to fall back to: fail with both reasons.
        fallback = {"reason": why[:300] or "a peer rank failed its warmup", "to": "launch-per-projection path"}
        if collective == "xgmi-device-exchange":
            if rccl_failed is not None or args.collective == "xgmi":
                raise RuntimeError(f"warmup failed on the device exchange ({fallback['reason']}) and there is no "
                                   f"RCCL communicator to fall back to ({rccl_failed or '--collective xgmi'})")
            ctx.xchg_enable(False)
            collective = "rccl"
            fallback["to"] += " + RCCL (device exchange failed in warmup)"
        ctx.tune(8, 0)  # GK_TUNE_RES off
        ok, why = guarded_warmup()
        if not ok:
            raise RuntimeError(f"warmup failed on the fallback path too: {why}")
    if not args.no_prof:
        ctx.profile(1 if args.method == "hh" else max(1, args.prof_every))
        ctx.profile_reset()
    barrier()
    t0 = time.perf_counter()
    res = run(args.steps, want_x=False)  # x stays in HBM: the PCIe-inclusive rate is pcie_inclusive()
    barrier()
    t1 = time.perf_counter()
    prof = ctx.profile_read() if not args.no_prof else {}
    resid = ctx.true_residual()  # outside the timed region; same value at any N
    comm = ctx.comm_info()
    elapsed = ctl.allreduce(t1 - t0, "max")
    log(f"timed {args.steps} cycle(s): {elapsed * 1e3:.1f} ms")
    cycles = res.n_cycles
    iters = (cycles - 1) * m + res.n_out if cycles > 0 else 0
    plan = ctx.res_info(hh=args.method == "hh")  # the resident variant the timed launches ran
    diag = None if args.no_diag else diagnostics(ctx, args, run, ctl, world)
    log("diagnostics done")
    if diag is not None:
        diag["pcie_inclusive"] = pcie_inclusive(ctx, args, run, ctl, line0, nlines)
        if (world > 1 and args.method == "mgsr" and fallback is None
                and not any(kv.split("=")[0] == "23" for kv in args.tune)):
            log("blocked leg")
            diag["blocked_leg"] = blocked_leg(ctx, args, run, ctl, world)
            log("strict prefetch leg")
            diag["strict_prefetch_leg"] = blocked_leg(ctx, args, run, ctl, world, key=27, S=1)

    cheb_sten = plan.get("cheb_sten", 0) == 1
    roof = roofline_entry(prof, args, ctx.nloc, cycles, world, plan) if rank == 0 else None
    runtime = ga.runtime_info()
    ctx.close()
    legs = None
    if rank == 0 and world == 1 and not args.no_configs and (N, m, args.prec, args.method) == (4096, 95, "identity",
                                                                                                 "mgsr"):
        log("BASELINE config legs")
        legs = config_legs(ga, args.prof_every)
        if not args.no_sr:
            log("short-recurrence legs (pcg / pbicgstab, 4096^2)")
            legs += sr_legs(ga, with_cpu=not args.no_cpu)
    if rank == 0:
        n = N * N
        it_s = iters / elapsed
        full = cycles == args.steps and res.n_out == m
        b_fused = cycle_bytes(n, m, args.prec, args.degree, args.method, "fused", cheb_sten) * cycles
        b_written = cycle_bytes(n, m, args.prec, args.degree, args.method, "as_written") * cycles
        cpu = None
        if not args.no_cpu and world == 1:
            log("CPU baseline (the reference on this host)")
            cpu = cpu_baseline(N, m, args.prec, args.degree, args.method, args.cpu_cap, args.cpu_steps)
        check = {"true_rel_residual_after_timed_cycles": resid}
        if "res" in warm and len(warm["res"].hist_res) > 0:
            check.update(history_vs_golden(warm["res"].hist_res, *GOLDEN_OF.get((N, m, args.prec, args.method),
                                                                                (None, None))))
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
                       "collective": collective, "comm_ranks_seen": comm["nranks"], "comm_kind": comm["kind"],
                       "comm_ranks_note": comm_ranks_note(comm, world, collective),
                       "first_contact": first_contact,
                       "rccl_init_failed": rccl_failed,
                       "resident_variant": plan.get("variant"), "resident_workgroups": plan.get("G"),
                       "arnoldi_iters": iters,
                       "runtime": runtime},
            "fallback": fallback,
            "check": check,
            "hbm_gbps_fused": round(b_fused / elapsed / 1e9, 1) if full else None,
            "cycle_roofline_frac": round(b_fused / elapsed / 1e9 / HBM_PEAK_GBPS, 4) if full else None,
            "hbm_gbps_alg_as_written": round(b_written / elapsed / 1e9, 1) if full else None,
            "alg_as_written_frac": round(b_written / elapsed / 1e9 / HBM_PEAK_GBPS, 4) if full else None,
            "roofline": roof,
            "cpu_baseline": cpu,
            "diagnostics": diag,
            "configs": legs,
        }
        print(json.dumps(out), flush=True)
    ctl.barrier()
    ctl.close()


if __name__ == "__main__":
    main()
