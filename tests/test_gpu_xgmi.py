"""Device-exchange collective back-end (include/gmres_hip.h gk_comm_init_xgmi /
gk_xchg_*) on ONE GPU.

The multi-GPU data path replaces the per-projection RCCL all-reduce, the
Householder broadcast and the halo send/recv with stores of tagged 8-byte
granules into every peer's receive region ("custom xGMI flag-based
all-reduce").  A 1-GPU box cannot host two RCCL ranks, but it can host the
device exchange: several contexts of one process (plain pointers), or several
processes sharing the GPU through IPC handles -- the same code path the
8-GPU run takes, minus the xGMI links.

Results: every rank takes the same decisions (rank-order sums are
bit-identical on all ranks) and the slab solve matches the single-context
solve within the tolerances of test_gpu_multirank.py.
"""
import multiprocessing as mp
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _single(N, m, method, prec, degree, max_cycles):
    import gmres_amd as ga

    with ga.Context(N, m) as c:
        c.set_precond(prec, (8.2, 0.2), degree)
        c.set_rhs_ones()
        return _solve(c, method, prec, max_cycles)


def _solve(c, method, prec, max_cycles):
    import gmres_amd as ga

    if method == "mgsr":
        return ga.gmres_mgsr(c, 1e-15, max_cycles=max_cycles, want_hist=True)
    return ga.gmres_hh(c, 1e-15, precondition=(prec != "identity"), max_cycles=max_cycles, want_hist=True)


def _run_threads(nranks, fn):
    out, err = [None] * nranks, []

    def work(r):
        try:
            out[r] = fn(r)
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not err, err
    return out


def _local_group(N, m, nranks):
    import gmres_amd as ga

    parts = ga.slab_partition(N, nranks)
    ml = max(nl for _, nl in parts)
    g = ga.LocalGroup(nranks)
    ctxs = [ga.Context(N, m, device=0, line0=l0, nlines=nl) for l0, nl in parts]
    for r, c in enumerate(ctxs):
        c.comm_init_local(g, r, ml)
    for c in ctxs:
        c.xchg_local()
    return g, ctxs


def _close(g, ctxs):
    for c in ctxs:
        c.close()
    g.close()


def _check_against_single(ref, res, method):
    assert len({(r.n_out, r.cycles_out, r.n_cycles) for r in res}) == 1
    for r in res[1:]:
        assert np.array_equal(res[0].hist_res, r.hist_res)
    k = min(len(ref.hist_res), len(res[0].hist_res))
    h, rr = res[0].hist_res[:k], ref.hist_res[:k]
    # Relative tiers set from the measured drift (tools/multirank_dev.py,
    # profiles/r03/multirank_dev_r03o.jsonl; 2 and 3 ranks): r > 1e-6 at most
    # 2.6e-12; MGS-R in (1e-10, 1e-6] at most 1.1e-7, below 1e-10 at most 4.2e-3
    # (there the 1e-16 absolute term decides).  Householder below 1e-6: the tiers
    # of test_gpu_solver._hist_close_hh.
    mg = np.where(rr > 1e-10, 1e-5, 1e-3)
    tol = np.where(rr > 1e-6, 1e-9, mg if method == "mgsr" else np.where(rr > 1e-12, 1e-3, 5e-2))
    assert np.all(np.abs(h - rr) <= tol * rr + 1e-16), (h, rr)
    x = np.concatenate([r.x for r in res])
    if ref.hist_res[-1] > 1e-6:
        assert np.allclose(x, ref.x, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("nranks", [1, 2, 3])
def test_selftest_in_process(nranks):
    g, ctxs = _local_group(40, 8, nranks)
    ok = _run_threads(nranks, lambda r: ctxs[r].xchg_selftest(5000))
    _close(g, ctxs)
    assert all(ok), [getattr(c, "xchg_error", "") for c in ctxs]


def test_missing_peer_times_out_instead_of_hanging():
    """Only rank 0 enters the exchange: its wait hits the deadline, the call
    reports the failure (no GPU hang) and the exchange is switched off."""
    import gmres_amd as ga

    g, ctxs = _local_group(32, 4, 2)
    assert ctxs[0].xchg_selftest(300) is False
    assert "deadline" in ctxs[0].xchg_error
    assert "rank 1" in ctxs[0].xchg_error  # the straggler is named
    _close(g, ctxs)


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("method,prec,degree", [("mgsr", "identity", 1), ("mgsr", "cbpr2", 1), ("mgsr", "cheb", 4),
                                                ("hh", "identity", 1), ("hh", "cbpr2", 1)])
def test_slabs_match_single_context(nranks, method, prec, degree):
    N, m, cyc = 66, 16, 6
    ref = _single(N, m, method, prec, degree, cyc)
    g, ctxs = _local_group(N, m, nranks)

    def work(r):
        c = ctxs[r]
        c.set_precond(prec, (8.2, 0.2), degree)
        c.set_rhs_ones()
        return _solve(c, method, prec, cyc)

    res = _run_threads(nranks, work)
    _close(g, ctxs)
    _check_against_single(ref, res, method)


@pytest.mark.parametrize("method,prec,degree", [("mgsr", "identity", 1), ("mgsr", "cbpr2", 1), ("mgsr", "cheb", 4),
                                                ("hh", "identity", 1), ("hh", "cbpr2", 1)])
def test_resident_step_over_device_exchange(method, prec, degree):
    """Resident launches (MGS-R step; Householder reflection chains) with the rank
    totals exchanged inside the launch: two ranks on one GPU, forced on
    (GK_TUNE_RES = 1; auto mode keeps it off when contexts share a device)."""
    N, m, cyc = 66, 16, 6
    ref = _single(N, m, method, prec, degree, cyc)
    g, ctxs = _local_group(N, m, 2)
    for c in ctxs:
        c.tune(8, 1)
        c.tune(11, 5000)

    def work(r):
        c = ctxs[r]
        c.set_precond(prec, (8.2, 0.2), degree)
        c.set_rhs_ones()
        c.profile(True)
        c.profile_reset()
        out = _solve(c, method, prec, cyc)
        return out, c.profile_read()

    out = _run_threads(2, work)
    _close(g, ctxs)
    res = [o[0] for o in out]
    assert all(o[1]["res"][1] > 0 for o in out)
    _check_against_single(ref, res, method)


def test_lanczos_and_verr_over_device_exchange():
    import gmres_amd as ga

    N = 40
    with ga.Context(N, 8) as c:
        ref = c.lanczos_bounds(30)
    g, ctxs = _local_group(N, 12, 3)
    out = _run_threads(3, lambda r: ctxs[r].lanczos_bounds(30))
    assert out[0] == out[1] == out[2]
    assert out[0][0] == pytest.approx(ref[0], rel=1e-9) and out[0][1] == pytest.approx(ref[1], rel=1e-12)

    def solve(r):
        c = ctxs[r]
        c.set_precond("cbpr2", (8.2, 0.2), 1)
        c.set_rhs_ones()
        return ga.gmres_mgsr(c, 1e-15, max_cycles=1000)

    res = _run_threads(3, solve)
    _close(g, ctxs)
    x = np.concatenate([r.x for r in res])
    assert np.max(np.abs(x - 1.0)) < 1e-9
    assert 0 <= res[0].v_err[res[0].n_out - 1] < 1e-12


# ---------------------------------------------------- several processes ----

def _proc_worker(rank, nranks, N, m, cyc, hq, hin, outq, force_res=0):
    try:
        import gmres_amd as ga

        parts = ga.slab_partition(N, nranks)
        ml = max(nl for _, nl in parts)
        l0, nl = parts[rank]
        c = ga.Context(N, m, device=0, line0=l0, nlines=nl)
        c.comm_init_xgmi(nranks, rank, ml)
        hq.put((rank, c.xchg_handle()))
        handles = hin.get(timeout=100)
        c.xchg_open(handles)
        c.tune(10, nranks)  # GK_TUNE_RES_SHARE: the ranks' resident launches share this one GPU
        if force_res:
            c.tune(8, 1)
            c.tune(11, 5000)
        ok = c.xchg_selftest(10000)
        if not ok:
            outq.put((rank, "selftest", getattr(c, "xchg_error", "")))
            return
        c.set_precond("cbpr2", (8.2, 0.2), 1)
        c.set_rhs_ones()
        r = ga.gmres_mgsr(c, 1e-15, max_cycles=cyc, want_hist=True)
        outq.put((rank, "ok", (r.x, r.hist_res, r.n_out, r.cycles_out, r.n_cycles)))
        c.close()
    except Exception as e:  # pragma: no cover - reported to the parent
        outq.put((rank, "error", repr(e)))


@pytest.mark.parametrize("nranks,force_res", [(2, 0), (2, 1)])
def test_processes_share_regions_by_ipc(nranks, force_res):
    """Two processes on one GPU, regions exchanged as IPC handles (the
    multi-GPU setup path of bench.py without RCCL)."""
    N, m, cyc = 64, 16, 4
    ref = _single(N, m, "mgsr", "cbpr2", 1, cyc)
    ctx = mp.get_context("spawn")
    hq, outq = ctx.Queue(), ctx.Queue()
    hins = [ctx.Queue() for _ in range(nranks)]
    ps = [ctx.Process(target=_proc_worker, args=(r, nranks, N, m, cyc, hq, hins[r], outq, force_res)) for r in range(nranks)]
    for p in ps:
        p.start()
    try:
        hs = dict(hq.get(timeout=100) for _ in range(nranks))
        for q in hins:
            q.put([hs[r] for r in range(nranks)])
        got = dict((r, (kind, val)) for r, kind, val in (outq.get(timeout=100) for _ in range(nranks)))
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(nranks):
        assert got[r][0] == "ok", got[r]
    res = [got[r][1] for r in range(nranks)]
    assert len({(v[2], v[3], v[4]) for v in res}) == 1
    assert all(np.array_equal(res[0][1], v[1]) for v in res)
    x = np.concatenate([v[0] for v in res])
    k = min(len(ref.hist_res), len(res[0][1]))
    assert np.allclose(res[0][1][:k], ref.hist_res[:k], rtol=1e-9, atol=1e-16)
    assert np.allclose(x, ref.x, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("N,nranks,degree", [(66, 3, 8), (40, 2, 5), (20, 4, 4)])
def test_chebyshev_deep_halo_over_device_exchange(oracle, N, nranks, degree):
    """The deep halo of the temporal-blocked Chebyshev passes through the
    device exchange (k_xhalo with L lines): bit-exact against the oracle."""
    r = np.random.default_rng(N * degree).standard_normal(N * N)
    ref = oracle.precond(oracle.PREC_CHEB, r, N, params=(8.2, 0.2), degree=degree)
    import gmres_amd as ga

    g, ctxs = _local_group(N, 8, nranks)
    parts = ga.slab_partition(N, nranks)
    for c in ctxs:
        c.set_precond("cheb", (8.2, 0.2), degree)
    out = _run_threads(nranks, lambda q: ctxs[q].apply(r[parts[q][0] * N:(parts[q][0] + parts[q][1]) * N], 1))
    _close(g, ctxs)
    assert np.array_equal(np.concatenate(out), ref)


@pytest.mark.parametrize("nranks", [2, 3])
def test_comm_latency_diagnostic(nranks):
    """gk_comm_latency (bench.py's multi-GPU diagnostic) through the device
    exchange: every rank returns a positive per-op cost, and the exchange still
    gives bit-identical slab solves afterwards."""
    g, ctxs = _local_group(64, 8, nranks)
    try:
        lat = _run_threads(nranks, lambda r: ctxs[r].comm_latency(50))
        for d in lat:
            assert 0.0 < d["allreduce_us"] < 5e4 and 0.0 < d["halo_us"] < 5e4, lat
        res = _run_threads(nranks, lambda r: (ctxs[r].set_rhs_ones(), _solve(ctxs[r], "mgsr", "identity", 2))[1])
        assert all(np.array_equal(res[0].hist_res, r.hist_res) for r in res)
    finally:
        _close(g, ctxs)


# ------------------------------------------------ a straggling process ------

def _straggler_worker(rank, delay_s, timeout_ms, hq, hin, outq, done):
    import time

    try:
        import gmres_amd as ga
        from gmres_amd import _native as nat

        N, m = 64, 16
        l0, nl = ga.slab_partition(N, 2)[rank]
        c = ga.Context(N, m, device=0, line0=l0, nlines=nl)
        c.comm_init_xgmi(2, rank, N // 2)
        hq.put((rank, c.xchg_handle()))
        c.xchg_open(hin.get(timeout=100))
        c.tune(nat.GK_TUNE_RES_SHARE, 2)
        c.tune(nat.GK_TUNE_RES, 1)  # the step is one resident launch with in-launch rank totals
        c.tune(nat.GK_TUNE_XCHG_TIMEOUT_MS, timeout_ms)
        c.tune(nat.GK_TUNE_RES_TIMEOUT_MS, timeout_ms)
        ok = c.xchg_selftest(10000)
        c.set_rhs_ones()
        c.mgs_cycle_start()  # collective: both ranks in step here
        time.sleep(delay_s)
        t0 = time.perf_counter()
        try:
            c.mgs_step(1)
            res = ("no error", time.perf_counter() - t0)
        except nat.GkError as e:
            res = (str(e), time.perf_counter() - t0)
        outq.put((rank, "ok", (ok, res)))
        done.wait(120)  # keep the exchange region mapped until the peer is done with it
        c.close()
    except Exception as e:  # pragma: no cover - reported to the parent
        outq.put((rank, "error", repr(e)))


def test_straggling_process_is_named_within_the_deadline():
    """Two IPC-connected processes (the multi-GPU transport); rank 1 starts its
    first Arnoldi step 2 s after the 1.5 s deadline of every exchange wait.
    Rank 0 must fail that step with GK_ERR_COMM naming rank 1 within the
    deadline (no GPU hang); rank 1, arriving late, finds rank 0 gone inside the
    resident launch and fails naming rank 0; both processes exit cleanly and
    the GPU still solves afterwards."""
    timeout_ms, delay = 1500, 3.5
    ctx = mp.get_context("spawn")
    hq, outq, done = ctx.Queue(), ctx.Queue(), ctx.Event()
    hins = [ctx.Queue() for _ in range(2)]
    ps = [ctx.Process(target=_straggler_worker, args=(r, [0.0, delay][r], timeout_ms, hq, hins[r], outq, done))
          for r in range(2)]
    for p in ps:
        p.start()
    try:
        hs = dict(hq.get(timeout=100) for _ in range(2))
        for q in hins:
            q.put([hs[0], hs[1]])
        got = dict((r, (kind, val)) for r, kind, val in (outq.get(timeout=100) for _ in range(2)))
    finally:
        done.set()
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert [p.exitcode for p in ps] == [0, 0]
    for r in range(2):
        assert got[r][0] == "ok", got[r]
        assert got[r][1][0], "the exchange self-test passed before the straggling"
    msg0, t0 = got[0][1][1]
    msg1, t1 = got[1][1][1]
    assert "status -6" in msg0 and "rank 1" in msg0, msg0
    assert timeout_ms / 1e3 * 0.9 < t0 < timeout_ms / 1e3 + 1.5, (t0, msg0)  # one deadline, not one per wait
    assert "status -6" in msg1 and "rank 0" in msg1, msg1
    assert t1 < timeout_ms / 1e3 + 1.5, (t1, msg1)
    # the device is healthy: a fresh solve converges as before
    r = _single(32, 10, "mgsr", "identity", 1, 100)
    assert r.hist_res[-1] < 1e-12


# ------------------------------------------- the driver's N-rank bench line ---

def test_bench_two_ranks_default_collective_on_one_gpu():
    """bench.py --gpus 2 as the driver runs it (its own torch.distributed
    launch, the default --collective auto), both ranks on this GPU
    (GK_BENCH_SAME_DEVICE): RCCL refuses two ranks on one device, so every rank
    falls back together to the device exchange alone, and the line's cycle-1
    residual still matches the reference's own 1024^2 run."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GK_BENCH_SAME_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--grid", "1024",
                        "--steps", "1", "--warmup", "1", "--no-cpu", "--no-diag"],
                       capture_output=True, text=True, env=env, cwd=root, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["fallback"] is None
    assert line["config"]["collective"] == "xgmi-device-exchange"
    assert line["config"]["comm_ranks_seen"] == 2
    assert line["check"]["pass"], line["check"]


# ------------------------------------- a self-test that fails on one rank ----

def _failing_selftest_worker(rank, port, hq, hin, outq):
    import os
    import sys
    import time

    try:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        import gmres_amd as ga
        from gmres_amd.ctl import Ctl

        N, m = 64, 16
        l0, nl = ga.slab_partition(N, 2)[rank]
        c = ga.Context(N, m, device=0, line0=l0, nlines=nl)
        c.comm_init_xgmi(2, rank, N // 2)
        ctl = Ctl(rank, 2, key=f"selftest_fail_{port}", timeout=120)
        t0 = time.perf_counter()
        out = bench.setup_xgmi(c, ctl, rank, required=False)
        dt = time.perf_counter() - t0
        rec = bench.first_contact_record(c, ctl, rank, 2, 0)
        outq.put((rank, "ok", (out, dt, getattr(c, "xchg_error", ""), rec)))
        ctl.barrier()
        ctl.close()
        c.close()
    except Exception as e:  # pragma: no cover - reported to the parent
        outq.put((rank, "error", repr(e)))


def test_selftest_failure_on_one_rank_is_agreed_within_the_deadline():
    """two processes on one GPU, the real device exchange
    over IPC, rank 1's self-test forced to fail (GK_DEBUG_SELFTEST_FAIL=1: it
    takes no part).  Rank 0 misses its 5 s deadline waiting for rank 1's
    granules; both ranks then take bench.setup_xgmi's documented decision
    together (exchange off on every rank; the caller falls back to RCCL or
    fails), each within the deadline plus margin, and the first-contact record
    names both errors."""
    import os
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["GK_DEBUG_SELFTEST_FAIL"] = "1"  # inherited by the spawned ranks
    try:
        ctx = mp.get_context("spawn")
        hq, outq = ctx.Queue(), ctx.Queue()
        ps = [ctx.Process(target=_failing_selftest_worker, args=(r, port, hq, None, outq)) for r in range(2)]
        for p in ps:
            p.start()
        try:
            got = dict((r, (kind, val)) for r, kind, val in (outq.get(timeout=120) for _ in range(2)))
        finally:
            for p in ps:
                p.join(timeout=60)
                if p.is_alive():
                    p.kill()
    finally:
        os.environ.pop("GK_DEBUG_SELFTEST_FAIL", None)
    assert [p.exitcode for p in ps] == [0, 0]
    for r in range(2):
        assert got[r][0] == "ok", got[r]
    (o0, dt0, e0, rec0), (o1, dt1, e1, rec1) = got[0][1], got[1][1]
    assert o0 is None and o1 is None  # the same decision on every rank: no device exchange
    assert "forced" in e1 and "rank 0" in e0 and ("deadline" in e0 or "rank 1" in e0), (e0, e1)
    assert dt1 < 5.0 + 3.0 and dt0 < 5.0 + 3.0, (dt0, dt1)  # the agreement waits one deadline, not forever
    assert rec0["selftest_errors"][1] and rec0["same_device_rehearsal"]
