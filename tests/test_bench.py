"""bench.py host logic on CPU: the multi-GPU launch plan, the refusal when
fewer GPUs are visible than asked for, the byte models behind roofline.frac
and the CPU-baseline extrapolation."""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env():
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    return e


def test_plan_only_spawns_one_rank_per_gpu():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3", "--plan-only"],
                         capture_output=True, text=True, env=_env(), timeout=120)
    assert out.returncode == 0, out.stderr
    plan = json.loads(out.stdout.strip().splitlines()[-1])
    cmd = plan["cmd"]
    assert plan["ranks"] == 8 and cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index(os.path.join(ROOT, "bench.py")) + 1:] == ["--gpus", "8", "--steps", "3"]
    assert plan["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_plan_only_under_a_launcher_is_one_rank():
    e = _env()
    e.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--plan-only"],
                         capture_output=True, text=True, env=e, timeout=120)
    assert out.returncode == 0 and json.loads(out.stdout)["launcher"] is None


def test_refuses_more_gpus_than_visible():
    """No GPU in the build container: --gpus 2 must fail loudly, not run 1 rank."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu"],
                         capture_output=True, text=True, env=_env(), timeout=300)
    assert out.returncode == 2
    assert "GPU(s) visible" in out.stderr


def test_byte_models():
    n = 4096 * 4096
    # the resident step launch at j = 48 (VERDICT r01 recomputation)
    assert bench.mgs_step_bytes(n, 48, "fused") == (32 * 48 + 16) * n
    assert bench.mgs_step_bytes(n, 48, "as_written") == (80 * 48 + 24) * n
    assert bench.mgs_step_bytes(n, 48, "fused") / 4069.9e-6 / 1e9 / bench.HBM_PEAK_GBPS == pytest.approx(0.80, abs=0.01)
    # SURVEY 8(d) per-cycle model: 6,198 GB at 4096^2, m = 95
    assert bench.cycle_bytes(n, 95, "identity", 1, "mgsr", "as_written") == pytest.approx(6198e9, rel=2e-3)
    assert bench.cycle_bytes(n, 95, "identity", 1, "mgsr", "fused") < bench.cycle_bytes(
        n, 95, "identity", 1, "mgsr", "as_written") / 2
    # Chebyshev(8) is ONE temporal-blocked pass (read z, write the result);
    # Chebyshev(16) hands (d, r, z) from the first pass to the second
    assert bench.prec_bytes(n, "cheb", 8, "fused") == 0 and bench.prec_bytes(n, "cheb", 8, "as_written") == 384 * n
    assert bench.prec_bytes(n, "cheb", 16, "fused") == 64 * n
    # without the stencil stage (GK_TUNE_CHEB_STEN 0, N < 128, thin slabs) the pass
    # reads z from a stencil launch: +16n
    assert bench.prec_bytes(n, "cheb", 8, "fused", cheb_sten=False) == 16 * n
    assert (bench.cycle_bytes(n, 95, "cheb", 8, "mgsr", "fused", cheb_sten=False)
            - bench.cycle_bytes(n, 95, "cheb", 8, "mgsr", "fused")) == 95 * 16 * n


def _plan(N, R=1, share=1, nt=-1):
    import gmres_amd as ga

    nl = max(k for _, k in ga.slab_partition(N, R))
    return N * nl, ga.res_plan_query(N * nl, 256, share, False, nt)


def test_resident_byte_model_follows_the_variant():
    """res_launch_bytes charges each variant what it moves: the w-only kernel 16 B
    per unknown per pass (nothing streamed since round 5), the pairs kernels 8 B per
    unknown whose running column sits in registers and 16 B per LDS-held unknown."""
    n, p = _plan(4096)  # bench default: w-only, all 128 chunks per workgroup on chip (89 + 39)
    assert p["variant"] == "w-only"
    r = bench.res_regions(p, n)
    assert sum(r.values()) == n and r["pairs"] == 0 and r["streamed"] == 0
    per_pass = (bench.res_launch_bytes(p, n, 97) - bench.res_launch_bytes(p, n, 96)) / n
    assert per_pass == 16.0
    # 4096^2 / 2 and 8192^2 / 8 (k_mgs_wpc, 512 threads, the MGS step): w in registers, 25 of
    # its 32 chunks' column cached (8 B per unknown), the other 7 read V_i too (16 B) -> 9.75 B
    n, p = _plan(4096, 2)
    assert p["variant"] == "w+column" and p["wt"] == 512
    r = bench.res_regions(p, n)
    assert r == {"pairs": 2 * 256 * 25 * 512, "w_on_chip": 2 * 256 * 7 * 512, "streamed": 0}
    per_pass = (bench.res_launch_bytes(p, n, 97) - bench.res_launch_bytes(p, n, 96)) / n
    assert per_pass == pytest.approx(9.75)
    # 4096^2 / 4: 16 chunks per workgroup, all cached -> 8 B per unknown
    n4, p4 = _plan(4096, 4)
    # (the MGS step of this load: the strict step on k_mgs_blk<S = 1>, the whole column cached too)
    assert p4["variant"] in ("w+column", "blocked") and bench.res_regions(p4, n4) == {"pairs": n4, "w_on_chip": 0, "streamed": 0}
    # the previous kernel of that split (k_mgs_res<12, 18> NT, GK_TUNE_RES_PC 0): 12 of 32 chunks
    # pairs, 18 in LDS, 2 streamed
    import gmres_amd as ga

    p = ga.res_plan_query(n, 256, 1, False, 1)
    p = dict(p, variant="pairs+lds", r2=12, l2=18, r2e=12, l2e=18, nres2=256 * 30 * 512, pf=0, cw=0, wo=0)
    r = bench.res_regions(p, n)
    assert sum(r.values()) == n
    assert r["pairs"] == 2 * 256 * 12 * 512 and r["w_on_chip"] == 2 * 256 * 18 * 512
    per_pass = (bench.res_launch_bytes(p, n, 97) - bench.res_launch_bytes(p, n, 96)) / n
    assert per_pass == pytest.approx(8 * 12 / 32 + 16 * 18 / 32 + 32 * 2 / 32, rel=1e-3)  # 14 B per unknown
    # 4096^2 / 8 (k_mgs_res<8, 0>): everything pairs -> 8 B per unknown per pass
    n, p = _plan(4096, 8)
    assert p["variant"] == "pairs"
    per_pass = (bench.res_launch_bytes(p, n, 97) - bench.res_launch_bytes(p, n, 96)) / n
    assert per_pass == pytest.approx(8.0, rel=2e-3)


def test_blocked_byte_model_of_the_one_wave_build():
    """The one-wave S = 4 blocked build (256 threads like the w-only one, but its whole block
    cached): 8 B per unknown per pass, as its PMC traffic over a full cycle at 1448^2 shows
    (profiles/r05/pmc_*_bench_1448_blk4_cycle_r05am.csv: 8.06 B, traffic / model 0.99-1.004)."""
    import gmres_amd as ga

    n = 4096 * 512
    p = ga.res_plan_query(n, 256, 1, False, -1, block=4)
    assert (p["variant"], p["wt"], p["r2"]) == ("blocked", 256, 16)
    per_pass = (bench.res_launch_bytes(p, n, 97) - bench.res_launch_bytes(p, n, 96)) / n
    assert per_pass == pytest.approx(8.0)
    p = ga.res_plan_query(4096 * 4096, 256, 1, False, -1, block=4)  # the w-only blocked build
    assert bench.res_regions(p, 4096 * 4096)["pairs"] == 0


def test_roofline_entry_is_a_fraction():
    """The round-1 bench's sampled launches (4,100 us per step launch at j = 16..80
    over 20 cycles) give frac ~0.8 on the fused-minimum model, and the
    as-written figure (> 1) is kept separately."""
    a = argparse.Namespace(m=95, method="mgsr", prof_every=16, grid=4096, prec="identity")
    prof = {k: (0.0, 0) for k in ["proj", "stencil", "scale", "update", "comm", "other"]}
    prof["res"] = (410.003, 100)
    n, p = _plan(4096)
    r = bench.roofline_entry(prof, a, n, 20, 1, p)
    # w-only: its reuse goes through the Infinity Cache -> the fabric read rate binds
    assert r["bound"] == "fabric" and r["peak"] == bench.FABRIC_REF_GBPS and r["variant"] == "w-only"
    assert 0.68 < r["frac"] < 0.78 and 0.74 < r["hbm_spec_frac"] < 0.84
    assert 0.3 < r["hbm"]["frac"] < 0.5  # the DRAM side: about half the bytes
    assert r["alg_as_written_frac"] > 1.8
    assert r["avg_launch_us"] == pytest.approx(4100.03)
    # a pairs+lds split (4096^2 on 2 GPUs): every byte from DRAM -> bound hbm
    n2, p2 = _plan(4096, 2)
    r2 = bench.roofline_entry(prof, a, n2, 20, 2, p2)
    assert r2["bound"] == "hbm" and r2["peak"] == bench.HBM_PEAK_GBPS and r2["variant"] == "w+column"


def test_cpu_extrapolation_recovers_a_linear_step_cost():
    a, b, m = 0.3, 0.02, 95
    t, st = 1.0, {}
    for j in range(1, 13):
        st[j] = t
        t += a + b * j
    est, how = bench._extrapolate(st, 0.5, m)
    exact = 0.5 + sum(a + b * j for j in range(1, m + 1)) + b * (m + 2) / 10
    assert est == pytest.approx(exact, rel=1e-9) and "a + b j" in how


def test_cpu_info_fields():
    info = bench.cpu_info()
    assert info["nproc"] >= 1 and 1 <= info["omp_threads"] <= info["affinity"]
    assert "all_cores" not in info  # the share is the process's OpenMP share, not the machine
    assert isinstance(info["cpu_model"], str)


def test_thread_sweep_is_the_reference_pattern():
    """tests/strong_scaling.f90:44-55 of the reference: 1, 2, 4, 8, 16 threads,
    here capped at the process's OpenMP share (always the last leg)."""
    assert bench.sweep_threads(16) == [1, 2, 4, 8, 16]
    assert bench.sweep_threads(8) == [1, 2, 4, 8]
    assert bench.sweep_threads(6) == [1, 2, 4, 6]
    assert bench.sweep_threads(1) == [1]
    assert bench.sweep_threads(64) == [1, 2, 4, 8, 16, 64]


def test_launcher_never_touches_hip():
    """The self-launching parent counts GPUs from the KFD topology / render
    nodes and never imports torch or loads the HIP runtime before its ranks
    start (a HIP call in the launcher would initialise the runtime there)."""
    code = ("import sys; sys.argv=['bench.py']; import bench; n = bench.visible_gpus(); "
            "maps = open('/proc/self/maps').read(); "
            "print(n, 'libamdhip64' in maps, any(k == 'torch' or k.startswith('torch.') for k in sys.modules))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=_env(), cwd=ROOT,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    n, hip, torch_loaded = out.stdout.split()
    assert int(n) >= 0 and hip == "False" and torch_loaded == "False"
    # the refusal path (no GPU here) and --plan-only never import torch either
    for extra in (["--no-cpu"], ["--plan-only"]):
        p = subprocess.run([sys.executable, "-X", "importtime", os.path.join(ROOT, "bench.py"), "--gpus", "2", *extra],
                           capture_output=True, text=True, env=_env(), timeout=120)
        imported = [ln.rsplit("|", 1)[-1].strip() for ln in p.stderr.splitlines() if ln.startswith("import time:")]
        assert not any(x == "torch" or x.startswith("torch.") for x in imported), extra
    assert bench.visible_gpus() == 0 or os.path.exists("/dev/kfd")


def test_same_device_rehearsal_gets_one_queue_per_rank():
    """The same-device rehearsal overrides an inherited GPU_MAX_HW_QUEUES (the GPU
    box exports 4: 8 ranks x 4 queues time-sliced the r05y 8-rank run); a real
    multi-GPU run keeps the inherited value."""
    box = {"GPU_MAX_HW_QUEUES": "4", "PATH": "/usr/bin"}
    assert bench.rank_env(box, {"X": "1"}) == dict(box, X="1")
    e = bench.rank_env(dict(box, GK_BENCH_SAME_DEVICE="1"), {})
    assert e["GPU_MAX_HW_QUEUES"] == "1"
    e = bench.rank_env(dict(box, GK_BENCH_SAME_DEVICE="1", GK_BENCH_SAME_DEVICE_QUEUES="2"), {})
    assert e["GPU_MAX_HW_QUEUES"] == "2"


def test_blocked_leg_block_follows_the_per_gpu_load():
    """The N-rank blocked leg takes S = 4 at the 4096^2 / 8 load (1448^2) and S = 2 above
    (tools/predict_scaling.py POINTS_BLOCKED)."""
    assert bench.blocked_leg_block(4096, 8) == 4
    assert bench.blocked_leg_block(4096, 4) == 2
    assert bench.blocked_leg_block(4096, 2) == 2
    assert bench.blocked_leg_block(8192, 8) == 2
    assert bench.blocked_leg_block(1448, 2) == 4


def test_visible_gpus_respects_visibility_env(monkeypatch):
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0


def test_host_rhs_matches_the_oracle_on_slabs():
    """bench.py's PCIe-inclusive leg uploads b = A*1 built on the host: equal to
    the oracle's manufactured RHS on every row-block slab."""
    import numpy as np

    from oracle import oracle as orc

    import gmres_amd as ga

    N = 37
    ref = orc.rhs_ones(N)
    for R in (1, 3):
        parts = ga.slab_partition(N, R)
        b = np.concatenate([bench.rhs_ones_host(N, l0, nl) for l0, nl in parts])
        assert np.array_equal(b, ref)


def _ctl_rank(rank, world, key, d, q):
    from gmres_amd.ctl import Ctl

    c = Ctl(rank, world, key=key, timeout=60, rdzv_dir=d)
    out = {"all": c.allgather(rank * 10), "b": c.bcast("root" if rank == 0 else None),
           "min": c.allreduce(rank + 1, "min"), "max": c.allreduce(rank + 0.5, "max"),
           "sum": c.allreduce(rank, "sum")}
    c.barrier()
    c.close()
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 3])
def test_control_plane_world_size(world, tmp_path):
    """bench.py's torch-free control plane (gmres_amd/ctl.py): rendezvous by a
    file, gather / broadcast / min / max / sum identical on every rank."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ctl_rank, args=(r, world, "t", str(tmp_path), q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        o = got[r]
        assert o["all"] == [10 * k for k in range(world)] and o["b"] == "root"
        assert o["min"] == 1 and o["max"] == world - 0.5 and o["sum"] == world * (world - 1) // 2
    assert not os.path.exists(os.path.join(str(tmp_path), "gk_ctl_t"))  # rank 0 removed the rendezvous file


def _ctl_stuck_rank(rank, world, key, d, q):
    """Rank 1 joins and then never takes part in a collective (a live but stuck peer)."""
    from gmres_amd.ctl import Ctl

    c = Ctl(rank, world, key=key, timeout=3, rdzv_dir=d)
    if rank == 0:
        t0 = time.monotonic()
        try:
            c.allgather(0)
            q.put(("no error", 0.0))
        except TimeoutError as e:
            q.put((str(e), time.monotonic() - t0))
    else:
        time.sleep(8)
    c.close()


def test_control_plane_bounds_a_stuck_peer(tmp_path):
    """Every control-plane receive is bounded: rank 0's
    gather from a rank that joined but never answers fails within the timeout,
    naming that rank, instead of blocking forever."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ctl_stuck_rank, args=(r, 2, "stuck", str(tmp_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    msg, dt = q.get(timeout=60)
    for p in ps:
        p.join(timeout=30)
    assert "rank 1" in msg and dt < 6, (msg, dt)


class _Planted:
    """A pickle that creates a file when unpickled (a stranger's hello)."""

    def __init__(self, path):
        self.path = path

    def __reduce__(self):
        return (open, (self.path, "w"))


def test_control_plane_authenticates_before_unpickling(tmp_path):
    """rank 0 reads a connecting peer's hello as raw bytes and
    checks the token before anything is unpickled -- a stranger's pickled payload
    is dropped unread -- and the rendezvous file (port + token) is private."""
    import pickle
    import socket
    import stat
    import struct
    import threading

    from gmres_amd.ctl import Ctl

    marker = tmp_path / "unpickled"
    out = {}

    def rank0():
        c = Ctl(0, 2, key="auth", timeout=30, rdzv_dir=str(tmp_path))
        out["v"] = c.allgather("r0")
        c.close()

    t = threading.Thread(target=rank0)
    t.start()
    f = tmp_path / "gk_ctl_auth"
    for _ in range(600):
        if f.exists():
            break
        time.sleep(0.01)
    assert stat.S_IMODE(f.stat().st_mode) == 0o600
    port = int(f.read_text().split()[0])
    data = pickle.dumps(_Planted(str(marker)))
    with socket.create_connection(("127.0.0.1", port)) as s:
        s.sendall(struct.pack("!Q", len(data)) + data)
        s.settimeout(5)
        try:
            assert s.recv(16) == b""  # dropped: closed without an answer
        except (ConnectionResetError, socket.timeout):
            pass
    c1 = Ctl(1, 2, key="auth", timeout=30, rdzv_dir=str(tmp_path))
    v = c1.allgather("r1")
    c1.close()
    t.join(timeout=30)
    assert v == out["v"] == ["r0", "r1"]
    assert not marker.exists()


def test_control_plane_skips_a_stale_rendezvous_file(tmp_path):
    """A rendezvous file left by a crashed launch (its rank 0 dead) is not
    connected to: the joining rank waits for the live rank 0's file."""
    import multiprocessing as mp

    p0 = subprocess.Popen([sys.executable, "-c", "pass"])
    p0.wait()
    dead = p0.pid
    with socket.socket() as s:  # a port nobody listens on after this
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    (tmp_path / "gk_ctl_stale").write_text(f"{port} {'0' * 32} {dead}\n")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    r1 = ctx.Process(target=_ctl_rank, args=(1, 2, "stale", str(tmp_path), q))
    r1.start()
    time.sleep(1.0)  # rank 1 polls the stale file meanwhile
    r0 = ctx.Process(target=_ctl_rank, args=(0, 2, "stale", str(tmp_path), q))
    r0.start()
    got = dict(q.get(timeout=60) for _ in range(2))
    for p in (r0, r1):
        p.join(timeout=30)
    assert got[0]["all"] == got[1]["all"] == [0, 10]


def test_pmc_lookup_by_variant_and_slab():
    """profiles/pmc_traffic.json is keyed by the resident variant and the slab it
    ran on; a split whose per-GPU slab is within 2 % of a measured one (4096^2 / 2
    vs the 2896^2 stand-in) reuses it scaled by the unknown count."""
    import json

    db = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    k, s = bench.pmc_lookup(db, "w-only", 4096 * 4096, 95, "identity", "mgsr")
    assert k == "res_w-only_16777216_95_identity_mgsr" and s == 1.0
    k, s = bench.pmc_lookup(db, "w+column", 4096 * 4096 // 2, 95, "identity", "mgsr")
    assert k == "res_w+column_8386816_95_identity_mgsr" and s == pytest.approx(8388608 / 8386816)
    assert bench.pmc_lookup(db, "w+column", 4096 * 4096, 95, "identity", "mgsr") == (None, 1.0)
    # a same-device rehearsal rank: half of 2896^2 on 128 workgroups carries the 2896^2 load per
    # workgroup (not the 2048^2 slab's, whose unknown count it shares)
    k, s = bench.pmc_lookup(db, "w+column", 2896 * 2896 // 2, 95, "identity", "mgsr", G=128)
    assert k == "res_w+column_8386816_95_identity_mgsr" and s == pytest.approx(0.5)
    k, s = bench.pmc_lookup(db, "w+column", 2048 * 2048, 95, "identity", "mgsr")
    assert k == "res_w+column_4194304_95_identity_mgsr" and s == 1.0


def test_read_scale_finds_bench_lines_in_a_driver_file():
    """tools/read_scale.py: bench lines nested anywhere in the driver's scaling
    file (dicts, lists, stdout tails) are set beside the committed prediction."""
    import json
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import read_scale

    line = {"metric": "m", "value": 500.0, "n_gpus": 2, "config": {"resident_variant": "w+column"},
            "diagnostics": {"resident_split_per_unit_us": {"mgs_step": {"wait_us": 5.0}}}}
    doc = {"runs": [{"n": 2, "run": {"stdout_tail": "log\n" + json.dumps(line) + "\n"}}, {"n": 4, "skipped": True}]}
    lines = read_scale.bench_lines(doc)
    assert lines == [line]
    pred = {"points": [{"world": 2, "grid": 4096, "predicted_it_s": [450.0, 600.0],
                        "predicted_wait_per_projection_us": [4.0, 7.0]}]}
    (row,) = read_scale.compare(lines, pred)
    assert row["verdict"] == "inside band" and row["wait_us"] == 5.0 and row["variant"] == "w+column"
    # round 5's two tables, and the N-rank line's blocked leg against the blocked one
    line["diagnostics"]["blocked_leg"] = {"it_s": 470.0, "projection_block": 2}
    pred5 = {"strict": pred, "blocked": {"points": [{"world": 2, "grid": 4096, "predicted_it_s": [480.0, 520.0]}]}}
    doc = {"runs": [{"n": 2, "run": {"stdout_tail": json.dumps(line)}}]}
    (row,) = read_scale.compare(read_scale.bench_lines(doc), pred5)
    assert row["verdict"] == "inside band" and row["blocked_S"] == 2 and row["blocked_verdict"] == "below band"


def test_sr_pmc_traffic_lookup():
    """The short-recurrence legs' dominant pass carries the committed PMC bytes
    (profiles/r06/pmc_sr_traffic_r06as.json): fetch x 2 + write per unknown, the
    identity x / r pass from its own (z2 = s) measurement, null off 4096^2 or
    for a pass never measured; every pass's writes match the byte model."""
    n = 4096 * 4096
    t = bench.sr_pmc_traffic("sr_cg_x", "identity", n)
    assert t["traffic_per_unknown"] == pytest.approx(40.95, abs=0.05) and t["traffic"] > 40 * n
    assert bench.sr_pmc_traffic("sr_bi_x", "identity", n)["traffic_per_unknown"] == pytest.approx(56.01, abs=0.01)
    assert bench.sr_pmc_traffic("sr_bi_x", "cbpr2", n)["traffic_per_unknown"] == pytest.approx(64.01, abs=0.01)
    assert bench.sr_pmc_traffic("sr_cg_x", "identity", 1024 * 1024) == {"traffic": None}
    assert bench.sr_pmc_traffic("sr_dot", "identity", n) == {"traffic": None}
    db = json.load(open(os.path.join(bench.ROOT, "profiles", "r06", "pmc_sr_traffic_r06as.json")))
    for key, e in db.items():
        if key.startswith("_") or "write_B_per_unknown" not in e:
            continue
        assert e["write_B_per_unknown"] == pytest.approx(e["model_write"], rel=1e-3), key
        assert 1.0 - 1e-3 <= e["fetch_B_per_unknown_x2"] / e["model_read"] <= 1.25, key
