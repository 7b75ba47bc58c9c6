"""Which HIP runtime the product runs on, and the configurations it refuses.

* A torch-free Python process runs the HIP path on the runtime libgmres_hip.so
  was built against (/opt/rocm): config 1 at 128^2 to convergence against the
  reference's own run (tests/golden/reference_runs.json), with
  gk_runtime_info / /proc/self/maps naming the mapped libamdhip64 and librccl.
* gk_xchg_local refuses, at once, a group of in-process ranks on one device
  that needs more hardware queues than the process has (GPU_MAX_HW_QUEUES):
  the configuration that deadlocked until the exchange deadline in round 3
  (4 ranks under HIP's default of 4 queues).
"""
import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_runs.json")))


def _child(code: str, env: dict | None = None, timeout: int = 100):
    e = dict(os.environ)
    e.pop("GK_TORCH_FIRST", None)
    if env:
        e.update(env)
    return subprocess.run([sys.executable, "-u", "-c", code], cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=timeout)


TORCH_FREE = r"""
import json, sys
import gmres_amd as ga
with ga.Context(128, 30) as c:
    c.set_rhs_ones()
    c.profile(True)
    r = ga.gmres_mgsr(c, 1e-15, variant=ga.MGSR_MF, want_hist=True)
    prof = c.profile_read()
rt = ga.runtime_info()
print(json.dumps({"iters": (r.n_cycles - 1) * 30 + r.n_out, "cycles": r.n_cycles, "hist": r.hist_res.tolist(),
                  "res_launches": prof["res"][1], "rt": rt,
                  "torch_loaded": any(k == "torch" or k.startswith("torch.") for k in sys.modules)}))
"""


def test_torch_free_process_runs_the_hip_path_on_the_built_runtime():
    p = _child(TORCH_FREE)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    rt = d["rt"]
    assert not d["torch_loaded"] and not rt["torch_imported"], d
    assert rt["libamdhip64"] and "/torch/" not in rt["libamdhip64"], rt
    assert rt["librccl"] and "/torch/" not in rt["librccl"], rt
    assert rt["hip_runtime_version"] > 0 and rt["rccl_version"] > 0, rt
    assert d["res_launches"] > 0  # the resident HIP step, not a fallback
    g = REF["mgsr_mf_identity_128_m30"]
    assert abs(d["iters"] - g["iterations"]) <= 0.01 * g["iterations"], (d["iters"], g["iterations"])
    k = min(len(d["hist"]), len(g["hist_res"]))
    for a, b in zip(d["hist"][:k], g["hist_res"][:k]):
        assert abs(a - b) <= 1e-5 * b + 1e-13, (a, b)


REFUSE = r"""
import time
import gmres_amd as ga
N, R = 64, 4
parts = ga.slab_partition(N, R)
g = ga.LocalGroup(R)
cs = [ga.Context(N, 10, device=0, line0=l0, nlines=nl) for l0, nl in parts]
for r, c in enumerate(cs):
    c.comm_init_local(g, r, max(n for _, n in parts))
t0 = time.time()
try:
    cs[0].xchg_local()
    print("ACCEPTED")
except ga.GkError as e:
    print("REFUSED", round(time.time() - t0, 3), str(e))
for c in cs:
    c.close()
g.close()
"""


def test_xchg_local_refuses_ranks_beyond_the_hardware_queues():
    t0 = time.time()
    p = _child(REFUSE, env={"GPU_MAX_HW_QUEUES": "4"})
    assert p.returncode == 0, p.stderr[-3000:]
    out = p.stdout.strip().splitlines()[-1]
    assert out.startswith("REFUSED"), out
    assert "hardware queues" in out and "GPU_MAX_HW_QUEUES" in out, out
    assert float(out.split()[1]) < 1.0  # at once, not after an exchange deadline
    assert time.time() - t0 < 90
    # with enough queues the same group is accepted
    p = _child(REFUSE, env={"GPU_MAX_HW_QUEUES": "8"})
    assert p.returncode == 0 and p.stdout.strip().splitlines()[-1] == "ACCEPTED", (p.stdout, p.stderr[-2000:])


def test_watchdog_bounds_a_stream_that_never_drains():
    """The host watchdog of every stream wait: a context
    whose stream is held behind a never-written mapped word (gk_debug_hold_stream,
    as when its hardware queue is never mapped) fails gk_sync with GK_ERR_COMM
    inside the GK_TUNE_WATCHDOG_MS bound, naming the cause; the context is then
    broken (later calls refuse) and, once released, is destroyed cleanly; a solve
    queued behind the hold fails within the bound too."""
    import time

    import gmres_amd as ga
    from gmres_amd import _native as nat

    c = ga.Context(64, 10)
    try:
        c.tune(nat.GK_TUNE_WATCHDOG_MS, 1500)
        c.set_rhs_ones()
        c.sync()
        c.debug_hold_stream(True)
        t0 = time.monotonic()
        with pytest.raises(nat.GkError) as e:
            c.sync()
        dt = time.monotonic() - t0
        assert "never scheduled" in str(e.value) and "status -6" in str(e.value), str(e.value)
        assert 1.4 < dt < 10, dt
        with pytest.raises(nat.GkError) as e2:
            c.set_rhs_ones()
        assert "broken" in str(e2.value)
    finally:
        c.debug_hold_stream(False)  # the stream drains; destroy then frees normally
        c.close()
    # a solve whose first kernels queue behind a hold: the Fortran host's step
    # wait fails within the bound instead of waiting forever
    c = ga.Context(64, 10)
    try:
        c.tune(nat.GK_TUNE_WATCHDOG_MS, 1500)
        c.set_rhs_ones()
        c.sync()
        c.debug_hold_stream(True)
        t0 = time.monotonic()
        with pytest.raises(nat.GkError):
            ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)
        assert time.monotonic() - t0 < 15
    finally:
        c.debug_hold_stream(False)
        c.close()
    with ga.Context(64, 10) as c:  # the device is sane afterwards
        c.set_rhs_ones()
        r = ga.gmres_mgsr(c, 1e-15, max_cycles=2, want_verr=False)
        assert r.n_out == 10
