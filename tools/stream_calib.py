"""Calibration of the streaming rate on this GPU at 4096^2 (fp64): the plain
stencil sweep k_stencil (gk_vec_apply: y = A x, 16 B/unknown) and the
preconditioner (cbpr2 epilogue, 16 B), each timed by HIP events around the
launch (ctx.profile), next to hipMemcpy device-to-device (16 B) -- the rates the
short-recurrence passes are compared with.  Prints one JSON."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gmres_amd as ga  # noqa: E402
from gmres_amd import _native as nat  # noqa: E402

N = 4096
n = N * N
out = {}
with ga.Context(N, 8) as c:
    c.set_precond("cbpr2", (8.2, 0.2), 1)
    c.set_rhs_ones()
    lib = nat.hip()
    for blocks in (0, 512, 1024, 4096):
        c.tune(2, blocks)
        for rep in range(2):
            c.profile(1)
            c.profile_reset()
            for _ in range(20):
                nat.check(lib.gk_vec_apply(c.handle, 0, 2, 3), "apply")  # V2 -> V3: A x
            c.sync()
            p = c.profile_read()
            c.profile(0)
        ms, k = p["stencil"]
        us = ms * 1e3 / k
        out[f"stencil_plain_blocks{blocks}"] = {"us": round(us, 2), "GBps": round(16 * n / us / 1e3, 1)}
    c.tune(2, 0)
    # cbpr2: precond of V2 into V4 (copy into z then the OP_CBPR2 sweep)
    c.profile(1)
    c.profile_reset()
    for _ in range(20):
        nat.check(lib.gk_vec_apply(c.handle, 1, 2, 4), "apply")
    c.sync()
    p = c.profile_read()
    ms, k = p["stencil"]
    out["stencil_cbpr2"] = {"us": round(ms * 1e3 / k, 2), "GBps": round(16 * n / (ms * 1e3 / k) / 1e3, 1)}
    # elementwise lincomb (read 2, write 1), host-timed over 50 launches
    for _ in range(3):
        nat.check(lib.gk_vec_lincomb(c.handle, 1, 3, 2, 4, 4, 0.5, 0.0), "lincomb")
    c.sync()
    t0 = time.perf_counter()
    for _ in range(50):
        nat.check(lib.gk_vec_lincomb(c.handle, 1, 3, 2, 4, 4, 0.5, 0.0), "lincomb")
    c.sync()
    us = (time.perf_counter() - t0) / 50 * 1e6
    out["lincomb_axpy_hosttimed"] = {"us": round(us, 2), "GBps": round(24 * n / us / 1e3, 1)}
print(json.dumps(out))
