#!/usr/bin/env python3
"""Does initialising torch's HIP context slow the host's per-step wait?  One
process: 1024^2 cycles (a) before torch touches the GPU, (b) after
torch.cuda.synchronize(), each with the step wait spinning (GK_TUNE_SPIN_WAIT 1)
and blocking (0).  Prints ms per cycle for each."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cycles(ga, nat, spin: int, K: int = 4) -> float:
    with ga.Context(1024, 95) as c:
        c.tune(nat.GK_TUNE_SPIN_WAIT, spin)
        c.set_precond("identity", (8.2, 0.2), 1)
        c.set_rhs_ones()
        ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)
        c.sync()
        t0 = time.perf_counter()
        ga.gmres_mgsr(c, 1e-15, max_cycles=K, want_verr=False)
        c.sync()
        return (time.perf_counter() - t0) / K * 1e3


def main() -> None:
    import gmres_amd as ga
    from gmres_amd import _native as nat

    out = {"before_torch": {"spin": cycles(ga, nat, 1), "block": cycles(ga, nat, 0)}}
    import torch

    torch.cuda.synchronize(0)
    out["after_torch"] = {"spin": cycles(ga, nat, 1), "block": cycles(ga, nat, 0)}
    print(json.dumps({k: {kk: round(v, 3) for kk, v in d.items()} for k, d in out.items()}))


if __name__ == "__main__":
    main()
