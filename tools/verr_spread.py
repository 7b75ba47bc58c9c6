#!/usr/bin/env python3
"""The oracle's own spread of the MGS-R v_err diagnostic (gmres_mgsr.f90:414-420)
across OpenMP thread counts 1..8 (every pair; the bases differ by reduction order
only): the yardstick of tests/test_gpu_solver.py::_mgs_verr_close, in decades.

  python tools/verr_spread.py > profiles/r05/verr_oracle_spread_r05.txt
"""
import itertools
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as o  # noqa: E402  (test infrastructure: a CPU measurement)


def main() -> None:
    for N, m, c in [(64, 20, 2), (128, 30, 3)]:
        runs = {t: np.asarray(o.gmres_mgsr(o.rhs_ones(N), N, m, variant=o.MGSR_OMP, max_cycles=c,
                                           threads=t).v_err[1:m + 1]) for t in range(1, 9)}
        d = [np.abs(np.log10(runs[a] / runs[b])) for a, b in itertools.combinations(runs, 2)]
        print(f"{N}^2 m={m} {c} cycles, threads 1..8 (28 pairs): entrywise max {max(x.max() for x in d):.3f}, "
              f"last {max(x[-1] for x in d):.3f}, median {max(np.median(x) for x in d):.3f} decades; "
              f"first entry {min(r[0] for r in runs.values()):.2e} .. {max(r[0] for r in runs.values()):.2e}")


if __name__ == "__main__":
    main()
