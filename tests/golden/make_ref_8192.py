"""Config 4's grid run by the REFERENCE itself: gmres_mgsr_omp at 8192^2,
m = 95, one restart cycle, b = A*1, x0 = 0 (oracle/_ref/ref_driver, the
reference's own src/*.f90 built by oracle/Makefile.ref).

The fixture pins the single-context 8192^2 run that
tests/test_gpu_configs.py::test_config4_* compares the 8 row-block ranks with
(its cycle-1 true residual).  V alone is 51.5 GB of host memory at this size,
more than the build container holds, so this runs on the GPU box's host cores
(the prebuilt oracle/_ref/ref_driver travels with the tree; no GPU is used):

  python tests/golden/make_ref_8192.py OUT.json [CYCLES]  # on the box, ~3 min per cycle
  python tests/golden/make_ref_8192.py --merge OUT.json   # here: into reference_runs.json

A heartbeat line is printed every 30 s while the reference runs.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

def key(cycles: int) -> str:
    return f"mgsr_omp_identity_8192_m95_{cycles}cyc_t16"


def run(out: str, cycles: int = 1) -> None:
    from oracle import refrun

    stop = threading.Event()

    def beat():
        t0 = time.time()
        while not stop.wait(30):
            print(f"reference 8192^2 running: {time.time() - t0:.0f} s", flush=True)

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    t0 = time.time()
    try:
        r = refrun.run("mgsr_omp", 8192, 95, "identity", threads=16, max_cycles=cycles, timeout=1100,
                       env={"OMP_PROC_BIND": "close", "OMP_PLACES": "cores"})
    finally:
        stop.set()
    d = {"solver": "mgsr_omp", "N": 8192, "m": 95, "prec": "identity", "threads": r.threads, "max_cycles": cycles,
         "cut": r.cut, "hist_res": r.hist_res.tolist(), "wall_s": round(time.time() - t0, 2),
         "host": "the GPU box's host cores (oracle/_ref/ref_driver, OMP_NUM_THREADS=16)"}
    json.dump({key(cycles): d}, open(out, "w"), indent=1)
    print(json.dumps(d), flush=True)


def merge(src: str) -> None:
    path = os.path.join(HERE, "reference_runs.json")
    ref = json.load(open(path))
    ref.update(json.load(open(src)))
    json.dump(dict(sorted(ref.items())), open(path, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--merge":
        merge(sys.argv[2])
    else:
        run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
