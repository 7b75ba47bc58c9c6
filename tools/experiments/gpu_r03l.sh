# Round 3, call l: default-off resident stencil prologue (GK_TUNE_RES_STEN 0):
# the default bench; the config legs alone twice (the 1024^2 leg read 2,142
# it/s beside 2,569 from tools/solve_overhead.py); the reference itself at
# 8192^2 on the box's host cores (config 4's pin, tests/golden/make_ref_8192.py).
OUT=gpurun_out/r03l
source tools/gpu_lib.sh
step bench_default 500 python -u bench.py
step legs 300 python -u -c "import json, bench, gmres_amd as ga; print(json.dumps(bench.config_legs(ga, 16))); print(json.dumps(bench.config_legs(ga, 16)))"
step ref8192 900 python -u tests/golden/make_ref_8192.py gpurun_out/r03l/ref8192.json
echo ALL_DONE
