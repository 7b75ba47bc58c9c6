# Round 3, call m: host wait probe (spin vs blocking event wait, before / after
# torch initialises its HIP context); the default bench with the spin wait and
# the PCIe-inclusive diagnostic; multi-rank drift per residual tier; config-4
# test against the reference's own 8192^2 cycle (now pinned).
OUT=gpurun_out/r03m
source tools/gpu_lib.sh
step wait_probe 200 python -u tools/host_wait_probe.py
step bench_default 500 python -u bench.py
step multirank_dev 300 python -u tools/multirank_dev.py
step config4 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread -k config4
echo ALL_DONE
