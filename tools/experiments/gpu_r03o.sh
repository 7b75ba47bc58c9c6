# Round 3, call o: after the one-HIP-runtime fix (torch imported before the
# native load) -- the full GPU suite, the host wait probe, the default bench,
# multi-rank drift per residual tier, config 4 against the 8192^2 pin.
OUT=gpurun_out/r03o
source tools/gpu_lib.sh
step gpu_tests 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step wait_probe 200 python -u tools/host_wait_probe.py
step bench_default 500 python -u bench.py
step multirank_dev 300 python -u tools/multirank_dev.py
echo ALL_DONE
