# Round 2, session E: R2 = 12 prefetch + control-wave variant for slabs of 8..12 chunks per
# thread (the per-GPU slab of 4096^2 on 8 GPUs): full GPU suite, A/B at 1448^2 and 1280^2
# against the two-array variant (nopf12), default bench unchanged.
OUT=gpurun_out/r02aj
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step ab1448 500 python -u tools/ab_lib.py --variants base nopf12 --rounds 3 -- --steps 5 --warmup 1 --no-diag --grid 1448
step ab1280 500 python -u tools/ab_lib.py --variants base nopf12 --rounds 2 -- --steps 5 --warmup 1 --no-diag --grid 1280
step bench_default 300 python -u bench.py --no-cpu --steps 5 --warmup 1
echo ALL_DONE
