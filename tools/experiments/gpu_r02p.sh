# Round 2, session D: two-hop exchange in the small-grid kernel only (tests + benches),
# and a rehearsal of the N-rank bench flow on ONE GPU (2 and 4 processes, device
# exchange over IPC, launch-per-projection path): self-launch, gloo control plane,
# max-over-ranks timing, one JSON line with n_gpus = N and its diagnostics.
OUT=gpurun_out/r02p
source tools/gpu_lib.sh
step tests 900 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_solver.py tests/test_gpu_configs.py tests/test_gpu_xgmi.py tests/test_gpu_multirank.py -v --timeout 200 --timeout-method thread
step bench_1024 300 python -u bench.py --no-cpu --steps 20 --warmup 5 --grid 1024
step bench_default 300 python -u bench.py --no-cpu --steps 5 --warmup 1
export GK_BENCH_SAME_DEVICE=1
step rehearse2 300 python -u bench.py --gpus 2 --collective xgmi --no-cpu --steps 2 --warmup 1 --grid 1024
step rehearse4 300 python -u bench.py --gpus 4 --collective xgmi --no-cpu --steps 2 --warmup 1 --grid 1024
echo ALL_DONE
