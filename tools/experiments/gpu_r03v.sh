# Round 3: N-rank bench rehearsal on one GPU with the final tree (every rank on
# device 0, the IPC device exchange between processes; the driver's default
# --collective auto), x kept in HBM by the timed solves.
OUT=gpurun_out/r03v
source tools/gpu_lib.sh
export GK_BENCH_SAME_DEVICE=1
step reh2_1024 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --grid 1024 --no-cpu
step reh4_1024 300 python -u bench.py --gpus 4 --steps 2 --warmup 1 --grid 1024 --no-cpu
step reh2_4096 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu
step reh2_4096_hh 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --method hh
step reh2_4096_cheb 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --prec cheb
echo ALL_DONE
