# Round 2, session E: N-rank bench rehearsal on one GPU (GK_BENCH_SAME_DEVICE: every rank on
# device 0, the IPC device exchange between processes) after the replicated rank totals.
OUT=gpurun_out/r02am
source tools/gpu_lib.sh
export GK_BENCH_SAME_DEVICE=1
step reh2 300 python -u bench.py --gpus 2 --collective xgmi --steps 2 --warmup 1 --grid 1024 --no-cpu
step reh4 300 python -u bench.py --gpus 4 --collective xgmi --steps 2 --warmup 1 --grid 1024 --no-cpu
echo ALL_DONE
