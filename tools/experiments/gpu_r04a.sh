# Round 4, first GPU call: the new multi-rank tests (4 / 8 ranks on the
# resident kernels, config 4 resident, 4-process IPC), the runtime tests,
# the history fixtures, the Chebyshev stencil stage on slabs; then a
# torch-free default bench line and the 2896^2 single-rank kernel
# (k_mgs_res<12,18> NT, the per-GPU kernel of 4096^2/2 and 8192^2/8).
OUT=gpurun_out/r04a
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
step t_runtime 300 $T tests/test_gpu_runtime.py
step t_splits 900 $T tests/test_gpu_splits.py
step t_configs 600 $T tests/test_gpu_configs.py
step t_hist 300 $T tests/test_gpu_solver.py -k "twelve_cycle"
step t_multirank 400 $T -s tests/test_gpu_multirank.py -k "stencil_stage or rccl or graphs"
step t_bench2 200 $T tests/test_gpu_xgmi.py -k "bench_two_ranks"
step bench_default 500 python -u bench.py
step bench_2896 300 python -u bench.py --grid 2896 --no-cpu --no-configs
step bench_2896_qdef 300 python -u bench.py --grid 2896 --no-cpu --no-configs --tune 20=1
step bench_2896b 300 python -u bench.py --grid 2896 --no-cpu --no-configs
step bench_2896_qdefb 300 python -u bench.py --grid 2896 --no-cpu --no-configs --tune 20=1
step bench_2048 300 python -u bench.py --grid 2048 --no-cpu --no-configs
step bench_1448 300 python -u bench.py --grid 1448 --no-cpu --no-configs
step split_2896 300 python -u tools/res_split.py --grid 2896 --method mgsr
step trace_2896 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_2896" -o t2896 --output-format csv -- python3 bench.py --grid 2896 --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
