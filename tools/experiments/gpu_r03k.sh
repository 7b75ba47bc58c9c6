# Round 3, call k: the resident MGS step forming w = A V(:,j) in its prologue
# (GK_TUNE_RES_STEN, k_mgs_wres<..., STEN>): full GPU suite; A/B against the
# stencil launch + resident step; rocprof of the headline.
OUT=gpurun_out/r03k
source tools/gpu_lib.sh
step gpu_tests 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step ab_res_sten 600 python -u tools/ab_lib.py --variants base tune:17=0 --rounds 3 -- --steps 3 --warmup 1
step rocprof_default 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o prof_default --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu --no-configs --no-diag
step bench_default 500 python -u bench.py
echo ALL_DONE
