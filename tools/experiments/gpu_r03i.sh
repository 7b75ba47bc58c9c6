# Round 3, call i: the fused stencil stage of the Arnoldi step's Chebyshev
# pass (GK_TUNE_CHEB_STEN): full GPU suite, config-3 bench + rocprof, SQ mix.
OUT=gpurun_out/r03i
source tools/gpu_lib.sh
step gpu_tests 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step bench_cheb 300 python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs
step rocprof_cheb 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cheb -o prof_cheb --output-format csv -- python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs --no-diag
pmc pmc_sq_cheb "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES GRBM_GUI_ACTIVE" python -u bench.py --prec cheb --steps 1 --warmup 0 --no-cpu --no-configs --no-diag --no-prof
echo ALL_DONE
