# Round 3, call c: the rewritten Chebyshev pass after the SMALL fix -- the whole
# GPU suite, the config-3 bench line, rocprof kernel stats, and one SQ counter
# pass for the pass's instruction mix (FP64 share of VALU).
OUT=gpurun_out/r03c
source tools/gpu_lib.sh
step gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step bench_cheb 300 python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs
step rocprof_cheb 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cheb -o prof_cheb --output-format csv -- python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs --no-diag
pmc pmc_sq_cheb "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES GRBM_GUI_ACTIVE" python -u bench.py --prec cheb --steps 1 --warmup 0 --no-cpu --no-configs --no-diag --no-prof
echo ALL_DONE
