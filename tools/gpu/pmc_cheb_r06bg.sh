# r06bg: SQ counters of the Chebyshev(8) pass on the last tree (one pass of 8 SQ counters)
OUT=gpurun_out/r06bg
. tools/gpu_lib.sh
pmc pmc_sq_cheb "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" python3 -u bench.py --prec cheb --no-cpu --no-sr --no-configs --no-diag --steps 1 --warmup 0
