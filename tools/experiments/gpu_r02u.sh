# Round 2, session D: FP64 VALU instruction mix and clock of the Chebyshev(8) pass
# (8 SQ + 2 GRBM counters = one pass) -- its VALU-issue roofline.
OUT=gpurun_out/r02u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $OUT/sq -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag --prec cheb > $OUT/sq.out 2> $OUT/sq.err
echo rc=$?
