# Round 2, session D: SQ counters of the Chebyshev(8) pass (what limits it: VALU issue,
# waiting on memory, or instruction issue stalls).  8 SQ counters = one pass.
OUT=gpurun_out/r02s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD -d $OUT/sq -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag --prec cheb > $OUT/sq.out 2> $OUT/sq.err
echo rc=$?
