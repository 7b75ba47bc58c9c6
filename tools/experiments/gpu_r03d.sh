# Round 3, call d: Chebyshev pass with buffer-descriptor addressing in the
# FAST steps (no spill, no vmcnt(0) drain per trip): its parity tests, config-3
# bench + rocprof; the Infinity-Cache probe (does a non-temporal load still
# leave V_q for the next pass?) and the resident-step A/B of the V_q load
# policy (GK_RES_QNT=1: V_q non-temporal too).
OUT=gpurun_out/r03d
source tools/gpu_lib.sh
step cheb_tests 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "cheb or precond or Cheb or config3"
step bench_cheb 300 python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs
step rocprof_cheb 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cheb -o prof_cheb --output-format csv -- python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs --no-diag
step mall 120 ./tools/mall_probe 4096
step ab_qnt 600 python -u tools/ab_lib.py --variants base qnt --rounds 3 -- --steps 3 --warmup 1
echo ALL_DONE
