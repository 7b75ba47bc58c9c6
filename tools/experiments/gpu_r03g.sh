# Round 3, call g: Chebyshev pass with the per-level running sum z in LDS (no
# VGPR spill in any variant; 205 VGPRs): parity tests incl. the fused
# epilogues at 1024..4096 and config 3; bench + rocprof; ring depth 2 vs 3 A/B.
OUT=gpurun_out/r03g
source tools/gpu_lib.sh
step cheb_tests 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "cheb or precond or Cheb or config3 or epilogue"
step rocprof_cheb 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cheb -o prof_cheb --output-format csv -- python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs --no-diag
step ab_depth 400 python -u tools/ab_lib.py --variants base cfd3 --rounds 2 -- --prec cheb --steps 2 --warmup 1 --no-diag
echo ALL_DONE
