# Round 2, session D: Chebyshev(8) single pass -- unroll / ring-depth variants, kernel stats each.
OUT=gpurun_out/r02j
source tools/gpu_lib.sh
for v in base u6d6 u4d4 u2d2 u6d2; do
  if [ "$v" = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  step prof_$v 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o $v --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --prec cheb
done
echo ALL_DONE
