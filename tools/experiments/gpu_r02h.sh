# Round 2, session D: per-kernel time of the Chebyshev passes per variant (rocprofv3 stats).
OUT=gpurun_out/r02h
source tools/gpu_lib.sh
for v in base cfd1 cfd2 cfd3 cfjt128 cfd2jt128; do
  if [ "$v" = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  step prof_$v 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o $v --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --prec cheb
done
echo ALL_DONE
