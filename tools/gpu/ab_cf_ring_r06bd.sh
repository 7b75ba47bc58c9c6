# A/B r06bd: Chebyshev pass on the fma build -- ring depth 3 (cf_d3) and a scheduling
# barrier after every level (cf_lvbar) vs the default (depth 2, barrier per time step);
# 2 interleaved rounds of the default bench line (no CPU, no SR legs) -> configs[2].chebyshev_pass;
# then rocprofv3 kernel stats of the 4096^2 Chebyshev(8) headline configuration (default build)
OUT=gpurun_out/r06bd
. tools/gpu_lib.sh
for r in 1 2; do
for v in base cf_d3 cf_lvbar; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  step bench_${v}_r$r 300 python -u bench.py --no-cpu --no-sr
done
done
unset GK_LIB_DIR
step prof_cheb 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cheb --output-format csv -- python3 -u bench.py --prec cheb --no-cpu --no-sr --no-configs --steps 2
