# A/B r06bc: Chebyshev pass with 4c - s as one exact fma (GK_CF_FMA4 1, default) vs the
# multiply + subtract (variant cf_fma0); Chebyshev GPU tests first, then 2 interleaved rounds
# of the default bench line (no CPU leg, no SR legs) -> configs[2].chebyshev_pass
OUT=gpurun_out/r06bc
. tools/gpu_lib.sh
step tests_cheb 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cheb or Cheb"
for r in 1 2; do
for v in fma0 fma1; do
  if [ $v = fma0 ]; then export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/cf_fma0; else unset GK_LIB_DIR; fi
  step bench_${v}_r$r 300 python -u bench.py --no-cpu --no-sr
done
done
unset GK_LIB_DIR
