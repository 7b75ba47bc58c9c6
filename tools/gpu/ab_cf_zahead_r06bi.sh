# A/B r06bi: Chebyshev pass with the z of level l+2 read while level l computes (cf_za2)
# vs one level ahead (default); Chebyshev GPU tests on the variant, then 3 interleaved
# rounds of bench.py --prec cheb --steps 3 (config 3 as the headline) without the CPU leg
OUT=gpurun_out/r06bi
. tools/gpu_lib.sh
export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/cf_za2
step tests_cheb_za2 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cheb or Cheb"
for r in 1 2 3; do
for v in base cf_za2; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  step bench_${v}_r$r 300 python -u bench.py --prec cheb --no-cpu --no-sr --no-configs --steps 3
done
done
unset GK_LIB_DIR
