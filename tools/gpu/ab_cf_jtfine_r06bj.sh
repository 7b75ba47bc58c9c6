# A/B r06bj: Chebyshev pass line tile JT picked from every even value 16..256 (default,
# GK_CF_JTFINE 1: 4096^2 -> JT 78, 2014 workgroups) vs the coarse list (cf_jtcoarse: JT 80,
# 1976); Chebyshev GPU tests on the default, then 3 interleaved rounds of bench.py --prec cheb
OUT=gpurun_out/r06bj
. tools/gpu_lib.sh
step tests_cheb 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cheb or Cheb"
for r in 1 2 3; do
for v in cf_jtcoarse base; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  step bench_${v}_r$r 300 python -u bench.py --prec cheb --no-cpu --no-sr --no-configs --steps 3
done
done
unset GK_LIB_DIR
