# A/B r06bh: the Chebyshev pass's output (w) stored non-temporally (variant cf_ntst) vs the
# default policy; 3 interleaved rounds of bench.py --prec cheb (headline = config 3) without
# the CPU leg, SR legs or the other configs; Chebyshev GPU tests on the variant first
OUT=gpurun_out/r06bh
. tools/gpu_lib.sh
export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/cf_ntst
step tests_cheb_ntst 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cheb or Cheb"
for r in 1 2 3; do
for v in base cf_ntst; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  step bench_${v}_r$r 300 python -u bench.py --prec cheb --no-cpu --no-sr --no-configs --steps 3
done
done
unset GK_LIB_DIR
