# r06be: GPU suite on the build with 4c - s as one exact fma in every stencil site
# (k_stencil, the short-recurrence marches; GK_FMA4 1), then A/B vs multiply + subtract
# (variant st_fma0): 2 interleaved rounds of the default bench line without the CPU leg
OUT=gpurun_out/r06be
. tools/gpu_lib.sh
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
for v in st_fma0 base; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  step bench_${v}_r$r 300 python -u bench.py --no-cpu
done
done
unset GK_LIB_DIR
