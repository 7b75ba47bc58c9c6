# r06bm: the short-recurrence legs on the last tree vs the r06bf build (cf_jtcoarse = the
# Chebyshev coarse line-tile list, otherwise the same sources), 2 interleaved rounds on one box
OUT=gpurun_out/r06bm
. tools/gpu_lib.sh
for r in 1 2; do
for v in cf_jtcoarse base; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  step sr_${v}_r$r 300 python -u bench.py --sr-only --no-cpu
done
done
unset GK_LIB_DIR
