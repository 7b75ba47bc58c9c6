# A/B r06ar: SR marches with XCD-aware line-block placement (GK_SR_XCD 1) vs base; 3 rounds
set -e
mkdir -p gpurun_out/r06ar
for r in 1 2 3; do
for v in base xcd1; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  timeout -k 10 150 python -u bench.py --sr-only --no-cpu > gpurun_out/r06ar/sr_${v}_r${r}.json 2> gpurun_out/r06ar/sr_${v}_r${r}.err
done
done
