# A/B r06ap: SR edge loads grouped per half-wave (GK_SR_EDGE_GROUP 1, base) vs per lane (eg0),
# and non-temporal march operand loads on top (GK_SR_NT 15) with / without grouping; 2 rounds
set -e
mkdir -p gpurun_out/r06ap
for r in 1 2; do
for v in base eg0 nt15 nt15eg0; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  timeout -k 10 150 python -u bench.py --sr-only --no-cpu > gpurun_out/r06ap/sr_${v}_r${r}.json 2> gpurun_out/r06ap/sr_${v}_r${r}.err
done
done
