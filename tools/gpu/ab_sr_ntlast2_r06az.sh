# A/B r06az: non-temporal loads of the march operands read for the last time (previous p / ap:
# GK_SR_NT bit 5 -> 62: also the two-level marches and r in the s pass) vs base (30); 3 rounds interleaved
set -e
mkdir -p gpurun_out/r06az
for r in 1 2 3; do
for v in base nt62; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  timeout -k 10 150 python -u bench.py --sr-only --no-cpu > gpurun_out/r06az/sr_${v}_r${r}.json 2> gpurun_out/r06az/sr_${v}_r${r}.err
done
done
