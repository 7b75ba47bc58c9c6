# A/B r06z: cache policy of the short-recurrence passes (GK_SR_NT 0 / 2 / 6 / 14), --sr-only legs, 2 rounds interleaved
set -e
mkdir -p gpurun_out/r06z
for r in 1 2; do
for v in base srnt2 srnt6 srnt14; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  timeout -k 10 150 python -u bench.py --sr-only --no-cpu > gpurun_out/r06z/sr_${v}_r${r}.json 2> gpurun_out/r06z/sr_${v}_r${r}.err
done
done
