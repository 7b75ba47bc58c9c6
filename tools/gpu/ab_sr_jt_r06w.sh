set -e
mkdir -p gpurun_out/r06w
for r in 1 2; do
for b in 0 510 504; do
  timeout -k 10 150 python -u bench.py --sr-only --no-cpu --tune 28=$b > gpurun_out/r06w/sr_b${b}_r${r}.json 2> gpurun_out/r06w/sr_b${b}_r${r}.err
done
done
