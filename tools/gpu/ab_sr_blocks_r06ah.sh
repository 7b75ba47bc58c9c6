# A/B r06ah: short-recurrence march geometry on the final tree (NT policy + two-level passes):
# GK_TUNE_SR_BLOCKS 0 (512 -> 64 lines per workgroup) / 768 / 1024 (32 lines), 2 rounds interleaved
set -e
mkdir -p gpurun_out/r06ah
for r in 1 2; do
for b in 0 768 1024; do
  timeout -k 10 150 python -u bench.py --sr-only --no-cpu --tune 28=$b > gpurun_out/r06ah/sr_b${b}_r${r}.json 2> gpurun_out/r06ah/sr_b${b}_r${r}.err
done
done
