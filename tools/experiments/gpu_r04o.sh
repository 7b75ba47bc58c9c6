# Round 4: at the 8-GPU per-GPU load (1448^2 ~ 4096^2 / 8) the byte model ties
# the column cache (8 B/unknown, all 8 chunks per thread cached) with
# k_mgs_res<12,0>: A/B with the column cache forced (--tune 21=1), MGS-R and HH.
OUT=gpurun_out/r04o
source tools/gpu_lib.sh
B="python -u bench.py --no-cpu --no-configs"
step pairs_a 120 $B --grid 1448
step pc_a 120 $B --grid 1448 --tune 21=1
step pairs_b 120 $B --grid 1448
step pc_b 120 $B --grid 1448 --tune 21=1
step hh_pairs 120 $B --grid 1448 --method hh
step hh_pc 120 $B --grid 1448 --method hh --tune 21=1
echo ALL_DONE
