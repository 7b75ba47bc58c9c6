# Round 2, session D: w residency vs column bytes in flight per lane in the w-only
# resident kernel (RW double2 of w in registers, WB double2 per column per batch).
OUT=gpurun_out/r02q
source tools/gpu_lib.sh
step ab_mgs 900 python -u tools/ab_lib.py --variants base rw84wb10 rw80wb12 rw72wb16 --rounds 2 -- --steps 3 --warmup 1 --no-diag
step ab_hh 900 python -u tools/ab_lib.py --variants base rw80wb12 --rounds 2 -- --steps 3 --warmup 1 --no-diag --method hh
echo ALL_DONE
