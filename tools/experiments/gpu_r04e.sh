# Round 4, fifth call: the column-cache kernel with the next pass's dot column
# touched into L2 during each all-gather (28 chunks, default) against 0 and 16
# (GK_LIB_DIR builds) and k_mgs_res (--tune 21=0) at 2896^2 / 2048^2; the
# resident tests; the default bench line (unchanged kernel) as a control.
OUT=gpurun_out/r04e
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
step t_resident 600 $T tests/test_gpu_resident.py
step b2896 120 $B --grid 2896
step b2896_t0 120 env GK_LIB_DIR=gmres_amd/lib/variants/pct0 $B --grid 2896
step b2896_t16 120 env GK_LIB_DIR=gmres_amd/lib/variants/pct16 $B --grid 2896
step b2896_old 120 $B --grid 2896 --tune 21=0
step b2896b 120 $B --grid 2896
step b2896_t0b 120 env GK_LIB_DIR=gmres_amd/lib/variants/pct0 $B --grid 2896
step b2048 120 $B --grid 2048
step b2048_t0 120 env GK_LIB_DIR=gmres_amd/lib/variants/pct0 $B --grid 2048
step b2048_t16 120 env GK_LIB_DIR=gmres_amd/lib/variants/pct16 $B --grid 2048
step b2048_old 120 $B --grid 2048 --tune 21=0
step b2896_hh 120 $B --grid 2896 --method hh
step b2896_hh_old 120 $B --grid 2896 --method hh --tune 21=0
step b4096 300 $B
echo BENCH_DONE
# the reference itself at 8192^2 for TWO cycles on this host's 16 cores (no GPU): pins config 4's cycle 2
step ref8192 1000 python -u tests/golden/make_ref_8192.py gpurun_out/r04e/ref8192_2cyc.json 2
echo REF_DONE
