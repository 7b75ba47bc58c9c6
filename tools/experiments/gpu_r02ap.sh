# Round 2, session E: parity-split ownership of the streamed part (GK_RES_SPAR): resident
# and full-size config tests on the variant, A/B at 4096^2, all-gather trace of the variant.
OUT=gpurun_out/r02ap
source tools/gpu_lib.sh
step tests_spar 600 env GK_LIB_DIR=gmres_amd/lib/variants/spar1 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_configs.py -m gpu -v --timeout 200 --timeout-method thread
step ab4096 600 python -u tools/ab_lib.py --variants base spar1 --rounds 4 -- --steps 3 --warmup 1 --no-diag
step trace_spar 300 env GK_LIB_DIR=gmres_amd/lib/variants/spar1 python -u tools/res_trace.py --grid 4096 --steps 32,64
echo ALL_DONE
