# Round 3: the two-rank bench line with the default collective as a GPU test.
OUT=gpurun_out/r03z
source tools/gpu_lib.sh
step test_bench2 300 python -u -m pytest tests/test_gpu_xgmi.py -k "bench_two_ranks or slabs_match" -v --timeout 150 --timeout-method thread
echo ALL_DONE
