# Round 2, session E: all-gather anatomy of the resident MGS-R step (gk_profile_res_trace):
# publish / seen stamps per workgroup and exchange at 4096^2, 2048^2, 1024^2; full GPU suite;
# default bench (the trace is off there).
OUT=gpurun_out/r02y
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step trace4096 300 python -u tools/res_trace.py --grid 4096 --steps 16,48,80
step trace2048 300 python -u tools/res_trace.py --grid 2048 --steps 16,48,80
step trace1024 300 python -u tools/res_trace.py --grid 1024 --steps 16,48,80
step bench_default 300 python -u bench.py --no-cpu --steps 10 --warmup 2
echo ALL_DONE
