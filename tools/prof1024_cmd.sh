cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1024 -o b --output-format csv -- python3 bench.py --grid 1024 --steps 2 --warmup 1 --no-cpu --no-prof > gpurun_out/prof1024.json 2> gpurun_out/prof1024.err; echo P1 $?
timeout -k 10 300 python3 bench.py --grid 1024 --steps 3 --warmup 1 --no-cpu --no-prof > gpurun_out/b1024_noprof.json 2>/dev/null; echo B $?
cat gpurun_out/b1024_noprof.json
python3 tools/trace_gaps.py gpurun_out/prof1024/b_kernel_trace.csv
