for pe in 0 8 32; do
  if [ $pe = 0 ]; then F=--no-prof; else F="--prof-every $pe"; fi
  timeout -k 10 200 python bench.py --grid 1024 --steps 3 --no-cpu $F > gpurun_out/q.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/q.json')); print('1024 prof_every=$pe', d['value'], d['ms_per_step'], (d['roofline'] or {}).get('avg_launch_us'))"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1024b -o b --output-format csv -- python3 bench.py --grid 1024 --steps 2 --warmup 1 --no-cpu --no-prof > /dev/null 2>&1; echo P $?
python3 tools/trace_gaps.py gpurun_out/prof1024b/b_kernel_trace.csv
