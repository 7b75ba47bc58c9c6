# Round-1 evidence: bench lines, rocprofv3 kernel trace + PMC passes -> gpurun_out/ev/
mkdir -p gpurun_out/ev
timeout -k 10 600 python bench.py > gpurun_out/ev/bench_default.json 2> gpurun_out/ev/bench_default.err; echo B0 $?
for cfg in "cheb --degree 8:cheb8" "cbpr2:cbpr2"; do
  a=${cfg%%:*}; n=${cfg##*:}
  timeout -k 10 400 python bench.py --no-cpu --prec $a > gpurun_out/ev/bench_$n.json 2>/dev/null; echo B_$n $?
done
timeout -k 10 400 python bench.py --no-cpu --method hh > gpurun_out/ev/bench_hh.json 2>/dev/null; echo B_hh $?
timeout -k 10 300 python bench.py --no-cpu --grid 1024 --steps 3 > gpurun_out/ev/bench_1024.json 2>/dev/null; echo B_1024 $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/trace -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-prof > gpurun_out/ev/trace_bench.json 2>/dev/null; echo P1 $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/trace_cheb8 -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-prof --prec cheb --degree 8 > gpurun_out/ev/trace_cheb8.json 2>/dev/null; echo P2 $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ev/pmc_fetch -o fetch --output-format csv -- python3 tools/pmc_probe.py > /dev/null 2>&1; echo P3 $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ev/pmc_write -o write --output-format csv -- python3 tools/pmc_probe.py > /dev/null 2>&1; echo P4 $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ev/pmc_fetch_cheb -o fetch --output-format csv -- python3 tools/pmc_probe.py --prec cheb > /dev/null 2>&1; echo P5 $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ev/pmc_write_cheb -o write --output-format csv -- python3 tools/pmc_probe.py --prec cheb > /dev/null 2>&1; echo P6 $?
for f in gpurun_out/ev/bench_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); r=d['roofline'] or {}; print('$f', d['value'], d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'), (d.get('cpu_baseline') or {}).get('value'))"; done
