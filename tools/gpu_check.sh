# full GPU test suite + bench lines (1024^2, 4096^2)
timeout -k 10 700 python -m pytest tests -m gpu -q -x > gpurun_out/tall.log 2>&1; echo TESTS $?; tail -3 gpurun_out/tall.log
timeout -k 10 200 python bench.py --grid 1024 --steps 3 --no-cpu > gpurun_out/b1024.json 2>/dev/null; echo B1 $?
python -c "import json; d=json.load(open('gpurun_out/b1024.json')); print('1024', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'] if d['roofline'] else None)"
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b4096.json 2>/dev/null; echo B2 $?
python -c "import json; d=json.load(open('gpurun_out/b4096.json')); print('4096', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
