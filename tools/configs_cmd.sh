for args in "--prec cheb --degree 8" "--prec cbpr2" "--method hh"; do
  timeout -k 10 400 python bench.py --no-cpu --steps 1 --warmup 1 $args > gpurun_out/cfg.json 2> gpurun_out/cfg.err; echo "RC $? $args"
  python -c "import json; d=json.load(open('gpurun_out/cfg.json')); r=d['roofline'] or {}; print(d['config']['workload'], d['value'], d['ms_per_step'], d['hbm_gbps_alg'], r.get('avg_launch_us'), r.get('per_kernel_ms_sampled'))"
done
