# A/B of the w-only register residency (RES_RW double2 of w per lane): 64 (tree), 80, 88
set -o pipefail
mkdir -p gpurun_out/ab_rw
for rep in 1 2; do
  for v in base rw80 rw88; do
    if [ $v = base ]; then b=bench.py; else b=abtest/$v/bench.py; fi
    timeout -k 10 200 python -u $b --no-cpu > gpurun_out/ab_rw/${v}_$rep.json 2> gpurun_out/ab_rw/${v}_$rep.err || { echo FAIL $v; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_rw/${v}_$rep.json')); print('$v', $rep, d['value'], d['roofline']['per_projection_us'], d['check']['true_rel_residual_after_timed_cycles'])"
  done
done
for v in base rw88; do
  if [ $v = base ]; then b=bench.py; else b=abtest/$v/bench.py; fi
  timeout -k 10 200 python -u $b --no-cpu --method hh > gpurun_out/ab_rw/${v}_hh.json 2> gpurun_out/ab_rw/${v}_hh.err || { echo FAIL $v hh; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_rw/${v}_hh.json')); print('$v hh', d['value'], d['roofline']['per_projection_us'])"
done
