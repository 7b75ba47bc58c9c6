timeout -k 10 700 python -m pytest tests -m gpu -q -x > gpurun_out/tall.log 2>&1; echo TESTS $?; tail -15 gpurun_out/tall.log
timeout -k 10 500 python tools/tune.py --grid 4096 --prec cheb --degree 8 --rounds 2 --variants base cf=0 --out gpurun_out/tune_cf.json > gpurun_out/tune_cf.log 2>&1; echo T $?
python tools/show_tune.py gpurun_out/tune_cf.json
