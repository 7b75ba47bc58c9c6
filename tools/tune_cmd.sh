timeout -k 10 300 python tools/tune.py --grid 1024 --rounds 3 --variants base unr=2 unr=4 pj=256 pj=256:unr=4 pj=1024:unr=2 --out gpurun_out/tune1024c.json > gpurun_out/tune1024c.log 2>&1; echo E1 $?
python tools/show_tune.py gpurun_out/tune1024c.json
timeout -k 10 600 python tools/tune.py --grid 4096 --rounds 2 --variants base unr=4 --out gpurun_out/tune4096c.json > gpurun_out/tune4096c.log 2>&1; echo E2 $?
python tools/show_tune.py gpurun_out/tune4096c.json
