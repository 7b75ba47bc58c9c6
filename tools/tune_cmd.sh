timeout -k 10 400 python tools/tune.py --grid 4096 --rounds 2 --variants base nt=1 pj=1024 nt=1:pj=1024 pj=4096 nt=1:pj=4096 --out gpurun_out/tune4096.json > gpurun_out/tune4096.log 2>&1; echo E1 $?
python tools/show_tune.py gpurun_out/tune4096.json
timeout -k 10 300 python tools/tune.py --grid 1024 --rounds 3 --variants base nt=1 pj=256 pj=1024 st=512 --out gpurun_out/tune1024.json > gpurun_out/tune1024.log 2>&1; echo E2 $?
python tools/show_tune.py gpurun_out/tune1024.json
