timeout -k 10 600 python tools/tune.py --grid 4096 --rounds 2 --variants base rev=1 blk=1 blk=1:rev=1 unr=2 unr=8 pj=512 rev=1:unr=8 --out gpurun_out/tune4096b.json > gpurun_out/tune4096b.log 2>&1; echo E1 $?
python tools/show_tune.py gpurun_out/tune4096b.json
