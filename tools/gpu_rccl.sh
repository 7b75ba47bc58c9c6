timeout -k 10 700 python -m pytest tests -m gpu -q > gpurun_out/tall.log 2>&1; echo TESTS $?; tail -5 gpurun_out/tall.log
GK_FORCE_RCCL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --grid 1024 --steps 2 --warmup 1 --no-cpu > gpurun_out/b_rccl1.json 2> gpurun_out/b_rccl1.err; echo R $?
tail -c 600 gpurun_out/b_rccl1.json; tail -3 gpurun_out/b_rccl1.err
