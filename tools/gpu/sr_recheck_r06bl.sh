# r06bl: the short-recurrence legs on the last tree, twice (box-to-box variance check after r06bk)
OUT=gpurun_out/r06bl
. tools/gpu_lib.sh
step sr_1 300 python -u bench.py --sr-only --no-cpu
step sr_2 300 python -u bench.py --sr-only --no-cpu
