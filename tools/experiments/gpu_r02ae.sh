# Round 2, session E: workgroup count of the small-slab resident step (GK_TUNE_RES_SHARE
# 1 / 2 / 4 = 256 / 128 / 64 workgroups) at 1024^2 and 2048^2.
OUT=gpurun_out/r02ae
source tools/gpu_lib.sh
step share1024 300 python -u tools/tune_res_share.py --grid 1024 --shares 1,2,4 --rounds 2 --cycles 5
step share2048 300 python -u tools/tune_res_share.py --grid 2048 --shares 1,2 --rounds 2 --cycles 3
echo ALL_DONE
