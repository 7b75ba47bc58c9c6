# Round 3, call p: why the bench's config legs run slower per cycle than the
# same config as a headline -- leg order in one process, with and without torch
# touching the device first, and the bench without its diagnostic block.
OUT=gpurun_out/r03p
source tools/gpu_lib.sh
step legs_plain 200 python -u tools/leg_order.py --legs cheb identity cheb identity
step legs_torch 200 python -u tools/leg_order.py --torch-sync --legs cheb identity cheb identity
step bench_nodiag 400 python -u bench.py --no-diag
echo ALL_DONE
