#!/bin/bash
# round 5: PMC traffic of the opt-in blocked step (S = 4) over one full cycle at 1024^2 (the
# config-2 leg) and 1448^2 (the 4096^2 / 8 load): FETCH_SIZE and WRITE_SIZE in separate passes.
OUT=gpurun_out/r05am
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
for g in 1024 1448; do
  pmc pmc_fetch_blk4_$g FETCH_SIZE python3 bench.py --grid $g --tune 23=4 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
  pmc pmc_write_blk4_$g WRITE_SIZE python3 bench.py --grid $g --tune 23=4 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
done
echo ALL_DONE
