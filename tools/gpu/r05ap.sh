#!/bin/bash
# round 5: the strict step on the prefetching blocked kernel (GK_TUNE_RES_PF 1) again, now
# with the 96 KiB prefetch cap (12 of 16 chunks at the 2048^2 load): single GPU at 2048^2 and
# 2896^2, and the 2-rank rehearsal at 2896^2 (2048^2 per rank on 128 CUs... the per-rank load
# of 4096^2 on 4 GPUs is 2048^2 on 256), alternating twice.
OUT=gpurun_out/r05ap
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
B="python -u bench.py --no-cpu --no-configs"
for k in 1 2; do
  for pf in 0 1; do
    for g in 2048 1448; do
      step b_${g}_pf${pf}_$k 150 $B --steps 4 --warmup 1 --grid $g --tune 27=$pf
      python - $OUT/b_${g}_pf${pf}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"], d["config"]["resident_variant"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
    done
    step reh4_2048_pf${pf}_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048 --tune 27=$pf
    python - $OUT/reh4_2048_pf${pf}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["config"]["resident_variant"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
  done
done
echo ALL_DONE
