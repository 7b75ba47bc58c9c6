#!/bin/bash
# round 5: the strict step on the prefetching blocked kernel (GK_TUNE_RES_PF 1) with its
# prefetch issued by the waves that do not poll (so a rank-total pusher's push does not queue
# behind it; main build) vs every wave its own (variant split0) vs the strict default (pf 0):
# single GPU at 2048^2 / 1448^2, 4 ranks at 2048^2, 8 ranks at 1448^2; twice.
OUT=gpurun_out/r05aq
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
( while sleep 45; do date +%T >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
V=$PWD/gmres_amd/lib/variants
B="python -u bench.py --no-cpu --no-configs"
show() {
  python - $OUT/$1.out <<'PY' || true
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["config"]["resident_variant"],
      d["diagnostics"]["resident_split_per_unit_us"].get("mgs_step"))
PY
}
for k in 1 2; do
  for v in strict pfsplit pf0split; do
    case $v in
      strict) unset GK_LIB_DIR; T="--tune 27=0";;
      pfsplit) unset GK_LIB_DIR; T="--tune 27=1";;
      pf0split) export GK_LIB_DIR=$V/split0; T="--tune 27=1";;
    esac
    step s2048_${v}_$k 150 $B --steps 4 --warmup 1 --grid 2048 $T; show s2048_${v}_$k
    step s1448_${v}_$k 150 $B --steps 4 --warmup 1 --grid 1448 $T; show s1448_${v}_$k
    step reh4_${v}_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048 --no-diag $T; show reh4_${v}_$k
    step reh8_${v}_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 8 --grid 1448 --steps 2 --warmup 1 --collective xgmi --tune 24=60000 --no-diag $T; show reh8_${v}_$k
  done
done
unset GK_LIB_DIR
echo ALL_DONE
