#!/bin/bash
# round 5: the streamed elements (the ragged tail past the resident chunks) from the LAST
# workgroup down instead of from workgroup 0 (r05ac's trace: workgroup 0 the straggler of
# every 1448^2 exchange).  Trace at 1448^2 (strict, S = 4), then bench lines alternating the
# main build with the round-4 assignment (variant swg0) at 1448^2 (strict, S = 4) and 2896^2
# (strict), then the whole GPU suite on the main build.
OUT=gpurun_out/r05ad
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
V=$PWD/gmres_amd/lib/variants
R="python -u tools/res_trace.py --grid 1448"
step tr_strict 200 $R
step tr_s4 200 $R --tune 23=4
for f in tr_strict tr_s4; do echo "== $f"; cut -c1-420 $OUT/$f.out; done
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
for k in 1 2; do
  for v in base swg0; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    for pt in "1448 1" "1448 4" "2896 1"; do
      set -- $pt
      step b_${v}_$1_s$2_$k 150 $B --grid $1 --tune 23=$2
      python - $OUT/b_${v}_$1_s$2_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
    done
  done
done
unset GK_LIB_DIR
step gpu_tests 1000 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests -m gpu
tail -3 $OUT/gpu_tests.out
echo ALL_DONE
