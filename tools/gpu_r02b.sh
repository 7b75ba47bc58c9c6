# Round 2, session B: in-kernel time split of the resident launches (pass vs
# exchange wait; MGS-R steps and the Householder UP / DOWN chains at 4096^2 and
# the MGS-R step at 1024^2), then an A/B of the exchange-overlap prefetch (XPF 2).
OUT=gpurun_out/r02b
source tools/gpu_lib.sh
step split4096 300 python -u tools/res_split.py --grid 4096
step split1024 300 python -u tools/res_split.py --grid 1024 --method mgsr
step ab 900 python -u tools/ab_lib.py --variants base x2_88 x2_80 --rounds 2 -- --steps 3 --warmup 1
echo ALL_DONE
