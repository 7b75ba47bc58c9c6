# Round 2, session B: new multi-rank Chebyshev deep-halo tests + the whole GPU
# suite, in-kernel time split of the resident launches (pass vs exchange wait;
# MGS-R steps and the Householder UP / DOWN chains at 4096^2, MGS-R at 1024^2),
# then an A/B of the exchange-overlap prefetch (XPF 2).
OUT=gpurun_out/r02b
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
step split4096 300 python -u tools/res_split.py --grid 4096
step split1024 300 python -u tools/res_split.py --grid 1024 --method mgsr
step ab 900 python -u tools/ab_lib.py --variants base x2_88 x2_80 --rounds 2 -- --steps 3 --warmup 1
echo ALL_DONE
