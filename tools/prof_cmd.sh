# rocprofv3 evidence for profiles/: kernel trace + stats of the bench, then
# HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate passes) on the probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-prof > gpurun_out/prof_r01_bench.json 2> gpurun_out/prof_r01_bench.err; echo P1 $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_fetch.log 2>&1; echo P2 $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_write.log 2>&1; echo P3 $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_nt0 -o fetch --output-format csv -- python3 tools/pmc_probe.py --nt 0 > gpurun_out/pmc_fetch_nt0.log 2>&1; echo P4 $?
find gpurun_out/prof_r01 gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_fetch_nt0 -name "*.csv" | head -20
