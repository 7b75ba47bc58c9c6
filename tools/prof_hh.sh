# rocprofv3 kernel trace + stats of the 4096^2 Householder bench (resident reflection chains)
set -o pipefail
mkdir -p gpurun_out/prof_hh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hh -o hh --output-format csv -- python3 bench.py --method hh --steps 1 --no-cpu --no-prof > gpurun_out/prof_hh/bench.json 2> gpurun_out/prof_hh/bench.err && echo PROF_OK &&
find gpurun_out/prof_hh -name "*kernel_stats.csv" | head -3
