#!/bin/bash
# One GPU call: bench lines for every BASELINE config (tools/bench_configs.sh),
# then rocprofv3 --kernel-trace --stats of the N=20 and N=60 bench commands.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/configs
cd $R
bash tools/bench_configs.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_n20 -o run -- \
  python3 $R/bench.py --N 20 --batch 262144 --mu-sweep --steps 5 --cpu-seconds 0 > $O/trace_n20.log 2>&1 || { echo trace n20 failed; exit 1; }
echo trace n20 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_n60 -o run -- \
  python3 $R/bench.py --N 60 --batch 4096 --steps 3 --warmup 1 --cpu-seconds 0 > $O/trace_n60.log 2>&1 || { echo trace n60 failed; exit 1; }
echo trace n60 ok
