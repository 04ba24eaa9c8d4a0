# round 5: GPU suite, default bench, the Runner (configs[0]) timing, N=60 trace
set -o pipefail
mkdir -p gpurun_out/r05d
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05d/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05d/tests.log; stop $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r05d/bench.json 2> gpurun_out/r05d/bench.err || exit 1
head -c 300 gpurun_out/r05d/bench.json; echo
timeout -k 10 300 python tools/runner_time.py > gpurun_out/r05d/runner_eager.json 2>&1 || exit 1
timeout -k 10 300 python tools/runner_time.py graph > gpurun_out/r05d/runner_graph.json 2>&1 || exit 1
tail -c 600 gpurun_out/r05d/runner_graph.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r05d/n60 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --N 60 --straight --batch 4096 --steps 10 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/r05d/n60.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r05d/n60 -name "*kernel_stats.csv" -exec cat {} \;
