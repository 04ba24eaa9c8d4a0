set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b/tests.log 2>&1; rc=$?
tail -15 gpurun_out/r05b/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r05b/bench.json 2> gpurun_out/r05b/bench.err || exit 1
head -c 400 gpurun_out/r05b/bench.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r05b/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/r05b/trace.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r05b/trace -name "*kernel_stats.csv" -exec cat {} \;
