#!/bin/bash
# One GPU call: smoke, the default bench (with its CPU baseline), a rocprofv3
# kernel-trace --stats run of the same bench, and the PMC passes.  Every GPU
# step has its own time limit; the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r01}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 10 --cpu-seconds 0 > $O/trace.log 2>&1 || { echo trace failed; exit 1; }
echo trace ok
cd $R && bash tools/pmc_passes.sh $TAG
