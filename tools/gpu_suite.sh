#!/bin/bash
# One GPU call: the whole GPU suite on the default build, then the profile
# evidence of every configuration (tools/profile.sh <tag>: bench line,
# rocprofv3 kernel trace + stats, PMC passes).  Summarise afterwards on the
# CPU with `python tools/summarize.py <tag>`.
#   /usr/local/graft/bin/gpurun --timeout 1500 -- bash tools/gpu_suite.sh r04
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log; stop $rc
[ $rc -eq 0 ] || exit 1
bash tools/profile.sh $TAG
