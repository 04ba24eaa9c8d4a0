#!/bin/bash
# Round-4 call D: the GPU suite on the final build, then the profile evidence
# of every configuration (bench line, rocprofv3 kernel trace + stats, PMC).
set -o pipefail
mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r04d_tests.log; stop $rc
[ $rc -eq 0 ] || exit 1
bash tools/profile.sh r04
