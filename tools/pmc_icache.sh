#!/bin/bash
# Instruction-cache counters for the default bench (one rocprofv3 pass each).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-icache}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_$TAG
CMD="python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -f csv -d $R/gpurun_out/pmc_$TAG/ic -o run -- $CMD > $R/gpurun_out/pmc_$TAG/ic.log 2>&1 && echo ic ok &&
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -f csv -d $R/gpurun_out/pmc_$TAG/if -o run -- $CMD > $R/gpurun_out/pmc_$TAG/if.log 2>&1 && echo if ok
