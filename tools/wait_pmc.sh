#!/bin/bash
# What the waves wait on: for one bench configuration,
# PMC passes of the memory-latency counters (one rocprofv3 --pmc run per
# group, each under its own time limit) -- the derived VmemLatency /
# LdsLatency / SmemLatency (in-flight level accumulated / instructions), the
# instruction counts they divide by, the vector L1 (TCP) and address (TA)
# stalls.  tools/wait_summary.py turns them into cycles per wave.
#   bash tools/wait_pmc.sh <tag> <name> <bench args...>
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=$1; NAME=$2; shift 2
O=$R/gpurun_out/$TAG/$NAME
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -f csv -d $O/pmc_$name -o run -- \
    python3 $R/bench.py "${BARGS[@]}" --steps 3 --warmup 1 --prewarm-ms 0 --cpu-seconds 0 > $O/pmc_$name.log 2>&1
}
BARGS=("$@")
run vlat VmemLatency || { echo "$NAME vlat failed"; exit 1; }
run llat LdsLatency || { echo "$NAME llat failed"; exit 1; }
run slat SmemLatency || { echo "$NAME slat failed"; exit 1; }
run sq3 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM_NORM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES || { echo "$NAME sq3 failed"; exit 1; }
run sq4 SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES || { echo "$NAME sq4 failed"; exit 1; }
run tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum || { echo "$NAME tcp failed"; exit 1; }
run ta TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum || { echo "$NAME ta failed"; exit 1; }
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum || { echo "$NAME tcc failed"; exit 1; }
echo "$NAME wait pmc ok"
