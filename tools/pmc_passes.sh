#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 --pmc pass per counter
# group, each under its own time limit).  Output: gpurun_out/pmc_<tag>/
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0"
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d $R/gpurun_out/pmc_$TAG/$name -o run -- $CMD \
    > $R/gpurun_out/pmc_$TAG/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
mkdir -p $R/gpurun_out/pmc_$TAG
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run grbm GRBM_GUI_ACTIVE GRBM_COUNT &&
run sq2 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES
