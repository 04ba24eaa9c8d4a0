#!/bin/bash
# Profile evidence, one GPU call: for each configuration a bench line,
# a rocprofv3 --kernel-trace --stats run of the same command and the PMC
# passes (one rocprofv3 --pmc run per counter group, each under its own time
# limit).  Outputs gpurun_out/<tag>/<cfg>/; tools/summarize.py copies the
# judged summaries into profiles/.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r04}
shift || true
CFGS=${CFGS:-"n10 n20 n60 n10_2f n10_f32 n10_f32r"}
declare -A ARGS=(
  [n10]="--N 10"
  [n20]="--N 20 --straight --mu-sweep --global-batch 262144"
  [n60]="--N 60 --straight --batch 4096"
  [n10_2f]="--variant 2f --N 10 --straight --batch 4096"
  [n10_f32]="--N 10 --precision f32"
  [n10_f32r]="--N 10 --precision f32_refined --refine 5"
)
for cfg in $CFGS; do
  O=$R/gpurun_out/$TAG/$cfg
  mkdir -p $O
  A=${ARGS[$cfg]}
  cd $R
  timeout -k 10 300 python bench.py $A > $O/bench.json 2> $O/bench.err || { echo "$cfg bench failed"; exit 1; }
  echo "$cfg bench ok"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- \
    python3 $R/bench.py $A --steps 10 --cpu-seconds 0 > $O/trace.log 2>&1 || { echo "$cfg trace failed"; exit 1; }
  echo "$cfg trace ok"
  run() {
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d $O/pmc_$name -o run -- \
      python3 $R/bench.py $A --steps 3 --warmup 1 --prewarm-ms 0 --cpu-seconds 0 > $O/pmc_$name.log 2>&1
  }
  run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY || { echo "$cfg sq1 failed"; exit 1; }
  run fetch FETCH_SIZE || { echo "$cfg fetch failed"; exit 1; }
  run write WRITE_SIZE || { echo "$cfg write failed"; exit 1; }
  run sq2 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES || { echo "$cfg sq2 failed"; exit 1; }
  run grbm GRBM_GUI_ACTIVE GRBM_COUNT || { echo "$cfg grbm failed"; exit 1; }
  run tcc TCC_HIT_sum TCC_MISS_sum || { echo "$cfg tcc failed"; exit 1; }
  echo "$cfg pmc ok"
done
