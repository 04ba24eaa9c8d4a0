#!/bin/bash
# Bench lines for BASELINE.json's GPU configs (and the Runner's N=60) on one
# GPU; each step under its own time limit, stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/configs
mkdir -p $O
cd $R
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  echo "$tag: $(python -c "import json,sys; d=json.load(open('$O/$tag.json')); print(round(d['value']), 'solves/s', round(d['roofline']['kernel_ms'],3), 'ms/launch', d.get('iters_mean'))")"
}
run cfg2_2f_N10_B4096 --variant 2f --N 10 --batch 4096 --straight --cpu-seconds 5
run cfg3_3f_N10_B65536 --cpu-seconds 0
run cfg4_3f_N20_B262144_mu --N 20 --batch 262144 --mu-sweep --steps 5 --cpu-seconds 5
run n60_3f_B4096 --N 60 --batch 4096 --steps 3 --warmup 1 --cpu-seconds 5
