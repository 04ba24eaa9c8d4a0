#!/bin/bash
# BASELINE configs[4]: fp32 vs fp64 at N=10, B=65536 (3f, curve).  The
# parity_sample of each line is max|u - u_port| over all instances.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/precision
mkdir -p $O
cd $R
for p in f64 f64_generic f32; do
  timeout -k 10 300 python bench.py --precision $p --cpu-seconds 3 > $O/$p.json 2> $O/$p.err || { echo "$p failed"; tail -5 $O/$p.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$p.json')); print('$p', round(d['value']), 'solves/s', round(d['roofline']['kernel_ms'], 3), 'ms', 'solved', d['solved_frac_min_rank'], 'max|du| vs port', d['parity_sample'])"
done
