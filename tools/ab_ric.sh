#!/bin/bash
# A/B of builds of libhmpc on the Riccati workloads (N=20 configs[3], N=60,
# N=10 on the Riccati kernel).   bash tools/ab_ric.sh libA.so [libB.so ...]
set -o pipefail
mkdir -p gpurun_out/ab
for lib in "$@"; do
  for cfg in "--N 20 --straight --mu-sweep --global-batch 262144" "--N 60 --straight --batch 4096" \
             "--N 10 --precision f64_riccati"; do
    HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 180 python -u bench.py $cfg --steps 5 --warmup 2 \
      --cpu-seconds 3 > gpurun_out/ab/out.json 2> gpurun_out/ab/err.log || { echo "$lib $cfg failed"; tail -5 gpurun_out/ab/err.log; exit 1; }
    python -c "import json;b=json.loads(open('gpurun_out/ab/out.json').read().strip().splitlines()[-1]);p=b['parity_sample'];print('$lib','$cfg',b['roofline']['kernel'],round(b['value']),round(b['roofline']['kernel_ms'],3),b['solved_frac_min_rank'],p['max_abs_du_vs_port'],p['status_mismatch'])"
  done
done
