#!/bin/bash
# A/B of the N = 20 (two-wave) kernel: parity tests on the new build, then
# configs[3] bench + phase stamps for libhmpc_prev*.so and libhmpc*.so.
set -o pipefail
mkdir -p gpurun_out/ab20
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab20/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab20/tests.log; exit 1; }
tail -1 gpurun_out/ab20/tests.log
for v in prev new; do
  if [ $v = prev ]; then L=hopper-mpc-inertial_amd/libhmpc_prev; else L=hopper-mpc-inertial_amd/libhmpc; fi
  HMPC_LIB=${L}.so timeout -k 10 200 python bench.py --N 20 --batch 262144 --mu-sweep --steps 5 --cpu-seconds 0 > gpurun_out/ab20/bench_$v.json 2> gpurun_out/ab20/bench_$v.err || { echo BENCH $v FAILED; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab20/bench_$v.json')); print('$v', d['value'], d['roofline']['kernel_ms'])"
  N=20 B=65536 HMPC_LIB=${L}_stamps.so timeout -k 10 200 python tools/phase_stamps.py > gpurun_out/ab20/stamps_$v.json 2> gpurun_out/ab20/stamps_$v.err || { echo STAMPS FAILED; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab20/stamps_$v.json')); print('$v', {k: round(x) for k, x in d.items()})"
done
