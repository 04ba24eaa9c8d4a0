#!/bin/bash
# Default-bench A/B over several builds:  tools/ab_libs.sh <lib.so>...
# (parity tests on libhmpc.so first; every step under its own time limit)
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
for rep in 1 2; do
  for L in "$@"; do
    t=$(basename $L .so)
    HMPC_LIB=$L timeout -k 10 200 python bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab/$t.json 2> gpurun_out/ab/$t.err || { echo BENCH $t FAILED; tail -3 gpurun_out/ab/$t.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab/$t.json')); print('$t', round(d['value']), round(d['roofline']['kernel_ms'], 4))"
  done
done
