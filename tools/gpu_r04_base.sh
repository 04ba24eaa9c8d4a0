#!/bin/bash
# Round-4 baseline: the GPU suite and the default bench line on the current build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_base_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_base_tests.log; exit 1; }
tail -2 gpurun_out/r04_base_tests.log
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r04_base_bench.json 2> gpurun_out/r04_base_bench.err || { echo BENCH FAILED; tail gpurun_out/r04_base_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04_base_bench.json')); print('N10', round(d['value']), d['roofline']['kernel_ms'])"
