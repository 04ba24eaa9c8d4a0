#!/bin/bash
# Round-4 call G: the overflow pass's no-overflow fast path (block 0 zeroes
# the counters, no done-counter atomics) against the previous pass.
set -o pipefail
mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_overflow.py tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_n60.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/r04g_tests.log)"; stop $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab.py --tag r04g_cfg1 --rounds 3 --args "--variant 2f --straight --batch 4096" libhmpc.so libhmpc_ovfold.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04g_cfg2 --rounds 2 libhmpc.so libhmpc_ovfold.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04g_n60 --rounds 2 --args "--N 60 --straight --batch 4096" libhmpc.so libhmpc_ovfold.so || exit 1
