#!/bin/bash
# Round-4 call A: parity of the persistent split (default build) and the
# narrow-class builds, then the dense split A/B on configs[2] and configs[1].
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_overflow.py tests/test_gpu_runner.py > gpurun_out/r04a_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r04a_tests.log; exit 1; }
tail -1 gpurun_out/r04a_tests.log
for v in sml4 sml3 np; do
  HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_$v.so timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_overflow.py -k "not kernel_names" > gpurun_out/r04a_tests_$v.log 2>&1 || { echo TESTS $v FAILED; tail -40 gpurun_out/r04a_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r04a_tests_$v.log)"
done
timeout -k 10 900 python tools/ab.py --tag r04a_cfg2 --rounds 2 libhmpc_np.so libhmpc.so libhmpc_sml4.so libhmpc_sml3.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04a_cfg1 --rounds 2 --args "--variant 2f --straight --batch 4096" libhmpc_np.so libhmpc.so libhmpc_sml4.so || exit 1
