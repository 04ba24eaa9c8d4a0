#!/bin/bash
# Round-4 call E: parity of the LPT-ordered and reduced-budget builds, then
# the A/B on configs[2], configs[1], configs[3] and the Runner's N = 60.
#   libhmpc_lpt.so   dense split classes served longest-first (HMPC_SPLIT_LPT=1)
#   libhmpc_c152.so  compacted class at a 152-VGPR budget
#   libhmpc_rlpt.so  Riccati work queue served longest-first (HMPC_RIC_LPT=1)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
for v in libhmpc.so libhmpc_lpt.so libhmpc_c152.so; do
  HMPC_LIB=hopper-mpc-inertial_amd/$v timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_overflow.py -k "not kernel_names" > gpurun_out/r04e_tests_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 gpurun_out/r04e_tests_$v.log)"; stop $rc
  [ $rc -eq 0 ] || exit 1
done
HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_rlpt.so timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gpu_n60.py tests/test_gpu_riccati_stress.py -k "not kernel_names" > gpurun_out/r04e_tests_rlpt.log 2>&1; rc=$?; echo "rlpt: $(tail -1 gpurun_out/r04e_tests_rlpt.log)"; stop $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab.py --tag r04e_n60 --rounds 3 --args "--N 60 --straight --batch 4096" libhmpc.so libhmpc_rlpt.so || exit 1
timeout -k 10 900 python tools/ab.py --tag r04e_cfg3 --rounds 2 --args "--N 20 --straight --mu-sweep --global-batch 262144 --steps 20" libhmpc.so libhmpc_rlpt.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04e_cfg2 --rounds 2 libhmpc.so libhmpc_lpt.so libhmpc_c152.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04e_cfg1 --rounds 2 --args "--variant 2f --straight --batch 4096" libhmpc.so libhmpc_lpt.so libhmpc_c152.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04e_b16k --rounds 2 --args "--batch 16384" libhmpc.so libhmpc_lpt.so libhmpc_c152.so || exit 1
