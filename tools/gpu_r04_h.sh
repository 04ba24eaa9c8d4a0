#!/bin/bash
# Round-4 call H: the N = 60 Riccati kernel with BW in the global slot
# (32.2 KB of LDS -> 5 workgroups / CU at the 2-wave register budget,
# libhmpc_bwg.so) against the 1-wave kernel (libhmpc.so) and the previous
# Riccati source (libhmpc_old.so: BW loads not hoisted to the stage top).
set -o pipefail
mkdir -p gpurun_out/r04h
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for v in libhmpc.so libhmpc_bwg.so; do
  HMPC_LIB=hopper-mpc-inertial_amd/$v timeout -k 10 400 $T tests/test_gpu_n60.py tests/test_gpu_riccati_stress.py tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_overflow.py -k "not kernel_names" > gpurun_out/r04h/tests_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/r04h/tests_$v.log)"; stop $rc
  [ $rc -eq 0 ] || exit 1
done
cd /tmp && export TMPDIR=/tmp
HMPC_LIB=$GRAFT_REPO_ROOT/hopper-mpc-inertial_amd/libhmpc_bwg.so timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r04h/trace_bwg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --N 60 --straight --batch 4096 --steps 3 --warmup 1 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/r04h/trace_bwg.log 2>&1; rc=$?; stop $rc
cd $GRAFT_REPO_ROOT
AB="timeout -k 10 900 python tools/ab.py --rounds 3"
$AB --tag r04h_n60 --args "--N 60 --straight --batch 4096" libhmpc.so libhmpc_bwg.so libhmpc_old.so || exit 1
$AB --tag r04h_n60_16k --args "--N 60 --straight --batch 16384" libhmpc.so libhmpc_bwg.so || exit 1
timeout -k 10 900 python tools/ab.py --rounds 2 --tag r04h_cfg3 --args "--N 20 --straight --mu-sweep --global-batch 262144 --steps 20" libhmpc.so libhmpc_old.so || exit 1
