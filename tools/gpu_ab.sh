#!/bin/bash
# One GPU call for an A/B of library builds (or of bench arguments):
# parity tests on every library, then tools/ab.py interleaved runs.
#   bash tools/gpu_ab.sh TAG "BENCH ARGS" lib_a.so lib_b.so ...
#   VARY="--order=index --order=longest_first" bash tools/gpu_ab.sh TAG "--N 60 --batch 4096"
# Build the variants first on the CPU, e.g.
#   BDIR=build_x OUT=libhmpc_x.so hopper-mpc-inertial_amd/build.sh -DSOME_FLAG=1
# TESTS overrides the parity test files (default: dense, Riccati, overflow,
# order).  Results: gpurun_out/ab/TAG.json.
set -o pipefail
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/ab
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gpu_n60.py tests/test_gpu_order.py"}
LIBS=${*:-libhmpc.so}
for v in $LIBS; do
  HMPC_LIB=hopper-mpc-inertial_amd/$v timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    $TESTS -k "not kernel_names" > gpurun_out/ab/${TAG}_tests_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/ab/${TAG}_tests_$v.log)"; stop $rc
  [ $rc -eq 0 ] || exit 1
done
if [ -n "${VARY:-}" ]; then
  V=""; for x in $VARY; do V="$V --vary=$x"; done
  timeout -k 10 1000 python tools/ab.py --tag $TAG --rounds ${ROUNDS:-2} --args "$ARGS" $V
else
  timeout -k 10 1000 python tools/ab.py --tag $TAG --rounds ${ROUNDS:-2} --args "$ARGS" "$@"
fi
