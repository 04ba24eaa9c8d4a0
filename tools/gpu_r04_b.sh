#!/bin/bash
# Round-4 call B: fp32 + fp64 refinement (parity, bench per k), dense split
# launch-policy A/B (P0 round-3 arrangement ... P5), configs[2] and configs[1].
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_overflow.py > gpurun_out/r04b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r04b_tests.log; stop $rc
[ $rc -eq 0 ] || { echo "DEFAULT TESTS FAILED"; exit 1; }
timeout -k 10 300 $T tests/test_gpu_f32.py > gpurun_out/r04b_f32.log 2>&1; rc=$?; tail -25 gpurun_out/r04b_f32.log; stop $rc
for k in 2 3; do
  timeout -k 10 300 python bench.py --precision f32_refined --refine $k --cpu-seconds 4 > gpurun_out/r04b_f32r_k$k.json 2> gpurun_out/r04b_f32r_k$k.err; rc=$?; stop $rc
  [ $rc -eq 0 ] && python -c "import json; d=json.load(open('gpurun_out/r04b_f32r_k$k.json')); print('f32r k=$k', round(d['value']/1e6,3), 'M/s du', d['parity_sample']['max_abs_du_vs_port'], d['parity_sample']['status_mismatch'])" || tail -5 gpurun_out/r04b_f32r_k$k.err
done
timeout -k 10 900 python tools/ab.py --tag r04b_cfg2 --rounds 2 libhmpc.so libhmpc_p1.so libhmpc_p2.so libhmpc_p4.so libhmpc_p5.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04b_cfg1 --rounds 2 --args "--variant 2f --straight --batch 4096" libhmpc.so libhmpc_p1.so libhmpc_p4.so libhmpc_p5.so || exit 1
timeout -k 10 300 python tools/ab.py --tag r04b_cfg4 --rounds 1 --args "--precision f32" libhmpc.so || exit 1
