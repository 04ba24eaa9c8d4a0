#!/bin/bash
# Round-4 call C: the whole GPU suite on the default build, the default bench
# line, configs[4] fp32 and fp32 + k fp64 corrections (k = 4, 5, 6).
set -o pipefail
mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r04c_tests.log; stop $rc
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err; rc=$?; stop $rc
python -c "import json; d=json.load(open('gpurun_out/r04c_bench.json')); print('cfg2', round(d['value']/1e6,3), d['roofline']['kernel_ms'], 'q', d['active_mean'], d['fp64_vector']['frac'])"
timeout -k 10 300 python bench.py --precision f32 --cpu-seconds 4 > gpurun_out/r04c_f32.json 2> gpurun_out/r04c_f32.err; rc=$?; stop $rc
python -c "import json; d=json.load(open('gpurun_out/r04c_f32.json')); print('f32', round(d['value']/1e6,3), 'du', d['parity_sample']['max_abs_du_vs_port'])"
for k in 4 5 6; do
  timeout -k 10 300 python bench.py --precision f32_refined --refine $k --cpu-seconds 4 > gpurun_out/r04c_f32r_k$k.json 2> gpurun_out/r04c_f32r_k$k.err; rc=$?; stop $rc
  python -c "import json; d=json.load(open('gpurun_out/r04c_f32r_k$k.json')); print('f32r k=$k', round(d['value']/1e6,3), 'M/s du', d['parity_sample']['max_abs_du_vs_port'], d['parity_sample']['status_mismatch'])"
done
timeout -k 10 600 python tools/ab.py --tag r04c_cfg2 --rounds 2 libhmpc.so libhmpc_filt.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04c_cfg1 --rounds 2 --args "--variant 2f --straight --batch 4096" libhmpc.so libhmpc_filt.so || exit 1
timeout -k 10 900 python tools/ab.py --tag r04c_cfg3 --rounds 2 --args "--N 20 --straight --mu-sweep --global-batch 262144 --steps 10 --warmup 3" libhmpc.so libhmpc_ricold.so || exit 1
timeout -k 10 600 python tools/ab.py --tag r04c_n60 --rounds 2 --args "--N 60 --straight --batch 4096 --steps 10 --warmup 3" libhmpc.so libhmpc_ricold.so || exit 1
