# round-3 GPU call AB3: order / concurrency of the dense split's two launches
# (HMPC_SPLIT_MODE 0 concurrent full first, 1 concurrent compacted first,
# 2 serial compacted then full, 3 serial full then compacted)
set -o pipefail
mkdir -p gpurun_out
L=hopper-mpc-inertial_amd
HMPC_SPLIT_MODE=1 HMPC_LIB=$PWD/$L/libhmpc_mode.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/ab3.log 2>&1 || { tail -n 30 gpurun_out/ab3.log; exit 1; }
for rep in 1 2; do
  for m in 0 1 2 3; do
    for cfg in "--steps 100 --warmup 20" "--variant 2f --straight --batch 4096 --steps 100 --warmup 20" "--batch 16384 --steps 100 --warmup 20"; do
      HMPC_SPLIT_MODE=$m HMPC_LIB=$PWD/$L/libhmpc_mode.so timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('mode $m', '$cfg'[:18], round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
    done
  done
done
