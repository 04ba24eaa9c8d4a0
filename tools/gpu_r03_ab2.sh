# round-3 GPU call AB2: register budgets of the dense split's two kernels
# (full 208 -> 176, compacted 166 -> 152: a SIMD with one full wave then holds
# two compacted ones): parity of each build, then interleaved A/B
set -o pipefail
mkdir -p gpurun_out
L=hopper-mpc-inertial_amd
for v in f176 c152 fc; do
  HMPC_LIB=$PWD/$L/libhmpc_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_overflow.py > gpurun_out/ab2_$v.log 2>&1 || { echo "$v tests failed"; tail -n 30 gpurun_out/ab2_$v.log; exit 1; }
  echo "$v tests: $(tail -n 1 gpurun_out/ab2_$v.log)"
done
for rep in 1 2; do
  for v in base f176 c152 fc; do
    for cfg in "--steps 100 --warmup 20" "--variant 2f --straight --batch 4096 --steps 100 --warmup 20"; do
      HMPC_LIB=$PWD/$L/libhmpc_$v.so timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$v', '$cfg'[:14], round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
    done
  done
done
