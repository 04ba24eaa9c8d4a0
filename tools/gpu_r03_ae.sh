# round-3 GPU call AE: 2f's full class on a 5N-wide compacted kernel
# (solve_kernel<2,10,double,50,20>) instead of the 6N-wide full one:
# dense parity + API tests with it, then interleaved A/B on configs[1] / 2f sizes
set -o pipefail
mkdir -p gpurun_out
L=hopper-mpc-inertial_amd
HMPC_LIB=$PWD/$L/libhmpc_w50.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_overflow.py tests/test_gpu_runner.py tests/test_gpu_dist.py > gpurun_out/ae_tests.log 2>&1 || { echo "w50 tests failed"; grep -B3 -A30 "Error\|assert" gpurun_out/ae_tests.log | head -60; exit 1; }
echo "w50 tests: $(tail -n 1 gpurun_out/ae_tests.log)"
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_w50.so; do
    for cfg in "--variant 2f --straight --batch 4096 --steps 100 --warmup 20" "--variant 2f --batch 65536 --steps 50 --warmup 10" "--steps 100 --warmup 20"; do
      HMPC_LIB=$PWD/$L/$lib timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', '$cfg'[:26], round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms', d['roofline']['kernel'][-40:])"
    done
  done
done
