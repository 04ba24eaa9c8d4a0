# round-3 GPU call AG: a narrow third class of the dense split (nf <= 32:
# all-swing windows, solve_kernel<V,10,double,32,13>) vs two classes
set -o pipefail
mkdir -p gpurun_out
L=hopper-mpc-inertial_amd
HMPC_LIB=$PWD/$L/libhmpc_s32.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_overflow.py tests/test_gpu_runner.py tests/test_gpu_dist.py > gpurun_out/ag_tests.log 2>&1 || { echo "s32 tests failed"; grep -B3 -A30 "Error\|assert" gpurun_out/ag_tests.log | head -60; exit 1; }
echo "s32 tests: $(tail -n 1 gpurun_out/ag_tests.log)"
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_s32.so; do
    for cfg in "--steps 100 --warmup 20" "--variant 2f --straight --batch 4096 --steps 100 --warmup 20" "--batch 16384 --steps 100 --warmup 20"; do
      HMPC_LIB=$PWD/$L/$lib timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', '$cfg'[:26], round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
    done
  done
done
