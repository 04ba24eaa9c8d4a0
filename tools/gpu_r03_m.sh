# round-3 GPU call M: compile-time N = 20 Riccati kernel (ric_kernel<3,2,20,38>)
# A/B against the runtime-N kernel on configs[3], then its parity tests
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_ric20.so; do
    HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 200 python -u bench.py --N 20 --straight --mu-sweep --global-batch 262144 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', d['roofline']['kernel'], round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],3), 'ms')"
  done
done
HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_ric20.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_riccati_stress.py tests/test_gpu_overflow.py tests/test_gpu_wide.py > gpurun_out/ric20_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/ric20_tests.log; exit $rc
