# round-3 GPU call S: MRHS columns in LDS for the compile-time N = 20 kernel
# (libhmpc_mrl.so) vs global columns (libhmpc.so): parity, then configs[3] A/B
set -o pipefail
mkdir -p gpurun_out
HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_mrl.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_riccati_stress.py tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_n60.py > gpurun_out/mrl_tests.log 2>&1; rc=$?; echo "mrl tests rc $rc: $(tail -n 1 gpurun_out/mrl_tests.log)"
[ $rc -eq 0 ] || { grep -B3 -A25 "Error\|assert" gpurun_out/mrl_tests.log | head -60; exit 1; }
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_mrl.so; do
    HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 200 python -u bench.py --N 20 --straight --mu-sweep --global-batch 262144 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', round(d['value']/1e6,4), 'M/s', round(d['roofline']['kernel_ms'],3), 'ms')"
  done
done
