# round-3 GPU call Y: the cached-column z with wide memory-level parallelism (zw1: one-wave kernels, zw2: all) vs the per-entry loop
set -o pipefail
mkdir -p gpurun_out
for lib in libhmpc_zw1.so libhmpc_zw2.so; do
  HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_riccati_stress.py tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_n60.py tests/test_gpu_overflow.py tests/test_gpu_wide.py > gpurun_out/mrl_tests.log 2>&1; rc=$?; echo "$lib tests rc $rc: $(tail -n 1 gpurun_out/mrl_tests.log)"
  [ $rc -eq 0 ] || { grep -B3 -A25 "Error\|assert" gpurun_out/mrl_tests.log | head -40; }
done
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_zw1.so libhmpc_zw2.so; do
    for cfg in "--N 60 --straight --batch 4096" "--N 20 --straight --mu-sweep --global-batch 262144"; do
      HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 200 python -u bench.py $cfg --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', '$cfg'[:7], round(d['value']/1e6,4), 'M/s', round(d['roofline']['kernel_ms'],3), 'ms')"
    done
  done
done
