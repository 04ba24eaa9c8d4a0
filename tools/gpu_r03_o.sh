# round-3 GPU call O: Riccati sweep prefetch depth at 1 wave/SIMD (N = 60):
# ring 3 (default) vs 4 / 5 / 6 slots, then the N = 60 parity tests per depth
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_ring4.so libhmpc_ring5.so libhmpc_ring6.so; do
    HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 200 python -u bench.py --N 60 --straight --batch 4096 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', round(d['value']/1e3,1), 'k/s', round(d['roofline']['kernel_ms'],3), 'ms')"
  done
done
for lib in libhmpc_ring4.so libhmpc_ring5.so libhmpc_ring6.so; do
  HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_n60.py tests/test_gpu_riccati_stress.py tests/test_gpu_wide.py > gpurun_out/ring_tests.log 2>&1; rc=$?; echo "$lib tests rc $rc: $(tail -n 1 gpurun_out/ring_tests.log)"; [ $rc -eq 0 ] || exit 1
done
