# round-3 GPU call B: DPP root-cause on the round-2 source, new API/dist/planner tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dpp_probe.py libhmpc_old0.so libhmpc_old1.so > gpurun_out/dpp_probe_old.log 2>&1; echo "probe rc $?"; tail -n 30 gpurun_out/dpp_probe_old.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_api.py tests/test_gpu_dist.py tests/test_gpu_planner.py > gpurun_out/r03_b_tests.log 2>&1; echo "tests rc $?"; tail -n 30 gpurun_out/r03_b_tests.log
# round-3 GPU call C: occupancy experiment (48-variable dense kernel at 2 vs 3 waves/SIMD)
set -o pipefail
mkdir -p gpurun_out
for v in n8w2 n8w3; do
  HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_$v.so timeout -k 10 120 python -u bench.py --N 8 --steps 50 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err || { echo "bench $v failed"; tail -n 5 gpurun_out/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value']/1e6, 'M/s', d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
timeout -k 10 120 python -u bench.py --steps 50 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_n10.json 2>gpurun_out/bench_n10.err && python -c "import json;d=json.load(open('gpurun_out/bench_n10.json'));print('n10', d['value']/1e6, 'M/s', d['roofline']['kernel_ms'])"
