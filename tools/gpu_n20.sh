set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_t3.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_t3.log; exit 1; }
tail -2 gpurun_out/gpu_t3.log
N=20 B=65536 HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 200 python tools/phase_stamps.py > gpurun_out/stamps_n20b.json 2> gpurun_out/stamps_n20b.err || { echo STAMPS FAILED; exit 1; }
cat gpurun_out/stamps_n20b.json
timeout -k 10 300 python bench.py --N 20 --batch 262144 --mu-sweep --steps 5 --cpu-seconds 0 > gpurun_out/bench_n20.json 2> gpurun_out/bench_n20.err || { echo BENCH FAILED; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_n20.json')); print(d['value'], d['roofline']['kernel_ms'])"
