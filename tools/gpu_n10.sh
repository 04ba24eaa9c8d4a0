set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_n10.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_n10.log; exit 1; }
tail -2 gpurun_out/gpu_n10.log
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench_n10.json 2> gpurun_out/bench_n10.err || { echo BENCH FAILED; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_n10.json')); print(d['value'], d['roofline']['kernel_ms'])"
timeout -k 10 300 python bench.py --variant 2f --cpu-seconds 0 > gpurun_out/bench_n10_2f.json 2> gpurun_out/bench_n10_2f.err || { echo BENCH2 FAILED; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_n10_2f.json')); print('2f', d['value'], d['roofline']['kernel_ms'])"
N=10 B=65536 HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 200 python tools/phase_stamps.py > gpurun_out/stamps_n10.json 2> gpurun_out/stamps_n10.err || { echo STAMPS FAILED; exit 1; }
cat gpurun_out/stamps_n10.json
