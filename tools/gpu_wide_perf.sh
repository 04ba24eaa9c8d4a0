set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_runner.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gw.log 2>&1 || { echo TESTS FAILED; tail -20 gpurun_out/gw.log; exit 1; }
tail -1 gpurun_out/gw.log
HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so N=60 B=1 timeout -k 10 200 python tools/wide_stamps.py 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print({k: round(v) for k, v in d.items()})"
timeout -k 10 300 python bench.py --N 60 --batch 4096 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_n60.json 2>/dev/null || { echo BENCH FAILED; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_n60.json')); print('N60', round(d['value']), d['roofline']['kernel_ms'])"
timeout -k 10 300 python tools/runner_n60.py
