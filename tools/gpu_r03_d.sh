# round-3 GPU call D: full GPU suite on the compacted/split dense kernel, then benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_d_tests.log 2>&1; rc=$?; echo "tests rc $rc"; grep -E "passed|failed|PASS|FAIL|Error" gpurun_out/r03_d_tests.log | tail -n 15
if [ $rc -ne 0 ]; then grep -B5 -A40 "Error\|assert" gpurun_out/r03_d_tests.log | head -n 120; exit 1; fi
timeout -k 10 120 python -u bench.py --steps 50 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_n10.json 2>gpurun_out/bench_n10.err && python -c "import json;d=json.load(open('gpurun_out/bench_n10.json'));print('n10 split', d['value']/1e6, 'M/s', d['roofline']['kernel_ms'])"
timeout -k 10 120 python -u bench.py --variant 2f --straight --batch 4096 --steps 50 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_2f.json 2>gpurun_out/bench_2f.err && python -c "import json;d=json.load(open('gpurun_out/bench_2f.json'));print('2f split', d['value']/1e6, 'M/s', d['roofline']['kernel_ms'])"
bash tools/gpu_r03_c.sh
