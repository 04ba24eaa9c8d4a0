set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests_r1.log; exit 1; }
tail -3 gpurun_out/gpu_tests_r1.log
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err || { echo BENCH FAILED; tail gpurun_out/bench_r1.err; exit 1; }
cat gpurun_out/bench_r1.json
