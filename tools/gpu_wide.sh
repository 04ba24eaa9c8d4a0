set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_wide.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/gpu_wide.log; exit 1; }
tail -12 gpurun_out/gpu_wide.log
