# A/B of the N=10 dense kernel: libhmpc.so (new) vs libhmpc_prev.so (build with OUT=libhmpc_prev.so), parity first
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gpu_f32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
bash tools/ab_n10.sh
