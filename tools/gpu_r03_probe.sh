set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/fp64_peak > gpurun_out/fp64_peak.json 2>&1 && cat gpurun_out/fp64_peak.json &&
timeout -k 10 400 python -u tools/dpp_probe.py libhmpc_v1.so libhmpc_v2.so libhmpc_v3.so > gpurun_out/dpp_probe.log 2>&1; echo "probe rc $?"; cat gpurun_out/dpp_probe.log | tail -n 30
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_riccati_stress.py tests/test_gpu_overflow.py tests/test_gpu_n60.py tests/test_gpu_wide.py > gpurun_out/ric_tests.log 2>&1; echo "tests rc $?"; tail -n 25 gpurun_out/ric_tests.log
