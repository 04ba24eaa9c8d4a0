# round-3 GPU call B: DPP root-cause on the round-2 source, new API/dist/planner tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dpp_probe.py libhmpc_old0.so libhmpc_old1.so > gpurun_out/dpp_probe_old.log 2>&1; echo "probe rc $?"; tail -n 30 gpurun_out/dpp_probe_old.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_api.py tests/test_gpu_dist.py tests/test_gpu_planner.py > gpurun_out/r03_b_tests.log 2>&1; echo "tests rc $?"; tail -n 30 gpurun_out/r03_b_tests.log
