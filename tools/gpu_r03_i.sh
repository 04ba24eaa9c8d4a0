# round-3 GPU call I: full -m gpu suite, the DPP root-cause probe, then
# profile evidence for every config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03_i_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_i_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u __graft_entry__.py smoke || exit 1
timeout -k 10 600 python -u tools/dpp_probe.py libhmpc_v1.so libhmpc_v2.so libhmpc_v3.so > gpurun_out/dpp_probe.log 2>&1; rc=$?; cat gpurun_out/dpp_probe.log; [ $rc -eq 0 ] || exit 1
CFGS="${CFGS:-n10 n10_2f n10_f32 n20 n60}" bash tools/profile_r03.sh r03
