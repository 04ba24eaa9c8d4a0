# round 5: GPU suite, then the configs[4] breakdown (tools/gpu_r05f.sh)
set -o pipefail
mkdir -p gpurun_out/r05g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05g/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05g/tests.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu_r05f.sh
