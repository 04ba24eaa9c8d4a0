# round-3 GPU call AA: classify with one atomic per 1024-thread block and list
# (libhmpc_cls.so) vs one per wave: parity of the dense path, then A/B + trace
set -o pipefail
mkdir -p gpurun_out
HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_cls.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_overflow.py tests/test_gpu_runner.py > gpurun_out/cls_tests.log 2>&1; rc=$?; echo "cls tests rc $rc: $(tail -n 1 gpurun_out/cls_tests.log)"
[ $rc -eq 0 ] || { grep -B3 -A25 "Error\|assert" gpurun_out/cls_tests.log | head -60; exit 1; }
for rep in 1 2 3; do
  for lib in libhmpc.so libhmpc_cls.so; do
    for cfg in "--steps 100 --warmup 20" "--variant 2f --straight --batch 4096 --steps 100 --warmup 20"; do
      HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', '$cfg'[:14], round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
HMPC_LIB=$GRAFT_REPO_ROOT/hopper-mpc-inertial_amd/libhmpc_cls.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/cls_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/cls_trace.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/cls_trace -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -6
