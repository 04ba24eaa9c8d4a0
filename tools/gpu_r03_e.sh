# round-3 GPU call E: split (concurrent classes) vs no split; per-kernel times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gpu_api.py > gpurun_out/r03_e_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_e_tests.log; [ $rc -eq 0 ] || exit 1
for lib in libhmpc.so libhmpc_noskip.so libhmpc_nosplit.so; do
  for cfg in "--steps 50 --warmup 20" "--variant 2f --straight --batch 4096 --steps 50 --warmup 20"; do
    HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', '$cfg'[:14], round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e -o run -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/prof_e.log 2>&1; echo "prof rc $?"
find gpurun_out/prof_e -name "*kernel_stats.csv" | head -1 | xargs -I{} cat {} | cut -d, -f1-8 | head -12
