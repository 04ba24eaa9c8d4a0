# round-3 GPU call Z: final build -- full -m gpu suite + smoke, N = 60 / configs[3]
# profiles, the default bench line; then the dense kernel's issue-priority A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03_z_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_z_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r03_z_tests.log | head -80; exit 1; }
timeout -k 10 120 python -u __graft_entry__.py smoke || exit 1
CFGS="n60 n20" bash tools/profile_r03.sh r03 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2>gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print('default', round(d['value']/1e6,3), 'M/s', d['roofline']['kernel'])"
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_prio0.so libhmpc_prio2.so; do
    for cfg in "--steps 100 --warmup 20" "--variant 2f --straight --batch 4096 --steps 100 --warmup 20"; do
      HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', '$cfg'[:14], round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
    done
  done
done
