# round-3 GPU call Q: MRHS on by default -- full -m gpu suite, smoke, then
# configs[3] A/B: compile-time N = 20 vs runtime N under MRHS, and a 16-slot
# candidate cache
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03_q_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_q_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r03_q_tests.log | head -80; exit 1; }
timeout -k 10 120 python -u __graft_entry__.py smoke || exit 1
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_mrrt.so libhmpc_mr16.so; do
    for cfg in "--N 60 --straight --batch 4096" "--N 20 --straight --mu-sweep --global-batch 262144"; do
      HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 200 python -u bench.py $cfg --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', '$cfg'[:7], round(d['value']/1e6,4), 'M/s', round(d['roofline']['kernel_ms'],3), 'ms', d['roofline']['kernel'])"
    done
  done
done
