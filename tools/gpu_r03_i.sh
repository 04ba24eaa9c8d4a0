# round-3 GPU call I: full -m gpu suite, the DPP root-cause probe, the dense
# split A/B (concurrent / serial / off), then profile evidence for every config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03_i_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_i_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r03_i_tests.log | head -80; exit 1; }
timeout -k 10 120 python -u __graft_entry__.py smoke || exit 1
timeout -k 10 600 python -u tools/dpp_probe.py libhmpc_v1.so libhmpc_v2.so libhmpc_v3.so > gpurun_out/dpp_probe.log 2>&1; rc=$?; cat gpurun_out/dpp_probe.log; [ $rc -eq 0 ] || exit 1
for mode in "" "HMPC_SPLIT_SERIAL=1" "HMPC_SPLIT=0"; do
  for cfg in "--steps 100 --warmup 20" "--variant 2f --straight --batch 4096 --steps 100 --warmup 20"; do
    env $mode timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b.json'));print('split[$mode]', '$cfg'[:14], round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
  done
done
CFGS="${CFGS:-n10 n10_2f n10_f32 n20 n60}" bash tools/profile_r03.sh r03
