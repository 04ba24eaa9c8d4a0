# round-3 GPU call AC: final dense build (block classify, class priorities, 2f 5N-wide full class) -- full -m gpu suite
# + smoke, configs[2] / configs[1] / fp32 profiles, the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03_ac_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_ac_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r03_ac_tests.log | head -80; exit 1; }
timeout -k 10 120 python -u __graft_entry__.py smoke || exit 1
CFGS="n10 n10_2f n10_f32" bash tools/profile_r03.sh r03 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2>gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print('default', round(d['value']/1e6,3), 'M/s', d['roofline']['kernel'])"
