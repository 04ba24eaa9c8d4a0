# round 5: GPU suite, then the configs[4] lines (fp32, fp32 + refinement k=5) and the default line
set -o pipefail
mkdir -p gpurun_out/r05e
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05e/tests.log 2>&1; rc=$?; tail -4 gpurun_out/r05e/tests.log; stop $rc; [ $rc -eq 0 ] || exit 1
for cfg in "f32r:--precision f32_refined --refine 5" "f32:--precision f32" "f64:"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python bench.py $args --cpu-seconds 4 > gpurun_out/r05e/bench_$tag.json 2> gpurun_out/r05e/bench_$tag.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r05e/bench_$tag.json')); print('$tag', round(d['value']/1e6,3), 'M/s', d['roofline']['kernel_ms'], d['overflow_pass'], d['parity_sample']['max_abs_du_vs_port'], d['parity_sample']['status_mismatch'])"
done
