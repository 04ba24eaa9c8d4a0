set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_quick.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_quick.log; exit 1; }
tail -1 gpurun_out/gpu_quick.log
for n in 10 20; do
  N=$n B=65536 HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 200 python tools/phase_stamps.py > gpurun_out/stamps_q$n.json 2>/dev/null || { echo STAMPS FAILED; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/stamps_q$n.json')); print($n, {k: round(v) for k, v in d.items()})"
done
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench_q.json 2>/dev/null || { echo BENCH FAILED; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print('N10', round(d['value']), d['roofline']['kernel_ms'])"
timeout -k 10 300 python bench.py --N 20 --batch 262144 --mu-sweep --steps 5 --cpu-seconds 0 > gpurun_out/bench_q20.json 2>/dev/null || { echo BENCH20 FAILED; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_q20.json')); print('N20', round(d['value']), d['roofline']['kernel_ms'])"
