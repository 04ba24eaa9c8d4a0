# A/B of the Riccati kernel: libhmpc.so (new) vs libhmpc_prev.so; parity first
set -o pipefail
mkdir -p gpurun_out/abr
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_n60.py tests/test_gpu_riccati_stress.py tests/test_gpu_overflow.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/abr/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/abr/tests.log; exit 1; }
tail -1 gpurun_out/abr/tests.log
for v in prev new; do
  if [ $v = prev ]; then L=hopper-mpc-inertial_amd/libhmpc_prev.so; else L=hopper-mpc-inertial_amd/libhmpc.so; fi
  HMPC_LIB=$L timeout -k 10 200 python bench.py --N 20 --straight --mu-sweep --global-batch 262144 --steps 5 --cpu-seconds 0 > gpurun_out/abr/n20_$v.json 2> gpurun_out/abr/n20_$v.err || { echo N20 $v FAILED; tail gpurun_out/abr/n20_$v.err; exit 1; }
  HMPC_LIB=$L timeout -k 10 200 python bench.py --N 60 --straight --batch 4096 --steps 10 --cpu-seconds 0 > gpurun_out/abr/n60_$v.json 2> gpurun_out/abr/n60_$v.err || { echo N60 $v FAILED; tail gpurun_out/abr/n60_$v.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/abr/n20_$v.json')); b=json.load(open('gpurun_out/abr/n60_$v.json')); print('$v', 'N20', round(a['value']), a['roofline']['kernel_ms'], a.get('parity_sample'), 'N60', round(b['value']), b['roofline']['kernel_ms'], b.get('parity_sample'))"
done
