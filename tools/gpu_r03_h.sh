# round-3 GPU call H: full suite, feasibility diagnostic (2 reps), stamps, benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_h_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_h_tests.log
[ $rc -eq 0 ] || { grep -B2 -A30 "Error\|assert" gpurun_out/r03_h_tests.log | head -60; exit 1; }
timeout -k 10 300 python -u tools/feas_diag.py 2>&1 | grep "rep"
HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 200 python -u tools/phase_stamps.py > gpurun_out/stamps_n10.json 2>gpurun_out/stamps.err; echo "stamps rc $?"; python -c "
import json; d=json.load(open('gpurun_out/stamps_n10.json'))
for k,v in d.items(): print(k, v['instances'], {n: round(v[n]/1e3,1) for n in ['load','gen_dt_dynamics','uniform_sweeps','hessian_rows','cholesky','unconstrained','active_set','outputs','total_mean']}, 'it', round(v['iters_mean'],2))"
for cfg in "--steps 100 --warmup 20" "--variant 2f --straight --batch 4096 --steps 100 --warmup 20"; do
  timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$cfg'[:14], round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
done
