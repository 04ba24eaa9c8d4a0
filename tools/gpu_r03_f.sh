# round-3 GPU call F: DPP probe on the round-2 source; per-class phase stamps; bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dpp_probe.py libhmpc_old0.so libhmpc_old1.so > gpurun_out/dpp_probe_old.log 2>&1; echo "probe rc $?"; tail -n 20 gpurun_out/dpp_probe_old.log
HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 200 python -u tools/phase_stamps.py > gpurun_out/stamps_n10.json 2>gpurun_out/stamps.err; echo "stamps rc $?"; python -c "
import json; d=json.load(open('gpurun_out/stamps_n10.json'))
for k,v in d.items(): print(k, v['instances'], {n: round(v[n]/1e3,1) for n in ['load','gen_dt_dynamics','uniform_sweeps','hessian_rows','cholesky','unconstrained','active_set','outputs','total_mean']}, 'it', round(v['iters_mean'],2))"
timeout -k 10 120 python -u bench.py --steps 100 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_n10.json 2>gpurun_out/bench_n10.err && python -c "import json;d=json.load(open('gpurun_out/bench_n10.json'));print('n10', d['value']/1e6, 'M/s', d['roofline']['kernel_ms'])"
