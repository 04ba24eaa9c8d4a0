# round-3 GPU call C: occupancy experiment (48-variable dense kernel at 2 vs 3 waves/SIMD)
set -o pipefail
mkdir -p gpurun_out
for v in n8w2 n8w3; do
  HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_$v.so timeout -k 10 120 python -u bench.py --N 8 --steps 50 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err || { echo "bench $v failed"; tail -n 5 gpurun_out/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value']/1e6, 'M/s', d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
timeout -k 10 120 python -u bench.py --steps 50 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_n10.json 2>gpurun_out/bench_n10.err && python -c "import json;d=json.load(open('gpurun_out/bench_n10.json'));print('n10', d['value']/1e6, 'M/s', d['roofline']['kernel_ms'])"
