set -o pipefail
mkdir -p gpurun_out/ab
for v in prev new; do
  if [ $v = prev ]; then L=hopper-mpc-inertial_amd/libhmpc_prev; else L=hopper-mpc-inertial_amd/libhmpc; fi
  HMPC_LIB=${L}.so timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err || { echo BENCH $v FAILED; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/bench_$v.json')); print('$v', d['value'], d['roofline']['kernel_ms'])"
  for B in 256 65536; do
    N=10 B=$B HMPC_LIB=${L}_stamps.so timeout -k 10 200 python tools/phase_stamps.py > gpurun_out/ab/stamps_${v}_$B.json 2> gpurun_out/ab/stamps_${v}_$B.err || { echo STAMPS FAILED; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab/stamps_${v}_$B.json')); print('$v', $B, {k: round(x) for k, x in d.items()})"
  done
done
