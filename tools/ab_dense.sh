# N=10 dense-kernel throughput A/B over libhmpc_<v>.so for the given v's
set -o pipefail
mkdir -p gpurun_out/abd
for v in "$@"; do
  HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_$v.so timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/abd/$v.json 2> gpurun_out/abd/$v.err || { echo $v FAILED; tail gpurun_out/abd/$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abd/$v.json')); print('$v', round(d['value']), round(d['roofline']['kernel_ms'],4))"
done
