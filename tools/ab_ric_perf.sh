# Riccati throughput A/B over the libs given as arguments (N=20 configs[3], N=60 B=4096)
set -o pipefail
mkdir -p gpurun_out/abp
for v in "$@"; do
  L=hopper-mpc-inertial_amd/libhmpc_$v.so
  HMPC_LIB=$L timeout -k 10 200 python bench.py --N 20 --straight --mu-sweep --global-batch 262144 --steps 5 --cpu-seconds 0 > gpurun_out/abp/n20_$v.json 2> gpurun_out/abp/n20_$v.err || { echo N20 $v FAILED; tail gpurun_out/abp/n20_$v.err; exit 1; }
  HMPC_LIB=$L timeout -k 10 200 python bench.py --N 60 --straight --batch 4096 --steps 10 --cpu-seconds 0 > gpurun_out/abp/n60_$v.json 2> gpurun_out/abp/n60_$v.err || { echo N60 $v FAILED; tail gpurun_out/abp/n60_$v.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/abp/n20_$v.json')); b=json.load(open('gpurun_out/abp/n60_$v.json')); print('$v', 'N20', round(a['value']), round(a['roofline']['kernel_ms'],3), 'N60', round(b['value']), round(b['roofline']['kernel_ms'],3))"
done
