# round-3 GPU call AD: issue priority between the dense split's classes
# (p1: compacted chain phases at 2, full at 3; p2: p1 + full base 1;
# p3: compacted chain 1, full base 2 / chain 3) vs the default (both chain 3)
set -o pipefail
mkdir -p gpurun_out
L=hopper-mpc-inertial_amd
for rep in 1 2; do
  for lib in libhmpc.so libhmpc_p1.so libhmpc_p2.so libhmpc_p3.so; do
    for cfg in "--steps 100 --warmup 20" "--variant 2f --straight --batch 4096 --steps 100 --warmup 20" "--batch 16384 --steps 100 --warmup 20"; do
      HMPC_LIB=$PWD/$L/$lib timeout -k 10 120 python -u bench.py $cfg --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib', '$cfg'[:18], round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
    done
  done
done
