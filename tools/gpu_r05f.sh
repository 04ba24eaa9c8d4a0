# round 5: configs[4] breakdown -- phase stamps of the fp64, fp32 and fp32 +
# refinement builds (B = 65536 configs[2]/[4] instances), and the refined
# line at k = 1..6 corrections
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r05f
mkdir -p $O
(cd /tmp && TMPDIR=/tmp timeout -k 10 120 rocprofv3 -L > $R/$O/counters.txt 2>&1) || echo "counter list failed"
L=hopper-mpc-inertial_amd/libhmpc_stamps.so
for p in "f64:5" "f32:5" "f32_refined:5" "f32_refined:2"; do
  prec=${p%%:*}; k=${p#*:}
  HMPC_LIB=$L PREC=$prec REFINE=$k timeout -k 10 180 python tools/phase_stamps.py > $O/stamps_${prec}_k$k.json 2> $O/stamps_${prec}_k$k.err || { echo "stamps $p failed"; exit 1; }
  echo "stamps $p ok"
done
for k in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --precision f32_refined --refine $k --cpu-seconds 0 > $O/bench_k$k.json 2> $O/bench_k$k.err || { echo "bench k=$k failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_k$k.json')); print('k=$k', round(d['value']/1e6,3), 'M/s', round(d['roofline']['kernel_ms'],4), d['overflow_pass'], d['parity_sample']['max_abs_du_vs_port'])"
done
# the early exit of the corrections (libhmpc.so) against always k (libhmpc_noee.so)
timeout -k 10 400 python tools/ab.py --tag r05_refine_exit --rounds 2 --args "--precision f32_refined --refine 5 --cpu-seconds 0" libhmpc.so libhmpc_noee.so > $O/ab_exit.log 2>&1 || { echo "ab failed"; exit 1; }
tail -3 $O/ab_exit.log
