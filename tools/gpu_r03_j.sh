# round-3 GPU call J: device Runner eager vs HIP-graph replay (configs[0],
# N = 60), and the fp32 + refinement lower bound (HMPC_REFINE_LB libraries)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/runner_time.py > gpurun_out/runner_eager.json 2>gpurun_out/runner_eager.err || { tail -n 20 gpurun_out/runner_eager.err; exit 1; }
cat gpurun_out/runner_eager.json
timeout -k 10 300 python -u tools/runner_time.py graph > gpurun_out/runner_graph.json 2>gpurun_out/runner_graph.err || { tail -n 20 gpurun_out/runner_graph.err; exit 1; }
cat gpurun_out/runner_graph.json
for lib in libhmpc.so libhmpc_lb2.so libhmpc_lb3.so; do
  HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 120 python -u bench.py --precision f32 --steps 100 --warmup 20 --cpu-seconds 0 > gpurun_out/b.json 2>gpurun_out/b.err || { tail -n 5 gpurun_out/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$lib f32', round(d['value']/1e6,2), 'M/s', round(d['roofline']['kernel_ms'],4), 'ms')"
done
# the DPP probe on the round-2 source (beb219c: old0 as committed, old1 with
# the sweep blocks in the overflow pass too -- the round-2 failure)
timeout -k 10 600 python -u tools/dpp_probe.py libhmpc_old0.so libhmpc_old1.so > gpurun_out/dpp_probe_old.log 2>&1; rc=$?; cat gpurun_out/dpp_probe_old.log; [ $rc -eq 0 ] || exit 1
# launch timelines (stamped build): configs[1] (2f, straight, B = 4096) and configs[2]
for c in "VARIANT=2f STRAIGHT=1 B=4096" "VARIANT=3f STRAIGHT=0 B=65536"; do
  env $c HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 200 python -u tools/phase_stamps.py > gpurun_out/stamps.json 2>gpurun_out/stamps.err || { tail -n 5 gpurun_out/stamps.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/stamps.json')); print('$c', json.dumps(d['timeline']))
for k in ('compacted', 'full'): v=d[k]; print('  ', k, v['instances'], round(v['total_mean']), round(v['total_max']), 'it', round(v['iters_mean'],2))"
  cp gpurun_out/stamps.json "gpurun_out/stamps_$(echo $c | tr ' =' '__').json"
done
