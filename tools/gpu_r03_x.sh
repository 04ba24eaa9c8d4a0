# round-3 GPU call X: Riccati phase stamps of the final build (N = 20 mu sweep, N = 60)
set -o pipefail
mkdir -p gpurun_out
for c in "3f 20 65536 mu" "3f 60 4096"; do
  HMPC_LIB=$PWD/hopper-mpc-inertial_amd/libhmpc_rstamps.so timeout -k 10 300 python -u tools/ric_stamps.py $c > gpurun_out/rst.json 2>gpurun_out/rst.err || { tail -5 gpurun_out/rst.err; exit 1; }
  cp gpurun_out/rst.json "gpurun_out/ricstamps_final_$(echo $c | tr ' ' '_').json"
  python -c "
import json; a=json.load(open('gpurun_out/rst.json'))
print('$c', {k: round(v/1e3,1) for k, v in a.items() if isinstance(v, (int, float)) and k != 'iters_mean'}, 'it', a['iters_mean'])"
done
