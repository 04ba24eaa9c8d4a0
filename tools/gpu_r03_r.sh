# round-3 GPU call R: the MRHS build (16 slots): full -m gpu suite + smoke,
# Riccati phase stamps with MRHS on / off (N = 20, N = 60), fresh profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03_r_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_r_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r03_r_tests.log | head -80; exit 1; }
timeout -k 10 120 python -u __graft_entry__.py smoke || exit 1
for lib in libhmpc_rstamps.so libhmpc_rstamps0.so; do
  for c in "3f 20 65536 mu" "3f 60 4096"; do
    HMPC_LIB=$PWD/hopper-mpc-inertial_amd/$lib timeout -k 10 300 python -u tools/ric_stamps.py $c > gpurun_out/rst.json 2>gpurun_out/rst.err || { tail -5 gpurun_out/rst.err; exit 1; }
    cp gpurun_out/rst.json "gpurun_out/ricstamps_${lib%.so}_$(echo $c | tr ' ' '_').json"
    python -c "
import json; d=json.load(open('gpurun_out/rst.json')); a=d.get('all', d)
print('$lib', '$c', {k: round(v/1e3,1) for k, v in a.items() if isinstance(v, (int, float)) and k not in ('instances',)})"
  done
done
CFGS="n20 n60" bash tools/profile_r03.sh r03
