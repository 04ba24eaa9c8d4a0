# round-3 GPU call W: the final Riccati build -- full -m gpu suite + smoke,
# configs[3] / N = 60 profiles, Riccati stamps, device Runner timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r03_w_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -n 3 gpurun_out/r03_w_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r03_w_tests.log | head -80; exit 1; }
timeout -k 10 120 python -u __graft_entry__.py smoke || exit 1
CFGS="n20 n60" bash tools/profile_r03.sh r03 || exit 1
timeout -k 10 300 python -u tools/runner_time.py > gpurun_out/runner_eager.json 2>gpurun_out/runner_eager.err || { tail -n 20 gpurun_out/runner_eager.err; exit 1; }
timeout -k 10 300 python -u tools/runner_time.py graph > gpurun_out/runner_graph.json 2>gpurun_out/runner_graph.err || { tail -n 20 gpurun_out/runner_graph.err; exit 1; }
python -c "
import json
e=json.load(open('gpurun_out/runner_eager.json'))['runner_N60_2000_steps']; g=json.load(open('gpurun_out/runner_graph.json'))['runner_N60_2000_steps']
for b in e: print('runner B', b, 'eager', round(e[b]['seconds'],4), 'graph', round(g[b]['seconds'],4))"
