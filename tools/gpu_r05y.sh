# round 5: GPU suite; A/B of the select-form scan / substitutions in the
# Riccati kernels (N = 60 one-wave; N = 20 two-wave for its allocation change)
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
L="libhmpc.so libhmpc_ab_head.so"
for t in "n60:--N 60 --straight --batch 4096 --steps 30 --cpu-seconds 0" "n60_16k:--N 60 --straight --batch 16384 --steps 10 --cpu-seconds 0" "c3:--N 20 --straight --mu-sweep --global-batch 262144 --steps 8 --warmup 2 --cpu-seconds 0"; do
  tag=${t%%:*}; args=${t#*:}
  timeout -k 10 500 python tools/ab.py --tag r05_ricshift_$tag --rounds 3 --args "$args" $L > $O/ab_$tag.log 2>&1 || { echo "ab $tag failed"; exit 1; }
  tail -3 $O/ab_$tag.log
done
timeout -k 10 300 python tools/runner_time.py graph > $O/runner_graph.json 2> $O/rg.err || { echo "runner failed"; exit 1; }
python -c "
import json; t=open('$O/runner_graph.json').read(); d=json.loads(t[t.index('{'):]); print({k: round(v['seconds'],4) for k,v in d['runner_N60_2000_steps'].items()})"
