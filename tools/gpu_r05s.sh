# round 5: GPU suite with the per-context step graph, then A/B graph on / off
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
L="libhmpc.so libhmpc.so:HMPC_STEP_GRAPH=0"
for t in "c1:--variant 2f --straight --batch 4096 --steps 200 --cpu-seconds 0" "3f4k:--N 10 --batch 4096 --steps 200 --cpu-seconds 0" "3f1k:--N 10 --batch 1024 --steps 300 --cpu-seconds 0" "c4_4k:--N 10 --precision f32 --batch 4096 --steps 200 --cpu-seconds 0"; do
  tag=${t%%:*}; args=${t#*:}
  timeout -k 10 500 python tools/ab.py --tag r05_graph_$tag --rounds 3 --args "$args" $L > $O/ab_$tag.log 2>&1 || { echo "ab $tag failed"; tail -5 $O/ab_$tag.log; exit 1; }
  tail -3 $O/ab_$tag.log
done
