# round 5: GPU suite; A/B of mov_dpp permutes (no materialised old value)
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
L="libhmpc.so libhmpc_ab_head.so"
for t in "c2:--N 10 --steps 60 --cpu-seconds 0" "c1:--variant 2f --straight --batch 4096 --steps 200 --cpu-seconds 0" "c4:--N 10 --precision f32 --steps 60 --cpu-seconds 0" "c3:--N 20 --straight --mu-sweep --global-batch 262144 --steps 8 --warmup 2 --cpu-seconds 0" "n60:--N 60 --straight --batch 4096 --steps 30 --cpu-seconds 0"; do
  tag=${t%%:*}; args=${t#*:}
  timeout -k 10 500 python tools/ab.py --tag r05_movdpp_$tag --rounds 3 --args "$args" $L > $O/ab_$tag.log 2>&1 || { echo "ab $tag failed"; exit 1; }
  tail -3 $O/ab_$tag.log
done
