# round 5: GPU suite; A/B of the select form in the 2-wave Riccati kernels too
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
L="libhmpc.so libhmpc_ab_head.so"
for t in "c3:--N 20 --straight --mu-sweep --global-batch 262144 --steps 8 --warmup 2 --cpu-seconds 0" "n20_16k:--N 20 --batch 16384 --steps 30 --cpu-seconds 0" "n60:--N 60 --straight --batch 4096 --steps 30 --cpu-seconds 0"; do
  tag=${t%%:*}; args=${t#*:}
  timeout -k 10 500 python tools/ab.py --tag r05_ricsel2_$tag --rounds 3 --args "$args" $L > $O/ab_$tag.log 2>&1 || { echo "ab $tag failed"; exit 1; }
  tail -3 $O/ab_$tag.log
done
