# round 5: launch-order knobs re-measured after the instruction-count work
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_swing.py tests/test_gpu_order.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit 1
HMPC_LPT_SWING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_order.py -x -q --timeout 120 --timeout-method thread > $O/tests_lsw.log 2>&1; rc=$?; tail -2 $O/tests_lsw.log
for t in "c2:--N 10 --steps 60 --cpu-seconds 0:libhmpc.so libhmpc.so:HMPC_SPLIT_ORDER=1" "c1:--variant 2f --straight --batch 4096 --steps 200 --cpu-seconds 0:libhmpc.so libhmpc.so:HMPC_LPT_SWING=1" "3f4k:--N 10 --batch 4096 --steps 200 --cpu-seconds 0:libhmpc.so libhmpc.so:HMPC_LPT_SWING=1" "3f8k:--N 10 --batch 8192 --steps 200 --cpu-seconds 0:libhmpc.so libhmpc.so:HMPC_LPT_SWING=1"; do
  tag=${t%%:*}; rest=${t#*:}; args=${rest%%:*}; L=${rest#*:}
  timeout -k 10 500 python tools/ab.py --tag r05_knob_$tag --rounds 3 --args "$args" $L > $O/ab_$tag.log 2>&1 || { echo "ab $tag failed"; tail -5 $O/ab_$tag.log; exit 1; }
  tail -3 $O/ab_$tag.log
done
