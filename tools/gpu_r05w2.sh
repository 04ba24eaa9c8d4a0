# round 5: GPU suite with the incremental-mask sweeps, then interleaved A/B
# against the previous commit (configs[2], configs[1], fp32 configs[4])
set -o pipefail
O=gpurun_out/r05w2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
L="libhmpc.so libhmpc_ab_head.so"
for t in "c2:--N 10 --steps 60 --cpu-seconds 0" "c1:--variant 2f --straight --batch 4096 --steps 200 --cpu-seconds 0" "c4:--N 10 --precision f32 --steps 60 --cpu-seconds 0" "b16k:--N 10 --batch 16384 --steps 100 --cpu-seconds 0"; do
  tag=${t%%:*}; args=${t#*:}
  timeout -k 10 400 python tools/ab.py --tag r05_xref_$tag --rounds 3 --args "$args" $L > $O/ab_$tag.log 2>&1 || { echo "ab $tag failed"; exit 1; }
  tail -3 $O/ab_$tag.log
done
