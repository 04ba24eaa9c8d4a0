# round 5: GPU suite; the Riccati bucket pass beside the factorisation kernel
# and skipped at B <= resident workgroups, A/B against the previous commit
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
L="libhmpc.so libhmpc_ab_head.so"
timeout -k 10 400 python tools/ab.py --tag r05_bk_n60 --rounds 3 --args "--N 60 --straight --batch 4096 --steps 30 --cpu-seconds 0" $L > $O/ab_n60.log 2>&1 || { echo "ab n60 failed"; exit 1; }
tail -3 $O/ab_n60.log
timeout -k 10 400 python tools/ab.py --tag r05_bk_n60_1k --rounds 3 --args "--N 60 --straight --batch 1024 --steps 30 --cpu-seconds 0" $L > $O/ab_n60_1k.log 2>&1 || { echo "ab n60 1k failed"; exit 1; }
tail -3 $O/ab_n60_1k.log
