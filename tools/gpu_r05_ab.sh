# interleaved A/B: swing-first order (abA) vs swing on the split stream (abB)
set -o pipefail
L="libhmpc_abA.so libhmpc_abB.so"
for B in 24576 32768 49152; do
timeout -k 10 300 python tools/ab.py --tag r05_first_$B --rounds 3 --args "--N 10 --batch $B --steps 100" $L > gpurun_out/ab_first_$B.log 2>&1; tail -3 gpurun_out/ab_first_$B.log
done
