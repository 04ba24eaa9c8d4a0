# interleaved A/B: with / without the all-swing class at small batches
set -o pipefail
L="libhmpc_sw.so libhmpc_nosw.so"
timeout -k 10 300 python tools/ab.py --tag r05_sw_c1 --rounds 3 --args "--variant 2f --straight --batch 4096 --steps 200" $L > gpurun_out/ab_sw_c1.log 2>&1; tail -3 gpurun_out/ab_sw_c1.log
timeout -k 10 300 python tools/ab.py --tag r05_sw_3f4k --rounds 2 --args "--N 10 --batch 4096 --steps 200" $L > gpurun_out/ab_sw_3f4k.log 2>&1; tail -3 gpurun_out/ab_sw_3f4k.log
timeout -k 10 300 python tools/ab.py --tag r05_sw_8k --rounds 2 --args "--N 10 --batch 8192 --steps 200" $L > gpurun_out/ab_sw_8k.log 2>&1; tail -3 gpurun_out/ab_sw_8k.log
timeout -k 10 300 python tools/ab.py --tag r05_sw_16k --rounds 2 --args "--N 10 --batch 16384 --steps 100" $L > gpurun_out/ab_sw_16k.log 2>&1; tail -3 gpurun_out/ab_sw_16k.log
