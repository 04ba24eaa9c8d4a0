#!/bin/bash
# Round-4 call F: the full GPU suite on the runtime instance order
# (hmpc_set_order), then the batch-size thresholds of the automatic
# longest-first choice: index vs longest-first order per batch size.
set -o pipefail
mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/r04f_tests.log)"; stop $rc
[ $rc -eq 0 ] || exit 1
AB="timeout -k 10 900 python tools/ab.py --rounds 2 --vary=--order=index --vary=--order=longest_first"
$AB --tag r04f_d4k --args "--variant 2f --straight --batch 4096" || exit 1
$AB --tag r04f_d8k --args "--batch 8192" || exit 1
$AB --tag r04f_d8k2f --args "--variant 2f --straight --batch 8192" || exit 1
$AB --tag r04f_d16k --args "--batch 16384" || exit 1
$AB --tag r04f_n60_4k --args "--N 60 --straight --batch 4096" || exit 1
$AB --tag r04f_n60_8k --args "--N 60 --straight --batch 8192" || exit 1
$AB --tag r04f_n60_16k --args "--N 60 --straight --batch 16384" || exit 1
$AB --tag r04f_n20_16k --args "--N 20 --straight --mu-sweep --batch 16384" || exit 1
$AB --tag r04f_n20_32k --args "--N 20 --straight --mu-sweep --batch 32768" || exit 1
