# round-3 GPU call K: which change after beb219c made the overflow-pass DPP
# sweeps give the right x* (libraries built by /tmp-side bisect builds: each
# intermediate commit with the DPP blocks forced into the overflow pass)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/dpp_probe.py libhmpc_bis_535c4c3.so libhmpc_bis_6d55104.so libhmpc_bis_4660919.so libhmpc_bis_2349a8b.so libhmpc_bis_06b728c.so libhmpc_bis_1318c95.so libhmpc_bis_ab8f7f3.so libhmpc_bis_91b3923.so libhmpc_bis_a54208d.so > gpurun_out/dpp_bisect.log 2>&1; rc=$?; grep -v "first bad row\|^  " gpurun_out/dpp_bisect.log; exit $rc
