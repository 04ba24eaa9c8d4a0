# round-3 GPU call L: fix candidates on the failing source (4660919 with the
# DPP blocks forced into the overflow pass): bound_ctrl:1, s_nop 4 after each
# block, asm volatile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/dpp_probe.py libhmpc_bis_4660919.so libhmpc_bis_4660919_bc.so libhmpc_bis_4660919_tail.so libhmpc_bis_4660919_vol.so > gpurun_out/dpp_fix.log 2>&1; rc=$?; grep -v "first bad row\|^  " gpurun_out/dpp_fix.log; exit $rc
