#!/bin/bash
# Builds the DPP root-cause variants for tools/dpp_probe.py:
#   v1  the v_fmac_f64_dpp blocks in the overflow pass too (round-2 failure)
#   v2  v1 + s_nop 4 after every block
#   v3  v1 + bound_ctrl:1 on every DPP instruction
set -euo pipefail
cd "$(dirname "$0")/../hopper-mpc-inertial_amd"
export HORIZONS="10" F32_HORIZONS="" CMP=""
OUT=libhmpc_v1.so BDIR=build_v1 bash build.sh -DHMPC_OVF_DPP=1 > /dev/null 2>&1 &
OUT=libhmpc_v2.so BDIR=build_v2 bash build.sh -DHMPC_OVF_DPP=1 '-DHMPC_DPP_TAIL="s_nop 4\n\t"' > /dev/null 2>&1 &
OUT=libhmpc_v3.so BDIR=build_v3 bash build.sh -DHMPC_OVF_DPP=1 '-DHMPC_DPP_BC=" bound_ctrl:1"' > /dev/null 2>&1 &
wait
ls -la libhmpc_v*.so
