#!/bin/bash
# Build a one-horizon libhmpc variant from an alternative kernel source (A/B
# experiments):  tools/build_variant.sh <kernel.hip> <out.so> <N> [extra flags]
set -euo pipefail
SRC=$1; OUT=$2; N=$3; shift 3
P=$(cd "$(dirname "$0")/../hopper-mpc-inertial_amd" && pwd)
B=$(mktemp -d)
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -I$P/csrc"
H=/opt/rocm/bin/hipcc
$H $F -DHMPC_INST_N=$N -c $SRC -o $B/k.o "$@" &
$H $F "-DHMPC_HORIZON_LIST(X)=X($N)" -c $P/csrc/hmpc_dispatch.cpp -o $B/d.o &
$H $F -c $P/csrc/hmpc_capi.cpp -o $B/c.o &
$H $F -c $P/csrc/hmpc_plant.hip -o $B/p.o &
$H $F -c $P/csrc/hmpc_wide.hip -o $B/w.o &
wait
$H --offload-arch=gfx950 -shared -fPIC $B/k.o $B/d.o $B/c.o $B/p.o $B/w.o -o $OUT
rm -rf $B
echo "built $OUT"
