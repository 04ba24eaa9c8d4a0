#!/bin/bash
# Build libhmpc.so in-tree for gfx950 (MI355X).
#   ./build.sh                 all horizons in HORIZONS (default "5 10 20")
#   HORIZONS="10" ./build.sh   a subset (the dispatch table follows)
# One object per horizon, compiled in parallel.
set -euo pipefail
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
HORIZONS=${HORIZONS:-"5 10 20"}
F32_HORIZONS=${F32_HORIZONS:-"10"}   # fp32 builds of the dense kernel (BASELINE configs[4])
F32_WAVES=${F32_WAVES:-3}           # their waves / SIMD (3: <= 168 VGPRs, no spill)
JOBS=${JOBS:-8}
OUT=${OUT:-libhmpc.so}
BDIR=${BDIR:-build}
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result"
mkdir -p $BDIR
LIST=""
for n in $HORIZONS; do LIST="$LIST X($n)"; done
F32LIST=""
for n in $F32_HORIZONS; do F32LIST="$F32LIST X($n)"; done
pids=()
# the split launch's compacted kernel (at most NV free variables, active-set
# capacity Q, 3 waves / SIMD) per horizon: "N:NV:Q" (CMP="" disables)
CMP=${CMP-"10:48:13"}
# the same for the fp32 builds (4 waves / SIMD; F32_CMP="" disables)
F32_CMP=${F32_CMP-"10:48:13"}
cmp_flags() {   # horizon [list]
  for e in ${2-$CMP}; do
    IFS=: read -r cn cv cq <<< "$e"
    if [ "$cn" = "$1" ]; then echo "-DHMPC_CMP_NV=$cv -DHMPC_CMP_Q=$cq"; fi
  done
}
# the split's all-swing class (csrc/hmpc_swing.hip: two instances per wave)
# per horizon: "N:Q:W" = active-set capacity Q, W waves / SIMD (SWING="" disables)
SWING=${SWING-"10:13:3"}
swing_flags() {   # horizon
  for e in $SWING; do
    IFS=: read -r sn sq sw <<< "$e"
    if [ "$sn" = "$1" ]; then echo "-DHMPC_SWING_Q=$sq -DHMPC_SWING_WAVES=$sw"; fi
  done
}
CMPOBJS=""
for n in $HORIZONS; do
  SWF=""
  if [ -n "$(swing_flags $n)" ] && [ -n "$(cmp_flags $n)" ]; then
    SWF="-DHMPC_SWING=1"
    $HIPCC $FLAGS -DHMPC_INST_N=$n $(swing_flags $n) -c csrc/hmpc_swing.hip -o $BDIR/hmpc_swing_n$n.o "$@" &
    pids+=($!)
    CMPOBJS="$CMPOBJS $BDIR/hmpc_swing_n$n.o"
  fi
  $HIPCC $FLAGS -DHMPC_INST_N=$n $(cmp_flags $n) $SWF -c ${KSRC:-csrc/hmpc_kernels.hip} -o $BDIR/hmpc_kernels_n$n.o "$@" &
  pids+=($!)
  if [ -n "$(cmp_flags $n)" ]; then   # the compacted kernel: a translation unit of its own
    $HIPCC $FLAGS -DHMPC_INST_N=$n $(cmp_flags $n) -DHMPC_CMP_ONLY -c ${KSRC:-csrc/hmpc_kernels.hip} -o $BDIR/hmpc_kernels_n${n}_cmp.o "$@" &
    pids+=($!)
    CMPOBJS="$CMPOBJS $BDIR/hmpc_kernels_n${n}_cmp.o"
  fi
  while [ "$(jobs -rp | wc -l)" -ge "$JOBS" ]; do sleep 1; done
done
# the fp32 builds' all-swing class (F32_SWING=0 disables): the fp64 swing
# kernel (two instances per wave, the torque-only QP), so fp32 and fp64 run
# the same three classes
F32_SWING=${F32_SWING-1}
for n in $F32_HORIZONS; do
  # fp32: 3 waves / SIMD fit (<= 168 VGPRs, 9.9 KB LDS) without spilling;
  # split like fp64, the compacted class at 4 waves / SIMD
  F32C=$(cmp_flags $n "$F32_CMP")
  F32SW=""
  if [ "$F32_SWING" = 1 ] && [ -n "$(swing_flags $n)" ] && [ -n "$F32C" ]; then F32SW="-DHMPC_SWING=1 $(swing_flags $n)"; fi
  $HIPCC $FLAGS -DHMPC_INST_N=$n -DHMPC_REAL=float -DHMPC_LAUNCH_SUFFIX=_f32 "-DHMPC_WAVES_PER_EU(W)=$F32_WAVES" \
    $F32C $F32SW -c ${KSRC:-csrc/hmpc_kernels.hip} -o $BDIR/hmpc_kernels_n${n}_f32.o "$@" &
  pids+=($!)
  if [ -n "$F32C" ]; then
    $HIPCC $FLAGS -DHMPC_INST_N=$n -DHMPC_REAL=float -DHMPC_LAUNCH_SUFFIX=_f32 "-DHMPC_WAVES_PER_EU(W)=$F32_WAVES" \
      $F32C -DHMPC_CMP_ONLY -c ${KSRC:-csrc/hmpc_kernels.hip} -o $BDIR/hmpc_kernels_n${n}_f32_cmp.o "$@" &
    pids+=($!)
    CMPOBJS="$CMPOBJS $BDIR/hmpc_kernels_n${n}_f32_cmp.o"
  fi
  # fp32 + fp64 refinement (HMPC_PREC_F32_REFINED), split like the others:
  # every class at 2 waves / SIMD (no scratch spill)
  $HIPCC $FLAGS -DHMPC_INST_N=$n -DHMPC_REAL=float -DHMPC_F32_REFINE=1 -DHMPC_LAUNCH_SUFFIX=_f32r \
    "-DHMPC_WAVES_PER_EU(W)=2" $F32C $F32SW -c csrc/hmpc_kernels.hip -o $BDIR/hmpc_kernels_n${n}_f32r.o "$@" &
  pids+=($!)
  if [ -n "$F32C" ]; then
    $HIPCC $FLAGS -DHMPC_INST_N=$n -DHMPC_REAL=float -DHMPC_F32_REFINE=1 -DHMPC_LAUNCH_SUFFIX=_f32r \
      "-DHMPC_WAVES_PER_EU(W)=2" $F32C -DHMPC_CMP_ONLY -c csrc/hmpc_kernels.hip -o $BDIR/hmpc_kernels_n${n}_f32r_cmp.o "$@" &
    pids+=($!)
    CMPOBJS="$CMPOBJS $BDIR/hmpc_kernels_n${n}_f32r_cmp.o"
  fi
done
$HIPCC $FLAGS "-DHMPC_HORIZON_LIST(X)=$LIST" "-DHMPC_F32_LIST(X)=$F32LIST" "-DHMPC_F32R_LIST(X)=$F32LIST" -c csrc/hmpc_dispatch.cpp -o $BDIR/hmpc_dispatch.o &
pids+=($!)
$HIPCC $FLAGS -c csrc/hmpc_capi.cpp -o $BDIR/hmpc_capi.o &
pids+=($!)
$HIPCC $FLAGS -c csrc/hmpc_plant.hip -o $BDIR/hmpc_plant.o &
pids+=($!)
$HIPCC $FLAGS -c csrc/hmpc_planner.hip -o $BDIR/hmpc_planner.o &
pids+=($!)
$HIPCC $FLAGS -c csrc/hmpc_cas.hip -o $BDIR/hmpc_cas.o "$@" &
pids+=($!)
$HIPCC $FLAGS -c csrc/hmpc_wide.hip -o $BDIR/hmpc_wide.o "$@" &
pids+=($!)
$HIPCC $FLAGS -c ${RIC_SRC:-csrc/hmpc_ric.hip} -o $BDIR/hmpc_ric.o "$@" &
pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
objs=""
for n in $HORIZONS; do objs="$objs $BDIR/hmpc_kernels_n$n.o"; done
objs="$objs $CMPOBJS"
for n in $F32_HORIZONS; do objs="$objs $BDIR/hmpc_kernels_n${n}_f32.o $BDIR/hmpc_kernels_n${n}_f32r.o"; done
# every object but the ABI/dispatch host code, for tests/test_sanitizers.py (which
# rebuilds those two under ASan/UBSan and links the kernels as built)
echo $objs $BDIR/hmpc_plant.o $BDIR/hmpc_planner.o $BDIR/hmpc_cas.o $BDIR/hmpc_wide.o $BDIR/hmpc_ric.o | tr ' ' '\n' > $BDIR/objs.txt
$HIPCC --offload-arch=gfx950 -shared -fPIC $objs $BDIR/hmpc_dispatch.o $BDIR/hmpc_capi.o $BDIR/hmpc_plant.o $BDIR/hmpc_planner.o $BDIR/hmpc_cas.o $BDIR/hmpc_wide.o $BDIR/hmpc_ric.o -o $OUT.tmp
mv $OUT.tmp $OUT
echo "built $(pwd)/$OUT (horizons: $HORIZONS)"
