#!/bin/bash
# Round-5 proof of the round-2 overflow-kernel miscompile:
# build the round-2 source (beb219c) with its DPP sweep blocks forced into the
# overflow pass, move ONE instruction of its gfx950 assembly -- the AGPR copy
# `v_accvgpr_write_b32 a43, v182` (v182 = lane - 6) from before to after the
# `s_or_b64 exec, exec, s[2:3]` of its join block -- reassemble, rebundle,
# relink.  tools/dpp_name.py then replays the reference's N = 60 run:
#   libhmpc_old1.so       (as compiled)          calls 94-99 wrong x*
#   libhmpc_old1_orig.so  (reassembled, unmoved) calls 94-99 wrong x*
#   libhmpc_old1_mod.so   (the copy moved)       every call right
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=${T:-/tmp/dpp_patch}
LL=/opt/rocm/lib/llvm/bin
rm -rf $T && mkdir -p $T/src && cd $T
git -C $R archive beb219c | tar -x -C $T/src
O=$T/src/hopper-mpc-inertial_amd
sed -i 's/if constexpr (ENT == 1) {/if constexpr (true) {/' $O/csrc/hmpc_ric.hip
(cd $O && HORIZONS=10 F32_HORIZONS="" OUT=libhmpc_old1.so BDIR=build_old1 bash build.sh > /dev/null)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -c $O/csrc/hmpc_ric.hip -o ric.o --save-temps 2> /dev/null
S=hmpc_ric-hip-amdgcn-amd-amdhsa-gfx950.s
python3 - "$S" <<'PY'
import sys
L = open(sys.argv[1]).read().split('\n')
k = next(i for i, l in enumerate(L) if l.strip() == 'v_accvgpr_write_b32 a43, v182')
r = next(i for i in range(k, k + 40) if L[i].strip().startswith('s_or_b64 exec, exec'))
open('orig.s', 'w').write('\n'.join(L))
M = L[:]
ins = M.pop(k)
M.insert(r, ins)            # just after the exec restore
open('mod.s', 'w').write('\n'.join(M))
print(f'moved line {k + 1} after line {r + 1}: {L[r].strip()}')
PY
$LL/llvm-objcopy -O binary --only-section=.hip_fatbin $O/build_old1/hmpc_ric.o fat.bin
$LL/clang-offload-bundler --unbundle --type=o --input=fat.bin --targets=host-x86_64-unknown-linux-gnu- --output=host.part
mkdir -p $R/tools/dpp_old && cp $O/*.py $O/libhmpc_old1.so $R/tools/dpp_old/
for v in orig mod; do
  $LL/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $v.s -o $v.o
  $LL/ld.lld -shared $v.o -o $v.hsaco
  $LL/clang-offload-bundler --type=o --targets=host-x86_64-unknown-linux-gnu-,hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=host.part --input=$v.hsaco --output=fat_$v.bin
  cp $O/build_old1/hmpc_ric.o ric_$v.o
  $LL/llvm-objcopy --update-section .hip_fatbin=fat_$v.bin ric_$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls $O/build_old1/*.o | grep -v hmpc_ric.o) ric_$v.o \
    -o $R/tools/dpp_old/libhmpc_old1_$v.so
done
python3 $R/tools/exec_lint.py orig.s | tail -1
echo "built $R/tools/dpp_old/libhmpc_old1{,_orig,_mod}.so"
