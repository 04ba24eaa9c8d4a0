"""Register, scratch and LDS budgets of the product kernels, read from the
gfx950 code objects inside the built libhmpc.so (no GPU needed).

The hot kernels' speed rests on these budgets: the
split's compacted class must fit 3 waves/SIMD (<= 168 VGPRs), no dense
kernel may spill, and the Riccati kernels keep their measured scratch.  A
change that moves the register allocation (round 4 saw a force-inlined body
add 36 B/lane of spill to the fp32 build) fails here, before any GPU run."""
import os
import struct
import subprocess
import tempfile

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'hopper-mpc-inertial_amd', 'libhmpc.so')
READELF = '/opt/rocm/lib/llvm/bin/llvm-readelf'
MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'


def _section(data, want):
    """(offset, size) of ELF64 section `want`."""
    shoff = struct.unpack_from('<Q', data, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', data, 0x3A)
    secs = [struct.unpack_from('<IIQQQQ', data, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]
    for name, _t, _f, _a, off, size in secs:
        end = data.index(b'\0', stroff + name)
        if data[stroff + name:end].decode() == want:
            return off, size
    raise KeyError(want)


def _code_objects(path):
    data = open(path, 'rb').read()
    off, size = _section(data, '.hip_fatbin')
    sec = data[off:off + size]
    pos, out = 0, []
    while True:
        i = sec.find(MAGIC, pos)
        if i < 0:
            return out
        n = struct.unpack_from('<Q', sec, i + 24)[0]
        p = i + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from('<QQQ', sec, p)
            p += 24
            triple = sec[p:p + tl]
            p += tl
            if b'gfx950' in triple:
                out.append(sec[i + eo:i + eo + es])
        pos = i + len(MAGIC)


@pytest.fixture(scope='module')
def kernels():
    if not os.path.exists(LIB):
        pytest.skip('libhmpc.so not built (python -c "import __graft_entry__ as g; g.build()")')
    if not os.path.exists(READELF):
        pytest.skip('llvm-readelf not found')
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for k, co in enumerate(_code_objects(LIB)):
            f = os.path.join(d, f'co{k}.o')
            open(f, 'wb').write(co)
            txt = subprocess.run([READELF, '--notes', f], capture_output=True, text=True, check=True).stdout
            body = txt[txt.index('---'):txt.rindex('...')]
            for kern in yaml.safe_load(body)['amdhsa.kernels']:
                res.setdefault(kern['.name'], []).append(kern)
    assert res, 'no gfx950 kernels found in libhmpc.so'
    return res


def solve(v, n, t, nvm, q):
    return f'_ZN4hmpc12_GLOBAL__N_112solve_kernelILi{v}ELi{n}E{t}Li{nvm}ELi{q}EEEvNS_9SolveArgsE'


def ric(v, occ, n, cap, part=0):
    return f'_ZN4hmpc12_GLOBAL__N_110ric_kernelILi{v}ELi{occ}ELi{n}ELi{cap}ELi{part}EEEvNS_9SolveArgsEii'


def ric_factor(v, n, cap):
    return f'_ZN4hmpc12_GLOBAL__N_117ric_factor_kernelILi{v}ELi{n}ELi{cap}EEEvNS_9SolveArgsEii'


@pytest.mark.parametrize('v', [3, 2])
def test_dense_split_budgets(kernels, v):
    (cmp,) = kernels[solve(v, 10, 'd', 48, 13)]
    assert cmp['.vgpr_count'] <= 168 and cmp['.agpr_count'] == 0   # 3 waves / SIMD
    assert cmp['.private_segment_fixed_size'] == 0 and cmp['.vgpr_spill_count'] == 0
    full = kernels[solve(3, 10, 'd', 0, 0)] if v == 3 else kernels[solve(2, 10, 'd', 50, 20)]
    (full,) = full
    assert full['.vgpr_count'] <= 256 and full['.agpr_count'] == 0   # 2 waves / SIMD
    assert full['.private_segment_fixed_size'] == 0 and full['.vgpr_spill_count'] == 0


def _plain_refined(ks):
    """The fp32 build and its fp64-refinement build share kernel names; the
    refined one has the larger LDS block (its fp64 region)."""
    ks = sorted(ks, key=lambda k: k['.group_segment_fixed_size'])
    assert len(ks) == 2
    return ks


@pytest.mark.parametrize('v', [3, 2])
def test_dense_fp32_split_budgets(kernels, v):
    cmp, cmp_r = _plain_refined(kernels[solve(v, 10, 'f', 48, 13)])
    assert cmp['.vgpr_count'] <= 128 and cmp['.agpr_count'] == 0   # 4 waves / SIMD
    assert cmp['.private_segment_fixed_size'] <= 16                # 12 / 8 B/lane measured
    # the refined build's classes run 2 waves / SIMD without scratch (round 5:
    # the unsplit refined kernel at 3 waves spilled 116 B/lane)
    assert cmp_r['.vgpr_count'] <= 256 and cmp_r['.private_segment_fixed_size'] == 0
    if v == 2:
        full, full_r = _plain_refined(kernels[solve(2, 10, 'f', 50, 20)])
        assert full['.vgpr_count'] <= 168 and full['.private_segment_fixed_size'] == 0   # 3 waves
        assert full_r['.vgpr_count'] <= 256 and full_r['.private_segment_fixed_size'] == 0


def test_dense_fp32_builds(kernels):
    plain, refined = _plain_refined(kernels[solve(3, 10, 'f', 0, 0)])
    assert plain['.vgpr_count'] <= 168 and plain['.private_segment_fixed_size'] == 0   # 3 waves, no spill
    assert plain['.group_segment_fixed_size'] <= 160 * 1024 // 12                     # 12 groups / CU
    assert refined['.vgpr_count'] <= 256 and refined['.private_segment_fixed_size'] == 0   # 2 waves, no spill


def test_swing_budget(kernels):
    # the all-swing class (two instances per wave): 3 waves / SIMD, no spill
    (sw,) = kernels['_ZN4hmpc12_GLOBAL__N_112swing_kernelILi10ELi13EEEvNS_9SolveArgsE']
    assert sw['.vgpr_count'] <= 168 and sw['.agpr_count'] == 0
    assert sw['.private_segment_fixed_size'] == 0 and sw['.vgpr_spill_count'] == 0
    assert sw['.group_segment_fixed_size'] <= 160 * 1024 // 12
    assert sw['.sgpr_spill_count'] <= 8   # (the sweep masks stay out of the loop: 196 when hoisted)


def test_riccati_budgets(kernels):
    # the Runner's horizon: the factorisation kernel (3 waves / SIMD, no
    # spill), then the solve kernel without phase 2 (1 wave / SIMD)
    (fac,) = kernels[ric_factor(3, 60, 47)]
    assert fac['.vgpr_count'] <= 168 and fac['.private_segment_fixed_size'] == 0
    (n60,) = kernels[ric(3, 1, 60, 47, 2)]
    assert n60['.private_segment_fixed_size'] == 0
    assert n60['.vgpr_count'] + n60['.agpr_count'] <= 512
    (n20,) = kernels[ric(3, 2, 20, 38)]   # configs[3], 2 waves / SIMD
    assert n20['.vgpr_count'] <= 256 and n20['.agpr_count'] == 0
    assert n20['.private_segment_fixed_size'] <= 24   # 20 B/lane since the one-body MRHS sweeps
    for name, ks in kernels.items():
        if 'ric_kernel' in name:
            for k in ks:
                assert k['.private_segment_fixed_size'] <= 24, name
