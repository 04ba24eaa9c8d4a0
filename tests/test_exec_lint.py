"""The round-2 overflow-kernel miscompile, named in round 5:
a VGPR -> AGPR spill copy of a value live into a divergent region, placed in
the region's join block before `s_or_b64 exec` restores the mask, runs with
the region's EXEC (empty after a divergent loop) and leaves the other lanes'
copy stale.  tools/exec_lint.py finds that pattern in the built gfx950 code
objects (no GPU needed).  No kernel on a default path may carry it; the only
findings allowed are in the two-wave dense kernels at N = 20, an A/B-only
precision (HMPC_PREC_F64_DENSE) whose parity test_gpu_parity.py's
test_dense_n20_forced checks on the GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'hopper-mpc-inertial_amd', 'libhmpc.so')
ALLOWED = ('_ZN4hmpc12_GLOBAL__N_112solve_kernelILi3ELi20EdLi0ELi0EEEvNS_9SolveArgsE',
           '_ZN4hmpc12_GLOBAL__N_112solve_kernelILi2ELi20EdLi0ELi0EEEvNS_9SolveArgsE')


def test_no_exec_masked_spill_copies():
    if not os.path.exists(LIB):
        pytest.skip('libhmpc.so not built')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'exec_lint.py'), '--lib', LIB],
                       capture_output=True, text=True)
    findings = [l for l in p.stdout.splitlines() if 'before the exec restore' in l]
    bad = [l for l in findings if l.split(': ')[1] not in ALLOWED]
    assert not bad, '\n'.join(bad)


def _lint(text):
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import exec_lint
    return exec_lint.lint_lines(list(enumerate(text.strip().splitlines(), 1)), 'synthetic')


# the round-2 shape: v182 is live into the region, its AGPR
# copy sits in the join block before the exec restore, and the copy is read
# after it by every lane
HAZARD = """
kern:
  v_add_u32_e32 v182, -6, v194
  s_and_saveexec_b64 s[2:3], s[8:9]
  s_cbranch_execz .LBB0_2
.LBB0_1:
  v_fma_f64 v[10:11], v[12:13], v[14:15], v[10:11]
  s_cbranch_vccnz .LBB0_1
.LBB0_2:
  v_accvgpr_write_b32 a43, v182
  s_or_b64 exec, exec, s[2:3]
  v_accvgpr_read_b32 v8, a43
  s_endpgm
"""


def test_lint_flags_the_named_miscompile():
    found = _lint(HAZARD)
    assert len(found) == 1 and 'a43, v182' in found[0][3]


def test_lint_ignores_region_local_save_restore():
    # a save / restore pair inside the region (the Riccati bucket pass's
    # shape): the inactive lanes never needed the copy
    text = HAZARD.replace('  s_or_b64 exec, exec, s[2:3]\n  v_accvgpr_read_b32 v8, a43',
                          '  v_accvgpr_read_b32 v182, a43\n  s_or_b64 exec, exec, s[2:3]')
    assert _lint(text) == []


def test_lint_ignores_values_made_inside_the_region():
    # the copied VGPR is written after the region's saveexec: a region-local value
    text = HAZARD.replace('.LBB0_2:\n  v_accvgpr_write_b32 a43, v182',
                          '.LBB0_2:\n  v_mov_b32_e32 v182, 0\n  v_accvgpr_write_b32 a43, v182')
    assert _lint(text) == []
