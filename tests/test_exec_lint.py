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
