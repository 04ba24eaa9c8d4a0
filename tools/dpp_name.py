"""Round-5 DPP probe: the round-2 source (beb219c) with
the v_fmac_f64_dpp sweep blocks forced into the overflow pass, instrumented
with printf in the x* rollout of call 93 (stages 14-17, lanes 6-11).
tools/dpp_old/ holds that build's Python package and libraries (built here
from `git archive beb219c`).  Prints each library's x*
error on the reference-recorded run and the rollout values."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OLD = os.path.join(ROOT, 'tools', 'dpp_old')
CODE = r'''
import os, sys, numpy as np
sys.path.insert(0, %(old)r); sys.path.insert(0, %(root)r)
import hmpc
from oracle import hmpc_oracle as ho
g = np.load(os.path.join(%(root)r, 'tests/golden/loop_3f_N60_config1.npz'))
N = int(g['N']); c0 = ho.runner_constants(); n = len(g['k'])
x_in = np.stack([g['x_in'][c] for c in range(1, n)])
x_lin = np.stack([np.vstack([g['x_in'][c], g[f'c{c - 1}_xstar'][2:], g[f'c{c - 1}_xstar'][-1:]]) for c in range(1, n)])
x_ref = np.stack([g[f'c{c}_x_ref'] for c in range(1, n)]); pf = np.stack([g[f'c{c}_pf'] for c in range(1, n)])
C = np.stack([g['C'][c] for c in range(1, n)])
cx = hmpc.Context('3f', N, t=c0['t'], m=c0['m'], g=c0['g'], mu=1.0, Jinv=c0['Jinv'], rh=c0['rh'])
r = cx.solve_host(x_in, x_lin, x_ref, pf, C)
X = np.stack([g[f'c{c}_xstar'] for c in range(1, n)])
dx = np.abs(r['x'] - X).reshape(len(X), -1).max(1)
print('RESULT max|dx| %%.3e bad calls %%s' %% (dx.max(), list(np.nonzero(dx > 1e-6)[0] + 1)), flush=True)
'''

for lib in sys.argv[1:]:
    env = dict(os.environ, HMPC_LIB=os.path.join(OLD, lib))
    p = subprocess.run([sys.executable, '-c', CODE % {'root': ROOT, 'old': OLD}], env=env, capture_output=True,
                       text=True, timeout=300)
    print(f'== {lib} rc {p.returncode}')
    lines = [l for l in p.stdout.splitlines() if l.startswith(('RESULT', 'DPPDBG'))]
    for l in sorted(set(lines), key=lambda l: (not l.startswith('RESULT'), l)):
        print(l)
    if p.returncode:
        print(p.stderr[-2000:])
