"""Root-cause probe for the x* corruption seen when the Riccati sweeps'
v_fmac_f64_dpp blocks ran in the overflow pass (VERDICT r02
item 1).  Replays every call of the reference's N = 60 run
(tests/golden/loop_3f_N60_config1.npz) as one batch through each library
named on the command line and compares u*, x*, obj with the reference-recorded
x* / u* and with the production library.

  python tools/dpp_probe.py libhmpc_v1.so libhmpc_v2.so ...

Variants (tools/dpp_probe.sh builds them):
  v1  DPP blocks in the overflow pass too (the round-2 failure)
  v2  v1 + s_nop 4 at the END of every block
  v3  v1 + bound_ctrl:1 (a disabled / out-of-row source lane reads 0)
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import os, sys, numpy as np
sys.path.insert(0, os.path.join(%(root)r, 'hopper-mpc-inertial_amd')); sys.path.insert(0, %(root)r)
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
# the overflowed calls: solved again alone, then in a batch of 8 copies
np.savez(os.environ['OUTF'], u=r['u'], x=r['x'], obj=r['obj'], st=r['status'], it=r['iters'])
'''


def run(lib, tag):
    out = os.path.join(ROOT, 'gpurun_out', 'dpp', f'{tag}.npz')
    os.makedirs(os.path.dirname(out), exist_ok=True)
    env = dict(os.environ, HMPC_LIB=os.path.join(ROOT, 'hopper-mpc-inertial_amd', lib), OUTF=out)
    subprocess.check_call([sys.executable, '-c', CODE % {'root': ROOT}], env=env, timeout=300)
    return np.load(out)


def main():
    g = np.load(os.path.join(ROOT, 'tests/golden/loop_3f_N60_config1.npz'))
    n = len(g['k'])
    X = np.stack([g[f'c{c}_xstar'] for c in range(1, n)])
    base = run('libhmpc.so', 'prod')
    print('prod: max|dx| vs reference-recorded x*', float(np.abs(base['x'] - X).max()))
    for lib in sys.argv[1:]:
        tag = os.path.splitext(lib)[0]
        r = run(lib, tag)
        du = np.abs(r['u'] - base['u']).reshape(len(r['u']), -1).max(1)
        dx = np.abs(r['x'] - base['x']).reshape(len(r['x']), -1).max(1)
        bad = np.nonzero(dx > 1e-6)[0]
        print(f'{tag}: max|du| {du.max():.3e}  max|dx| {dx.max():.3e}  max|dobj| '
              f'{np.abs(r["obj"] - base["obj"]).max():.3e}  bad x calls {bad.tolist()}')
        for i in bad[:3]:
            d = np.abs(r['x'][i] - base['x'][i])
            rows = np.nonzero(d.max(1) > 1e-6)[0]
            cols = np.nonzero(d.max(0) > 1e-6)[0]
            print(f'   call {i}: status {int(r["st"][i])} iters {int(r["it"][i])}/{int(base["it"][i])} '
                  f'rows {rows.tolist()[:12]}{"..." if len(rows) > 12 else ""} cols {cols.tolist()}')
            print('   first bad row new ', np.array2string(r['x'][i][rows[0]], precision=4))
            print('   first bad row prod', np.array2string(base['x'][i][rows[0]], precision=4))


if __name__ == '__main__':
    main()
