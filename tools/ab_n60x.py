"""x* and u* of the N=60 reference-loop replay (tests/golden/loop_3f_N60_config1.npz)
through libhmpc.so vs libhmpc_prev.so (and any libhmpc_<tag>.so named on the
command line): a mismatch in x* that u* does not show points at the outputs
phase or the overflow pass."""
import os, sys, numpy as np, subprocess
ROOT='/root/repo'
code = r'''
import os, sys, numpy as np
sys.path.insert(0, os.path.join(%r, 'hopper-mpc-inertial_amd')); sys.path.insert(0, %r)
import hmpc
from oracle import hmpc_oracle as ho
g = np.load(os.path.join(%r, 'tests/golden/loop_3f_N60_config1.npz'))
N = int(g['N']); c0 = ho.runner_constants(); n = len(g['k'])
x_in = np.stack([g['x_in'][c] for c in range(1, n)])
x_lin = np.stack([np.vstack([g['x_in'][c], g[f'c{c - 1}_xstar'][2:], g[f'c{c - 1}_xstar'][-1:]]) for c in range(1, n)])
x_ref = np.stack([g[f'c{c}_x_ref'] for c in range(1, n)]); pf = np.stack([g[f'c{c}_pf'] for c in range(1, n)])
C = np.stack([g['C'][c] for c in range(1, n)])
cx = hmpc.Context('3f', N, t=c0['t'], m=c0['m'], g=c0['g'], mu=1.0, Jinv=c0['Jinv'], rh=c0['rh'])
r = cx.solve_host(x_in, x_lin, x_ref, pf, C)
np.savez(os.environ['OUTF'], u=r['u'], x=r['x'], st=r['status'], it=r.get('iters', r['status']))
''' % (ROOT, ROOT, ROOT)
os.makedirs(ROOT + '/gpurun_out/abx', exist_ok=True)
extra = sys.argv[1:]   # more libhmpc_<tag>.so builds to compare with prev
for tag, lib in [('new', 'libhmpc.so'), ('prev', 'libhmpc_prev.so')] + [(t, f'libhmpc_{t}.so') for t in extra]:
    env = dict(os.environ, HMPC_LIB=os.path.join(ROOT, 'hopper-mpc-inertial_amd', lib), OUTF=ROOT + f'/gpurun_out/abx/{tag}.npz')
    subprocess.check_call([sys.executable, '-c', code], env=env, timeout=200)
a = np.load(ROOT + '/gpurun_out/abx/new.npz'); b = np.load(ROOT + '/gpurun_out/abx/prev.npz')
du = np.abs(a['u'] - b['u']).reshape(len(a['u']), -1).max(1); dx = np.abs(a['x'] - b['x']).reshape(len(a['x']), -1).max(1)
print('du max', du.max(), 'dx max', dx.max(), 'bad x calls', np.nonzero(dx > 1e-6)[0].tolist()[:20])
i = int(np.argmax(dx)); print('call', i, 'iters new/prev', a['it'][i], b['it'][i], 'status', a['st'][i], b['st'][i])
d = np.abs(a['x'][i] - b['x'][i]); print('rows with diff', np.nonzero(d.max(1) > 1e-6)[0].tolist()[:10], 'cols', np.nonzero(d.max(0) > 1e-6)[0].tolist())
print(a['x'][i][-3:], b['x'][i][-3:])
for tag in extra:
    f = ROOT + f'/gpurun_out/abx/{tag}.npz'
    if os.path.exists(f):
        c = np.load(f)
        print(tag, 'du', np.abs(c['u'] - b['u']).max(), 'dx', np.abs(c['x'] - b['x']).max())
