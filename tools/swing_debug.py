"""Swing-class debug: repeat the same batch, report instances whose results
differ between runs or from the C port."""
import sys, os
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd')); sys.path.insert(0, ROOT)
import hmpc, hmpc_plan as hp
from oracle import port
N = 10
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
curve = True
a = hp.sample_instances(B, N, curve=curve, seed=11, mu_sweep=(0.3, 1.2))
c = hp.runner_constants()
d = {k: torch.from_numpy(np.ascontiguousarray(a[k])).cuda() for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
nst = (a['C'] != 0).sum(1)
outs = []
for r in range(4):
    cx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'], device=0)
    o = cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    torch.cuda.synchronize()
    outs.append({k: v.cpu().numpy() for k, v in o.items()})
    cx.close()
p = port.solve_batch('3f', N, a['x_in'], a['x_lin'], a['x_ref'], a['pf'], a['C'], mu=a['mu'], nthreads=8)
print('nst==0:', int((nst == 0).sum()), 'of', B)
for r in range(1, 4):
    for k in ('u', 'x', 'obj', 'status', 'iters'):
        x0, x1 = outs[0][k], outs[r][k]
        bad = np.where((x0 != x1).reshape(B, -1).any(1))[0]
        if len(bad):
            print(f'run {r} {k}: {len(bad)} differ, nst {np.bincount(nst[bad])}, idx {bad[:10]}',
                  'maxdiff', float(np.abs(x0[bad] - x1[bad]).max()))
sw = nst == 0
ok = (p['status'] == 0) & (outs[0]['status'] == 0)
du = np.abs(outs[0]['u'] - p['u']).reshape(B, -1).max(1)
print('status mismatch', int((p['status'] != outs[0]['status']).sum()), 'swing', int((p['status'] != outs[0]['status'])[sw].sum()))
print('max du swing', float(du[ok & sw].max()) if (ok & sw).any() else None, 'non-swing', float(du[ok & ~sw].max()))
dob = np.abs(outs[0]['obj'] - p['obj']) / np.abs(p['obj'])
print('max dobj swing', float(dob[ok & sw].max()), 'iters swing', np.bincount(outs[0]['iters'][sw]))
w = np.where(ok & sw & (du > 1e-6))[0]
print('bad swing idx', w[:20], du[w[:20]])
