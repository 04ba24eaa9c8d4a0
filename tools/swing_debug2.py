"""Swing-class debug 2: all-swing batches with deterministic pairing (one
classify block): distinct pairs vs duplicated pairs, each against the port."""
import sys, os
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd')); sys.path.insert(0, ROOT)
import hmpc, hmpc_plan as hp
from oracle import port
N = 10
a = hp.sample_instances(4096, N, curve=True, seed=11, mu_sweep=(0.3, 1.2))
nst = (a['C'] != 0).sum(1)
sw = np.where(nst == 0)[0][:512]
c = hp.runner_constants()
keys = ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')
def run(idx, tag):
    inst = {k: np.ascontiguousarray(a[k][idx]) for k in keys}
    d = {k: torch.from_numpy(inst[k]).cuda() for k in keys}
    cx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'], device=0)
    o = cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in o.items()}
    cx.close()
    p = port.solve_batch('3f', N, *[inst[k] for k in keys[:5]], mu=inst['mu'], nthreads=8)
    du = np.abs(o['u'] - p['u']).reshape(len(idx), -1).max(1)
    bad = du > 1e-6
    print(f'{tag}: B={len(idx)} bad {int(bad.sum())} (even {int(bad[0::2].sum())}, odd {int(bad[1::2].sum())}); '
          f'iters gpu {np.bincount(o["iters"])} port {np.bincount(p["iters"])}')
    w = np.where(bad)[0][:8]
    for i in w:
        print(f'   i={i} du={du[i]:.3e} it gpu {o["iters"][i]} port {p["iters"][i]} st {o["status"][i]},{p["status"][i]} '
              f'u gpu {np.round(o["u"][i, :, 3:].ravel()[:9], 4)} port {np.round(p["u"][i, :, 3:].ravel()[:9], 4)}')
    return o
run(sw, 'distinct')
run(np.repeat(sw[:256], 2), 'duplicated')
o1 = run(np.repeat(sw[:1], 2), 'one pair')
it = a['C'][sw]
# instances with port iterations > 0 paired with themselves
p = port.solve_batch('3f', N, *[np.ascontiguousarray(a[k][sw]) for k in keys[:5]], mu=a['mu'][sw], nthreads=8)
hard = sw[p['iters'] > 0][:64]
run(np.repeat(hard, 2), 'hard duplicated')
run(hard, 'hard distinct')
