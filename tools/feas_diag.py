"""Diagnostic: feasibility violations of solved instances at B = 65536 (the
test_large_batch_feasibility_properties workload), per library."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd')); sys.path.insert(0, ROOT)
import hmpc, hmpc_plan
from oracle import hmpc_oracle as ho, port
N = 10
inst = hmpc_plan.sample_instances(65536, N, curve=True, seed=9)
c = ho.runner_constants()
ctx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in inst.items() if k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C')}
for rep in range(2):
    out = ctx.solve_device(dev['x_in'], dev['x_lin'], dev['x_ref'], dev['pf'], dev['C'])
    torch.cuda.synchronize()
    st = out['status'].cpu().numpy(); u = out['u'].cpu().numpy(); it = out['iters'].cpu().numpy()
    viol = np.maximum(np.abs(u[..., 3:5]) - 7.78, 0).max(axis=(1, 2))
    viol = np.maximum(viol, np.maximum(np.abs(u[..., 5]) - 4, 0).max(axis=1))
    bad = np.where((st == 0) & (viol > 1e-7))[0]
    nst = (inst['C'] != 0).sum(1)
    print('rep', rep, 'status counts', np.bincount(st), 'violating', len(bad), 'max viol', viol[st == 0].max())
    for b in bad[:8]:
        print('  b', b, 'viol', viol[b], 'nf', 30 + 3 * nst[b], 'iters', it[b])
    if len(bad):
        sl = bad[:64]
        r = port.solve_batch('3f', N, inst['x_in'][sl], inst['x_lin'][sl], inst['x_ref'][sl], inst['pf'][sl], inst['C'][sl], nthreads=8)
        print('  port status', r['status'][:8], 'max|du| gpu-port', np.abs(r['u'] - u[sl]).reshape(len(sl), -1).max(1)[:8])
