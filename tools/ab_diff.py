"""u* of two libhmpc builds on the same instances (A/B correctness check)."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(%r, 'hopper-mpc-inertial_amd')); sys.path.insert(0, %r)
import hmpc, hmpc_plan
from oracle import hmpc_oracle as ho
c = ho.runner_constants()
res = {}
for var, N, curve in (('3f', 10, True), ('2f', 10, True), ('3f', 5, False), ('2f', 5, True)):
    inst = hmpc_plan.sample_instances(256, N, curve=curve, seed=3, variant=var) if 'variant' in hmpc_plan.sample_instances.__code__.co_varnames else hmpc_plan.sample_instances(256, N, curve=curve, seed=3)
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda() for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    ctx = hmpc.Context(var, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    o = ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    torch.cuda.synchronize()
    np.save(os.environ['OUTF'] + f'_{var}{N}.npy', o['u'].cpu().numpy())
    np.save(os.environ['OUTF'] + f'_{var}{N}_st.npy', o['status'].cpu().numpy())
''' % (ROOT, ROOT)
out = os.path.join(ROOT, 'gpurun_out', 'abdiff')
os.makedirs(out, exist_ok=True)
for tag, lib in (('new', 'libhmpc.so'), ('prev', 'libhmpc_prev.so')):
    env = dict(os.environ, HMPC_LIB=os.path.join(ROOT, 'hopper-mpc-inertial_amd', lib), OUTF=os.path.join(out, tag))
    subprocess.check_call([sys.executable, '-c', code], env=env, timeout=200)
import numpy as np
for k in ('3f10', '2f10', '3f5', '2f5'):
    a = np.load(os.path.join(out, f'new_{k}.npy')); b = np.load(os.path.join(out, f'prev_{k}.npy'))
    sa = np.load(os.path.join(out, f'new_{k}_st.npy')); sb = np.load(os.path.join(out, f'prev_{k}_st.npy'))
    d = np.abs(a - b).max(axis=(1, 2)) if a.ndim == 3 else np.abs(a - b).reshape(len(a), -1).max(axis=1)
    print(k, 'max|du|', float(d.max()), 'n_bad', int((d > 1e-6).sum()), 'status diff', int((sa != sb).sum()), 'first bad', np.nonzero(d > 1e-6)[0][:8].tolist())
