"""Per-phase cycles of the generic-horizon kernel (diagnostic build):
    OUT=libhmpc_stamps.so BDIR=build_stamps hopper-mpc-inertial_amd/build.sh -DHMPC_STAMPS
    HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so N=60 B=1 python tools/wide_stamps.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import hmpc  # noqa: E402
import hmpc_plan  # noqa: E402
from oracle import hmpc_oracle as ho  # noqa: E402

NAMES = ['load', 'gen_dt_dynamics', 'sweeps', 'hessian', 'cholesky', 'j_inverse', 'active_set', 'outputs']
N = int(os.environ.get('N', '60'))
B = int(os.environ.get('B', '1'))
inst = hmpc_plan.sample_instances(B, N, curve=True, seed=2024)
d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda() for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
c = ho.runner_constants()
ctx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                   precision=os.environ.get('PREC', 'f64_generic' if N in (5, 10, 20) else 'f64'))
for _ in range(2):
    out = ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
torch.cuda.synchronize()
st = out['x'].view(torch.int64).reshape(B, -1)[:, :9].cpu().numpy()
dur = np.diff(st, axis=1)
res = {n: float(dur[:, i].mean()) for i, n in enumerate(NAMES)}
res['total'] = float((st[:, 8] - st[:, 0]).mean())
res['iters_mean'] = float(out['iters'].float().mean())
print(json.dumps(res, indent=1))
