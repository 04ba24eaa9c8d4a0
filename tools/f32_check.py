"""fp32 vs fp64 on the dense N = 10 kernel (BASELINE configs[4]): statuses,
|du| and objective error against the C port over a sample of the bench
workload.   python tools/f32_check.py [B]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import hmpc  # noqa: E402
import hmpc_plan  # noqa: E402
from oracle import port  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = 10
inst = hmpc_plan.sample_instances(B, N, curve=True, seed=2024)
c = hmpc_plan.runner_constants()
ref = port.solve_batch('3f', N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                       mu=inst['mu'], nthreads=16)
out = {}
for prec in ('f64', 'f32', 'f32_generic'):
    cx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                      precision=prec)
    g = cx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    name = cx.kernel_name
    cx.close()
    ok = (ref['status'] == 0) & (g['status'] == 0)
    du = np.abs(g['u'][ok] - ref['u'][ok]).max(axis=(1, 2))
    rel = np.abs(g['obj'][ok] - ref['obj'][ok]) / np.abs(ref['obj'][ok])
    mism = {}
    for a, b in zip(g['status'][g['status'] != ref['status']], ref['status'][g['status'] != ref['status']]):
        mism[f'{int(a)},{int(b)}'] = mism.get(f'{int(a)},{int(b)}', 0) + 1
    out[prec] = {'kernel': name, 'solved': int((g['status'] == 0).sum()), 'status_mismatch': mism,
                 'du_max': float(du.max()), 'du_p50': float(np.median(du)), 'du_p99': float(np.percentile(du, 99)),
                 'obj_rel_max': float(rel.max()), 'obj_rel_p50': float(np.median(rel)),
                 'iters_mean': float(g['iters'].mean())}
print(json.dumps({'B': B, 'port_solved': int((ref['status'] == 0).sum()), 'results': out}, indent=1))
