"""What the dense split's early-exit workgroups cost (round 5 probe).

Each class kernel is launched with one workgroup per batch entry (the host
does not know the class sizes); a workgroup past its class list exits at
once.  This times configs[2]-shaped batches whose instances all fall into
one class (C = 0: every window all-swing, so the compacted and full kernels
launch B workgroups that all exit), against the same batch's swing kernel
alone, with rocprofv3's kernel trace giving each kernel's own duration.
    rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/empty_dispatch.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import hmpc  # noqa: E402
import hmpc_plan  # noqa: E402


def main():
    B, N = 65536, 10
    inst = hmpc_plan.sample_instances(B, N, curve=True, seed=2024)
    inst['C'][:] = 0.0   # every window all-swing
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda() for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    c = hmpc_plan.runner_constants()
    cx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    cx.set_order('index')
    out = None
    for _ in range(5):
        out = cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'], out=out)
    torch.cuda.synchronize()
    st = torch.cuda.Event(enable_timing=True)
    en = torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(20):
        out = cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'], out=out)
    en.record()
    torch.cuda.synchronize()
    print('all-swing step ms', st.elapsed_time(en) / 20, 'solved', int((out['status'] == 0).sum()))


if __name__ == '__main__':
    main()
