"""Kernel throughput of one configuration (device-resident inputs, HIP events
inside the library, hmpc_time_solve_batch): solves/s per precision/kernel.
  python tools/ric_perf.py variant N B [curve] [mu] precision...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hmpc  # noqa: E402
import hmpc_plan as hp  # noqa: E402
from oracle import hmpc_oracle as ho  # noqa: E402


def main():
    variant, N, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    flags = sys.argv[4:]
    curve = 'curve' in flags
    mus = 'mu' in flags
    precs = [f for f in flags if f.startswith('f')] or ['f64']
    inst = hp.sample_instances(B, N, curve=curve, seed=2024, mu_sweep=(0.3, 1.2) if mus else None)
    dev = torch.device('cuda', 0)
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).to(dev)
         for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    c = ho.runner_constants()
    for prec in precs:
        cx = hmpc.Context(variant, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                          precision=prec)
        out = dict(u=torch.empty((B, N, 6), dtype=torch.float64, device=dev),
                   x=torch.empty((B, N + 1, 12), dtype=torch.float64, device=dev),
                   obj=torch.empty(B, dtype=torch.float64, device=dev),
                   status=torch.empty(B, dtype=torch.int32, device=dev),
                   iters=torch.empty(B, dtype=torch.int32, device=dev))
        s = torch.cuda.current_stream(dev).cuda_stream
        cx.time_solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], d['mu'], out, 1, s)
        reps = 3 if N >= 30 or B >= 200000 else 10
        ms = cx.time_solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], d['mu'], out, reps, s)
        st = out['status'].cpu().numpy()
        it = out['iters'].cpu().numpy()
        print(f'{variant} N={N} B={B} {"curve" if curve else "straight"}{" mu" if mus else ""} {prec}: '
              f'{ms:.3f} ms/launch = {B / ms * 1e3:.4g} solves/s; solved {np.mean(st == 0):.4f} '
              f'iters {it.mean():.2f}', flush=True)
        cx.close()


if __name__ == '__main__':
    main()
