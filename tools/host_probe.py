"""Host-side cost of one solve step (GPU box): is the launch loop ahead of the GPU?

    python tools/host_probe.py [B] [variant] [N] [straight]

Times K back-to-back ``Context.solve_device`` calls twice: the enqueue loop
alone (perf_counter until the loop returns, no sync) and enqueue + sync.  If
the enqueue time per step is close to the synced time per step, the GPU waits
for the host between launches (the gaps a kernel trace shows between steps).
Also times the bare C call (pointers prepared once) to split Python checks
from the library's own host work.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import hmpc  # noqa: E402
import hmpc_plan  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    var = sys.argv[2] if len(sys.argv) > 2 else '2f'
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    straight = (sys.argv[4] == 'straight') if len(sys.argv) > 4 else True
    inst = hmpc_plan.sample_instances(B, N, curve=not straight, seed=2024)
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda() for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    c = hmpc_plan.runner_constants()
    cx = hmpc.Context(var, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    dev = d['x_in'].device
    out = dict(u=torch.empty((B, N, 6), dtype=torch.float64, device=dev),
               x=torch.empty((B, N + 1, 12), dtype=torch.float64, device=dev),
               obj=torch.empty(B, dtype=torch.float64, device=dev),
               status=torch.empty(B, dtype=torch.int32, device=dev),
               iters=torch.empty(B, dtype=torch.int32, device=dev),
               active=torch.empty(B, dtype=torch.int32, device=dev))
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream

    def py_step():
        cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'], out=out, stream=s)

    ptrs = [ctypes.c_void_p(t.data_ptr()) for t in (d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], d['mu'],
                                                    out['u'], out['x'], out['obj'], out['status'],
                                                    out['iters'], out['active'])]
    fn = cx._lib.hmpc_solve_batch_stats
    h = cx._h
    sv = ctypes.c_void_p(s)

    def c_step():
        fn(h, B, *ptrs, sv)

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def ev_step():
        ev[0].record(stream)
        py_step()
        ev[1].record(stream)

    res = {'B': B, 'variant': var, 'N': N, 'straight': straight}
    for _ in range(300):
        py_step()
    torch.cuda.synchronize()
    K = 200
    for name, f in (('python', py_step), ('c_call', c_step), ('bench_step', ev_step)):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                f()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        res[name] = {'enqueue_us_per_step': (t1 - t0) / K * 1e6, 'synced_us_per_step': (t2 - t0) / K * 1e6}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
