"""PCIe-inclusive rate of the host-buffer entry point (hmpc_solve_batch_host):
inputs in pageable host numpy arrays, outputs back in host arrays, i.e. the
staging copies through the context's device buffers are inside the timed
region.  Reported in DESIGN.md beside bench.py's HBM-resident `value`.

    python tools/bench_host.py [--batch 65536] [--N 10] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'hopper-mpc-inertial_amd'), ROOT):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import hmpc  # noqa: E402
import hmpc_plan  # noqa: E402
from oracle import hmpc_oracle as ho  # noqa: E402  (runner constants only)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=65536)
    ap.add_argument('--N', type=int, default=10)
    ap.add_argument('--reps', type=int, default=10)
    args = ap.parse_args()
    B, N = args.batch, args.N
    inst = hmpc_plan.sample_instances(B, N, curve=True, seed=2024)
    c = ho.runner_constants()
    ctx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                       device=0)
    ins = [np.ascontiguousarray(inst[k]) for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')]
    ctx.solve_host(*ins[:5], mu=ins[5])   # warm-up (allocates the staging buffers)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        out = ctx.solve_host(*ins[:5], mu=ins[5])
    dt = (time.perf_counter() - t0) / args.reps
    ok = float(np.mean(np.asarray(out['status']) == 0))
    ctx.close()
    print(json.dumps({'path': 'hmpc_solve_batch_host (pageable host buffers, PCIe-inclusive)',
                      'variant': '3f', 'N': N, 'batch': B, 'reps': args.reps,
                      'ms_per_batch': dt * 1e3, 'solves_per_s': B / dt, 'solved_frac': ok}))


if __name__ == '__main__':
    main()
