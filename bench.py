#!/usr/bin/env python3
"""Benchmark of the MI355X batched MPC/QP solve path (BASELINE.json metric).

One *step* = one pass of the hot path over one batch: every instance's
``Mpc.gen_dt_dynamics`` + ``Mpc.build_qp`` + ``Mpc.solve_qp``
(src/mpc_cvx_euler_3f.py:71-160) on the GPU through the C ABI
(``hmpc_solve_batch``), then -- for N > 1 ranks -- the RCCL all-gather of the
per-instance objective and status, one packed collective per
step on a side stream, overlapping the next step's solve
(``hmpc_dist.ResultExchange``); the timed region ends after every exchange.
Inputs are resident in HBM before the timed region starts.

Default workload = BASELINE.json configs[2]: 65536 randomised instances per
GPU, 3f, horizon N = 10, --curve reference plan, fp64 (weak scaling: every
rank solves its own 65536-instance shard of the global batch).

Launch:  python bench.py [--gpus 1] [--steps K] [--warmup W]
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'hopper-mpc-inertial_amd')
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

METRIC = 'QP solves/sec (N=10, 3f) at batch=65k, 1→8 MI355X; max |u*−u*_cvxpy|'
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
FP64_VECTOR_PEAK_TFS = 78.6   # MI355X FP64 vector (half the 157.3 TF FP32 vector rate)


def algorithmic_bytes(N, with_mu=True):
    """HBM bytes one solve must move: inputs x_in, x_lin,
    x_ref, pf, C (+ mu), outputs u, x, obj (fp64) and status (int32)."""
    nin = 12 + 12 * (N + 1) + 12 * N + 3 * N + N + (1 if with_mu else 0)
    nout = 6 * N + 12 * (N + 1) + 1
    return 8 * (nin + nout) + 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=65536, help='instances per GPU')
    ap.add_argument('--variant', default='3f', choices=['3f', '2f'])
    ap.add_argument('--N', type=int, default=10)
    ap.add_argument('--straight', action='store_true', help='straight plan (default: --curve)')
    ap.add_argument('--mu-sweep', action='store_true', help='mu ~ U(0.3, 1.2)')
    ap.add_argument('--seed', type=int, default=2024)
    ap.add_argument('--precision', default='f64', choices=['f64', 'f32', 'f64_generic'],
                    help='configs[4]: f32 = fp32 arithmetic on the generic kernel; '
                         'f64_generic = its fp64 twin (f64 = the dedicated fp64 kernel)')
    ap.add_argument('--cpu-seconds', type=float, default=10.0,
                    help='budget of the bounded CPU-baseline sample (0 disables)')
    return ap.parse_args()


def cpu_baseline(args, inst, gpu_u, gpu_status, budget_s):
    """Reported baseline, not the target: the oracle's C port (oracle/hmpc_port.c:
    the reference's gen_dt_dynamics/build_qp restated in C, condensed densely
    and solved exactly by a classic dual active set; OpenMP over instances)
    timed on this host's cores over a bounded prefix of the same workload.
    Also returns the parity of those instances against the GPU results."""
    from oracle import port
    if budget_s <= 0:
        return None, None
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))   # the GPU box's CPU share per GPU
    chunk = 256 * cores
    keys = ('x_in', 'x_lin', 'x_ref', 'pf', 'C')
    port.solve_batch(args.variant, args.N, *[inst[k][:cores] for k in keys],
                     mu=inst['mu'][:cores], nthreads=cores)   # warm (thread pool)
    # chunks of the rank-0 shard in order, wrapping round (further passes over
    # the same instances) until the budget is spent; parity on the first pass
    n, done, du, el = 0, 0, 0.0, 0.0
    B = len(inst['x_in'])
    while el < budget_s:
        lo = done % B
        sl = slice(lo, min(lo + chunk, B))
        t0 = time.perf_counter()
        r = port.solve_batch(args.variant, args.N, *[inst[k][sl] for k in keys], mu=inst['mu'][sl],
                             nthreads=cores)
        el += time.perf_counter() - t0
        if done < B:
            ok = (r['status'] == 0) & (gpu_status[sl] == 0)
            if ok.any():
                du = max(du, float(np.abs(r['u'][ok] - gpu_u[sl][ok]).max()))
            n = sl.stop
        done += sl.stop - sl.start
    base = {'value': done / el, 'unit': 'QP solves/s', 'cores': cores, 'kind': 'port',
            'sample': f'{done} solves = {done / B:.1f} passes over the {B}-instance rank-0 shard '
                      f'in {el:.1f} s; C restatement of the reference gen_dt_dynamics/build_qp + '
                      f'exact dense dual active-set solve (oracle/hmpc_port.c, OpenMP, '
                      f'{cores} threads)'}
    parity = {'instances': n, 'max_abs_du_vs_port': du}
    return base, parity


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}')
    if not torch.cuda.is_available():
        raise SystemExit('bench.py needs an MI355X (torch.cuda.is_available() is False)')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)

    import hmpc
    import hmpc_plan
    from oracle import hmpc_oracle as ho   # constants only (Runner values)

    N, B = args.N, args.batch
    inst = hmpc_plan.sample_instances(B, N, curve=not args.straight, seed=args.seed,
                                      mu_sweep=(0.3, 1.2) if args.mu_sweep else None,
                                      start=rank * B)   # hmpc_dist.shard_start
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).to(dev)
         for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    c = ho.runner_constants()
    ctx = hmpc.Context(args.variant, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'],
                       rh=c['rh'], device=local, precision=args.precision)
    out = dict(u=torch.empty((B, N, 6), dtype=torch.float64, device=dev),
               x=torch.empty((B, N + 1, 12), dtype=torch.float64, device=dev),
               obj=torch.empty(B, dtype=torch.float64, device=dev),
               status=torch.empty(B, dtype=torch.int32, device=dev),
               iters=torch.empty(B, dtype=torch.int32, device=dev))
    import hmpc_dist
    stream = torch.cuda.current_stream(dev)
    # N > 1: the exchange step (per-instance cost + status) is one
    # all-gather of a packed [obj | status] slot on a side stream, pipelined
    # with the next step's solve (double-buffered slots, hmpc_dist)
    ex = hmpc_dist.ResultExchange(B, dev) if world > 1 else None
    last = [out]

    def step(ev=None):
        o = out
        if ex is not None:
            ob, sb = ex.outputs()
            o = dict(out, obj=ob, status=sb)
        if ev is not None:
            ev[0].record(stream)
        ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'],
                         out=o, stream=stream.cuda_stream)
        if ev is not None:
            ev[1].record(stream)
        if ex is not None:
            ex.exchange()
        last[0] = o

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    tt = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el, kern_ms_max = float(tt[0]), float(tt[1])

    st = last[0]['status'].cpu().numpy()
    it = out['iters'].cpu().numpy()
    solved_local = float((st == 0).mean())
    sf = torch.tensor([solved_local], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(sf, op=dist.ReduceOp.MIN)

    base = parity = None
    if rank == 0 and world == 1:
        base, parity = cpu_baseline(args, inst, out['u'].cpu().numpy(), st, args.cpu_seconds)

    if rank == 0:
        bpsolve = algorithmic_bytes(N)
        achieved = bpsolve * B / (kern_ms * 1e-3) / 1e9
        traffic = None
        flops = None
        tpath = os.path.join(ROOT, 'profiles', 'traffic.json')
        wl = f'{args.variant}_N{N}_B{B}_{"straight" if args.straight else "curve"}' \
             f'{"_musweep" if args.mu_sweep else ""}'
        if os.path.exists(tpath) and args.precision == 'f64':
            tj = json.load(open(tpath))
            traffic = tj.get(wl, {}).get('bytes_per_launch')
            flops = tj.get(wl, {}).get('fp64_flops_per_solve')
        total = B * world * args.steps
        rec = {
            'metric': METRIC,
            'value': total / el,
            'unit': 'QP solves/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': el / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f32' if args.precision == 'f32' else 'f64',
            'data': 'synthetic: Runner path_plan_init plan (--curve) + randomised x0 '
                    '(SURVEY.md 8d), generated on host, resident in HBM before timing',
            'config': {'workload': f'configs[2]: batch={B}/GPU randomised x0 + '
                                   f'{"straight" if args.straight else "--curve"} ref traj, '
                                   f'{args.variant}, horizon N={N}, fp64'
                                   f'{", mu sweep" if args.mu_sweep else ""}'
                                   f'{"" if args.precision == "f64" else ", " + args.precision + " (generic kernel)"}',
                       'global_batch': B * world, 'horizon': N, 'variant': args.variant,
                       'parallelism': f'shard{world}'},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'kernel': (f'hmpc::solve_kernel<{args.variant[0]}, {N}>' if args.precision == 'f64' else f'hmpc::wide_kernel<{args.variant[0]}, {"float" if args.precision == "f32" else "double"}>'),
                         'kernel_ms': kern_ms, 'kernel_ms_max_rank': kern_ms_max,
                         'algorithmic_bytes_per_solve': bpsolve, 'solves_per_launch': B},
            # the bound that matters for this path: executed fp64
            # VALU flops (rocprofv3 SQ_INSTS_VALU_*_F64 x 64 lanes, profiles/)
            'fp64_vector': None if flops is None else {
                'achieved': flops * B / (kern_ms * 1e-3) / 1e12, 'peak': FP64_VECTOR_PEAK_TFS,
                'unit': 'TFLOP/s', 'frac': flops * B / (kern_ms * 1e-3) / 1e12 / FP64_VECTOR_PEAK_TFS,
                'flops_per_solve': flops},
            'cpu_baseline': base,
            'solved_frac_min_rank': float(sf[0]),
            'iters_mean': float(it.mean()), 'iters_max': int(it.max()),
            'parity_sample': parity,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == '__main__':
    main()
