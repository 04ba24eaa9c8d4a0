#!/usr/bin/env python3
"""Benchmark of the MI355X batched MPC/QP solve path (BASELINE.json metric).

One *step* = one pass of the hot path over one batch: every instance's
``Mpc.gen_dt_dynamics`` + ``Mpc.build_qp`` + ``Mpc.solve_qp``
(src/mpc_cvx_euler_3f.py:71-160) on the GPU through the C ABI
(``hmpc_solve_batch``: the solve kernel, then the active-set overflow pass),
then -- for N > 1 ranks -- the RCCL all-gather of the per-instance objective
and status, one packed collective per step on a side stream,
overlapping the next step's solve (``hmpc_dist.ResultExchange``); the timed
region ends after every exchange.  Inputs are resident in HBM before the
timed region starts.

Default workload = BASELINE.json configs[2]: 65536 randomised instances per
GPU, 3f, horizon N = 10, --curve reference plan, fp64 (weak scaling: every
rank solves its own 65536-instance shard).  ``--global-batch G`` instead
splits a fixed global batch over the ranks (strong scaling; configs[3] is
``--N 20 --straight --mu-sweep --global-batch 262144``).

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
FP64_VECTOR_SPEC_TFS = 78.6   # MI355X FP64 vector datasheet figure (half the FP32 vector rate)
FP32_VECTOR_SPEC_TFS = 157.3  # MI355X FP32 vector (MI355X_MICROARCH.md)


def measured_peaks():
    """The vector FMA peaks measured on the box (tools/fp64_peak.hip, committed
    as profiles/r03_fp64_peak.json); the datasheet figures when absent."""
    p = os.path.join(ROOT, 'profiles', 'r03_fp64_peak.json')
    if os.path.exists(p):
        d = json.load(open(p))
        return d['fp64_fma_tflops'], d['fp32_fma_tflops'], 'measured (profiles/r03_fp64_peak.json)'
    return FP64_VECTOR_SPEC_TFS, FP32_VECTOR_SPEC_TFS, 'datasheet'


def algorithmic_bytes(N, with_mu=True):
    """HBM bytes one solve must move: inputs x_in, x_lin,
    x_ref, pf, C (+ mu), outputs u, x, obj (fp64) and status (int32)."""
    nin = 12 + 12 * (N + 1) + 12 * N + 3 * N + N + (1 if with_mu else 0)
    nout = 6 * N + 12 * (N + 1) + 1
    return 8 * (nin + nout) + 4


def algorithmic_flops(kernel, N, iters, q):
    """fp64 flops one solve needs in the algorithm the kernel runs (2 per
    FMA; DESIGN.md 5 derives each term), as a closed form over the horizon N,
    the active-set iterations and the active-set size q (the mean final size
    the kernels report, hmpc_solve_batch_stats) -- useful arithmetic, not
    executed lanes.

    dense (condensed, NV = 6N): Hessian rows 210 N(N+1) + Cholesky NV^3/3 +
      unconstrained 2 NV^2 + per iteration (2 NV^2 + 4 q NV + q^2) + 400 N
    Riccati: factorisation 4480 N + unconstrained 720 N + per iteration
      (1440 N + 2 q^2 + 80 N) + 400 N
    """
    NV = 6 * N
    if 'ric_kernel' in kernel:
        return 4480 * N + 720 * N + iters * (1440 * N + 2 * q * q + 80 * N) + 400 * N
    return 210 * N * (N + 1) + NV ** 3 / 3 + 2 * NV * NV + iters * (2 * NV * NV + 4 * q * NV + q * q) + 400 * N


def workload_label(args, world):
    """Which BASELINE.json config this run measures (configs[0] is the
    reference's own CPU run.py, whose MPC horizon is N = 60)."""
    gb = args.global_batch or args.batch * world
    curve = not args.straight
    if args.precision in ('f32', 'f32_generic') and args.variant == '3f' and args.N == 10:
        return f'configs[4]: batch={gb}, 3f, N=10, fp32 (vs fp64) tolerance/throughput trade-off'
    if args.precision == 'f32_refined' and args.variant == '3f' and args.N == 10:
        return (f'configs[4]: batch={gb}, 3f, N=10, fp32 + {args.refine} fp64 corrections (vs fp64) '
                f'tolerance/throughput trade-off')
    if args.variant == '2f' and args.N == 10 and not curve:
        return f'configs[1]: batch={gb} randomised x0, 2f (planar, Fy=0), horizon N=10, fp64'
    if args.variant == '3f' and args.N == 10 and curve:
        return f'configs[2]: batch={gb} randomised x0 + --curve ref traj, 3f, horizon N=10, fp64'
    if args.variant == '3f' and args.N == 20 and args.mu_sweep:
        return (f'configs[3]: batch={gb}, 3f, horizon N=20 + friction-cone sweep, '
                f'{"strong" if args.global_batch else "weak"} scaling over {world} GPU(s)')
    if args.N == 60:
        return (f'Runner horizon N=60 (configs[0]: run.py 3f --N_run=2000, src/robotrunner.py:46): '
                f'batch={gb}, {args.variant}, {"--curve" if curve else "straight"}')
    return (f'custom: batch={gb}, {args.variant}, N={args.N}, {"--curve" if curve else "straight"}'
            f'{", mu sweep" if args.mu_sweep else ""}, {args.precision}')


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--batch', type=int, default=65536, help='instances per GPU (weak scaling)')
    ap.add_argument('--global-batch', type=int, default=0,
                    help='fixed global batch split over the ranks (strong scaling)')
    ap.add_argument('--variant', default='3f', choices=['3f', '2f'])
    ap.add_argument('--N', type=int, default=10)
    ap.add_argument('--straight', action='store_true', help='straight plan (default: --curve)')
    ap.add_argument('--mu-sweep', action='store_true', help='mu ~ U(0.3, 1.2)')
    ap.add_argument('--seed', type=int, default=2024)
    ap.add_argument('--precision', default='f64',
                    choices=['f64', 'f32', 'f32_refined', 'f64_generic', 'f64_riccati', 'f64_dense',
                             'f32_generic'],
                    help='f64 = the fastest fp64 kernel for N (default); f32 = fp32 one-wave '
                         'kernel, f32_refined = fp32 + --refine fp64 corrections (configs[4]); '
                         'others force a kernel for A/B runs')
    ap.add_argument('--refine', type=int, default=5, help='fp64 corrections of f32_refined (5: max|du| <= 1e-6)')
    ap.add_argument('--order', default='auto', choices=['auto', 'index', 'longest_first'],
                    help='instance order (hmpc_set_order; auto = longest-first for small batches)')
    ap.add_argument('--prewarm-ms', type=float, default=1500.0,
                    help='untimed, duration-based pre-warm before the warm-up steps (solves only, no '
                         'exchange): brings the clock to its steady state, which the first ~15 launches '
                         'otherwise ramp through (DESIGN.md 5); 0 disables.  Changes neither --steps, '
                         '--warmup nor the timed region')
    ap.add_argument('--cpu-seconds', type=float, default=12.0,
                    help='budget of the bounded CPU-baseline sample, split over its two legs '
                         '(all cores, then one core); 0 disables')
    return ap.parse_args()


def cpu_threads():
    """The CPU share this process may use: its affinity set, capped by
    OMP_NUM_THREADS (the GPU box sets 16 per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get('OMP_NUM_THREADS')
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(args, inst, gpu_u, gpu_status, budget_s):
    """Reported baseline, not the target: the oracle's C port (oracle/hmpc_port.c:
    the reference's gen_dt_dynamics/build_qp restated in C, condensed densely
    and solved exactly by a classic dual active set; OpenMP over instances)
    timed on this host over a bounded prefix of the same workload, on every
    core of this process's CPU share and on one core.  Also returns the parity
    of those instances against the GPU: max|du| where both solved, and every
    (gpu status, port status) disagreement counted."""
    from oracle import port
    if budget_s <= 0:
        return None, None
    keys = ('x_in', 'x_lin', 'x_ref', 'pf', 'C')
    B = len(inst['x_in'])

    def leg(threads, seconds, check):
        chunk = 64 * threads
        port.solve_batch(args.variant, args.N, *[inst[k][:threads] for k in keys], mu=inst['mu'][:threads],
                         nthreads=threads)   # warm (thread pool)
        done, el = 0, 0.0
        du, mism, n = 0.0, {}, 0
        while el < seconds:
            lo = done % B
            sl = slice(lo, min(lo + chunk, B))
            t0 = time.perf_counter()
            r = port.solve_batch(args.variant, args.N, *[inst[k][sl] for k in keys], mu=inst['mu'][sl],
                                 nthreads=threads)
            el += time.perf_counter() - t0
            if check and done < B:
                gs, ps = gpu_status[sl], r['status']
                ok = (ps == 0) & (gs == 0)
                if ok.any():
                    du = max(du, float(np.abs(r['u'][ok] - gpu_u[sl][ok]).max()))
                for a, b in zip(gs[gs != ps], ps[gs != ps]):
                    key = f'{int(a)},{int(b)}'
                    mism[key] = mism.get(key, 0) + 1
                n = sl.stop
            done += sl.stop - sl.start
        return done, el, du, mism, n

    threads = cpu_threads()
    d_all, e_all, du, mism, n = leg(threads, 0.75 * budget_s, True)
    d_one, e_one, _, _, _ = leg(1, 0.25 * budget_s, False)
    base = {'value': d_all / e_all, 'unit': 'QP solves/s', 'cores': threads, 'kind': 'port',
            'sample': f'{d_all} solves = {d_all / B:.2f} passes over the {B}-instance rank-0 shard in '
                      f'{e_all:.1f} s on {threads} threads (this process\'s CPU share; the host reports '
                      f'os.cpu_count() = {os.cpu_count()}); C restatement of the reference '
                      f'gen_dt_dynamics/build_qp + exact dense dual active-set solve '
                      f'(oracle/hmpc_port.c, OpenMP)',
            'one_core': {'value': d_one / e_one, 'cores': 1,
                         'sample': f'{d_one} solves in {e_one:.1f} s, 1 thread'},
            'host_cpu_count': os.cpu_count()}
    parity = {'instances': n, 'max_abs_du_vs_port': du,
              'status_mismatch': mism, 'status_mismatch_total': int(sum(mism.values())),
              'note': 'max_abs_du over instances both solve; status_mismatch keys are '
                      '"gpu_status,port_status" (0 solved, 1 max_iter, 2 primal_infeasible, 3 numerical)'}
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
    backend = None
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)
        backend = dist.get_backend()
        assert dist.get_world_size() == world, (dist.get_world_size(), world)

    import hmpc
    import hmpc_dist
    import hmpc_plan

    N = args.N
    if args.global_batch:
        start, B = hmpc_dist.strong_shard(args.global_batch, world, rank)
    else:
        B = args.batch
        start = hmpc_dist.shard_start(rank, B)
    inst = hmpc_plan.sample_instances(B, N, curve=not args.straight, seed=args.seed,
                                      mu_sweep=(0.3, 1.2) if args.mu_sweep else None, start=start)
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).to(dev)
         for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    c = hmpc_plan.runner_constants()
    ctx = hmpc.Context(args.variant, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'],
                       rh=c['rh'], device=local, precision=args.precision)
    if args.precision == 'f32_refined':
        ctx.set_refinement(args.refine)
    ctx.set_order(args.order)
    out = dict(u=torch.empty((B, N, 6), dtype=torch.float64, device=dev),
               x=torch.empty((B, N + 1, 12), dtype=torch.float64, device=dev),
               obj=torch.empty(B, dtype=torch.float64, device=dev),
               status=torch.empty(B, dtype=torch.int32, device=dev),
               iters=torch.empty(B, dtype=torch.int32, device=dev),
               active=torch.empty(B, dtype=torch.int32, device=dev))   # final active-set sizes
    stream = torch.cuda.current_stream(dev)
    # N > 1: the exchange step (per-instance cost + status) is one
    # all-gather of a packed [obj | status] slot on a side stream, pipelined
    # with the next step's solve (double-buffered slots, hmpc_dist)
    counts = [hmpc_dist.strong_shard(args.global_batch, world, r)[1] for r in range(world)] \
        if args.global_batch else None
    ex = hmpc_dist.ResultExchange(B, dev, counts=counts) if world > 1 else None
    last = [out]

    def step():
        o = out
        if ex is not None:
            ob, sb = ex.outputs()
            o = dict(out, obj=ob, status=sb)
        ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'],
                         out=o, stream=stream.cuda_stream)
        if ex is not None:
            ex.exchange()
        last[0] = o

    # untimed pre-warm (solves only: no collective, so a rank-local duration
    # cannot unbalance the ranks' exchange calls)
    pw_steps, t_pw = 0, time.perf_counter()
    while (time.perf_counter() - t_pw) * 1e3 < args.prewarm_ms:
        for _ in range(4):
            ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'],
                             out=out, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        pw_steps += 4
    prewarm_ms = (time.perf_counter() - t_pw) * 1e3
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    kernel = ctx.kernel_name   # (the classes this batch's solves ran)
    ovf0 = ctx.overflow_total   # instances the overflow pass re-solved so far
    # one HIP event pair on the launch stream around the K timed steps (a
    # timing event pair per step put ~11 us of marker packets between the
    # steps of a 0.14 ms configs[1] solve: tools/host_probe.py)
    evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k in range(args.steps):
        step()
    evs[1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # solve time per step on the launch stream (hmpc_solve_batch: classify,
    # the class kernels, the overflow pass), averaged over the timed steps
    kern_ms = evs[0].elapsed_time(evs[1]) / args.steps
    tt = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el, kern_ms_max = float(tt[0]), float(tt[1])

    ovf_step = (ctx.overflow_total - ovf0) / args.steps
    st = last[0]['status'].cpu().numpy()
    it = out['iters'].cpu().numpy()
    act = out['active'].cpu().numpy()
    solved_local = float((st == 0).mean())
    sf = torch.tensor([solved_local], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(sf, op=dist.ReduceOp.MIN)
    dist_info = None
    if world > 1:
        ex.wait()
        torch.cuda.synchronize(dev)
        if backend == 'nccl':
            # the RCCL path is the one taken: one all_gather_into_tensor per step
            assert ex.calls['all_gather_into_tensor'] == args.warmup + args.steps, ex.calls
            assert ex.calls['all_gather_list'] == 0, ex.calls
        dist_info = {'world_size': dist.get_world_size(), 'backend': backend,
                     'exchange_calls': ex.calls, 'exchange_bytes_per_rank_per_step': ex.slot}

    base = parity = None
    if rank == 0 and world == 1:
        base, parity = cpu_baseline(args, inst, out['u'].cpu().numpy(), st, args.cpu_seconds)

    if rank == 0:
        bpsolve = algorithmic_bytes(N)
        achieved = bpsolve * B / (kern_ms * 1e-3) / 1e9
        iters_mean = float(it.mean())
        q_mean = float(act.mean())   # the kernels' reported final active-set sizes
        flops = algorithmic_flops(kernel, N, iters_mean, q_mean)
        traffic = executed = None
        wl = f'{args.variant}_N{N}_B{B}_{"straight" if args.straight else "curve"}' \
             f'{"_musweep" if args.mu_sweep else ""}' \
             f'{"" if args.precision == "f64" else "_" + args.precision}'
        tpath = os.path.join(ROOT, 'profiles', 'traffic.json')
        tj = json.load(open(tpath)).get(wl, {}) if os.path.exists(tpath) else {}
        valu = None
        if tj.get('kernel') == kernel:
            traffic = tj.get('bytes_per_launch_x2_corrected')
            executed = None if 'float' in kernel else tj.get('fp64_flops_executed_per_solve')
            if tj.get('valu_busy') is not None:
                valu = {'busy': tj['valu_busy'], 'wait_any_frac': tj.get('wait_any_frac'),
                        'valu_insts_per_solve': tj.get('valu_insts_per_solve'),
                        'definition': 'SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs) '
                                      'summed over the step\'s kernels: the fraction of SIMD cycles '
                                      'issuing VALU work while they run',
                        'source': tj.get('source')}
        total = B * world * args.steps
        f32 = 'float' in kernel
        vec_key = 'fp32_vector' if f32 else 'fp64_vector'
        p64, p32, peak_src = measured_peaks()
        vec_meas = p32 if f32 else p64
        vec_spec = FP32_VECTOR_SPEC_TFS if f32 else FP64_VECTOR_SPEC_TFS
        vec_ach = flops * B / (kern_ms * 1e-3) / 1e12
        prec = 'fp32' if f32 else 'fp64'
        rec = {
            'metric': METRIC,
            'value': total / el,
            'unit': 'QP solves/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'prewarm_ms': prewarm_ms, 'prewarm_steps': pw_steps,
            'ms_per_step': el / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'strong' if args.global_batch else 'weak',
            'vs_baseline': None,
            'dtype': {'f32': 'f32', 'f32_generic': 'f32', 'f32_refined': 'f32+f64 refinement'}.get(args.precision,
                                                                                                   'f64'),
            'data': 'synthetic: Runner path_plan_init plan + randomised x0 (SURVEY.md 8d), generated on '
                    'host, resident in HBM before timing',
            'config': {'workload': workload_label(args, world), 'global_batch': B * world
                       if not args.global_batch else args.global_batch, 'per_gpu_batch': B,
                       'horizon': N, 'variant': args.variant,
                       'plan': 'straight' if args.straight else 'curve', 'mu_sweep': args.mu_sweep,
                       'precision': args.precision, 'order': args.order,
                       'parallelism': f'shard{world}'},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'bound_effective': f'{prec}_valu_latency',
                         'limiter': f'not HBM: {prec} VALU issue (valu.busy) and dependent-chain latency of '
                                    'an LDS/register-resident iterative solve (SURVEY 8d, DESIGN 5)',
                         'hbm_note': 'the HBM roofline is unreachable by design: a solve moves '
                                     f'{algorithmic_bytes(N)} B, so 40 % of 8 TB/s would need '
                                     f'{0.4 * HBM_PEAK_GBS * 1e9 / algorithmic_bytes(N) / 1e6:.0f} M solves/s '
                                     '(SURVEY 0.3 / 8d); the frac is reported, not targeted',
                         'traffic_over_algorithmic': traffic / (bpsolve * B) if traffic else None,
                         'kernel': kernel, 'kernel_ms': kern_ms, 'kernel_ms_max_rank': kern_ms_max,
                         'kernel_ms_basis': 'HIP events on the launch stream around the timed steps, / steps',
                         'algorithmic_bytes_per_solve': bpsolve, 'solves_per_launch': B,
                         'traffic_note': 'HBM bytes per launch from profiles/traffic.json (rocprofv3 '
                                         'FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md), null '
                                         'when no profile of this workload and kernel'},
            # the bound that matters for this path: fp64 VALU
            vec_key: {
                'achieved': vec_ach, 'peak': vec_spec, 'peak_source': 'datasheet (MI355X_MICROARCH.md)',
                'unit': 'TFLOP/s', 'frac': vec_ach / vec_spec,
                'peak_measured': vec_meas, 'peak_measured_source': peak_src,
                'frac_measured': vec_ach / vec_meas,
                'flops_per_solve': flops, 'basis': 'algorithmic (bench.algorithmic_flops, DESIGN.md 5) at the '
                                                    'measured iters_mean and active_mean',
                'iters_mean': iters_mean, 'active_mean': q_mean,
                'executed_flops_per_solve': executed,
                'executed_frac': (executed * B / (kern_ms * 1e-3) / 1e12 / vec_spec) if executed else None},
            'valu': valu,
            'cpu_baseline': base,
            'solved_frac_min_rank': float(sf[0]),
            'iters_mean': iters_mean, 'iters_max': int(it.max()),
            'active_mean': q_mean, 'active_max': int(act.max()),
            # the slow fp64 pass (hmpc_overflow_total): active sets beyond the
            # main pass's capacity; for f32_refined also the fp64-check and
            # convergence fallbacks
            'overflow_pass': {'instances_per_step': ovf_step, 'frac': ovf_step / B},
            'parity_sample': parity,
            'dist': dist_info,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == '__main__':
    main()
