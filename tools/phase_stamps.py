"""Per-phase cycle breakdown of the solve kernel (diagnostic build).

Build:  OUT=libhmpc_stamps.so BDIR=build_stamps HORIZONS=10 \
        hopper-mpc-inertial_amd/build.sh -DHMPC_STAMPS
Run:    HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so python tools/phase_stamps.py
The stamped kernel writes s_memtime values over each instance's x* row.
PREC=f32 / f32_refined (REFINE=k) stamp the fp32 builds; in the refined
build phase 'outputs' is the refinement (fp64 set-up, k corrections, final
rollout and the fp64 check) and 'refine_corrections' the cycles of the k
corrections alone.  Instances handed to the fp64 overflow pass carry no
stamps and are left out ('stamped' counts the rest).
"""
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

NAMES = ['load', 'gen_dt_dynamics', 'uniform_sweeps', 'hessian_rows', 'cholesky', 'unconstrained',
         'active_set', 'outputs']


def main():
    N = int(os.environ.get('N', '10'))
    B = int(os.environ.get('B', '65536'))
    var = os.environ.get('VARIANT', '3f')
    curve = os.environ.get('STRAIGHT', '0') != '1'
    inst = hmpc_plan.sample_instances(B, N, curve=curve, seed=2024)
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda()
         for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    c = ho.runner_constants()
    prec = os.environ.get('PREC', 'f64')
    ctx = hmpc.Context(var, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                       precision=prec)
    nref = int(os.environ.get('REFINE', '5'))
    if prec == 'f32_refined':
        ctx.set_refinement(nref)
    for _ in range(3):
        out = ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    torch.cuda.synchronize()
    st = out['x'].view(torch.int64).reshape(B, -1)[:, :len(NAMES) + 1].cpu().numpy()
    dur = np.diff(st, axis=1)
    tot = st[:, len(NAMES)] - st[:, 0]
    acc = out['x'].view(torch.int64).reshape(B, -1)[:, 9:15].cpu().numpy()
    it = out['iters'].float().cpu().numpy()
    ref_cyc = out['x'].view(torch.int64).reshape(B, -1)[:, 15].cpu().numpy()
    stamped = (st[:, 0] > 0) & (dur >= 0).all(axis=1) & (tot < 10**8)

    def summary(m):
        m = m & stamped
        if not m.any():
            return {'instances': 0}
        res = {n: float(dur[m, i].mean()) for i, n in enumerate(NAMES)}
        res['total_mean'] = float(tot[m].mean())
        res['total_p50'] = float(np.median(tot[m]))
        res['total_max'] = float(tot[m].max())
        res['iters_mean'] = float(it[m].mean())
        res['instances'] = int(m.sum())
        # accumulated active-set sub-phases (slots 9..14 of the stamped build)
        for i, n in enumerate(['gi_scan', 'gi_fwd_sweep', 'gi_gram_schmidt', 'gi_bwd_sweep',
                               'gi_dual_step', 'gi_add_drop']):
            res[n] = float(acc[m, i].mean())
        if prec == 'f32_refined':
            res['refine_corrections'] = float(ref_cyc[m].mean())
            res['refine_per_correction'] = float(ref_cyc[m].mean()) / max(nref, 1)
        return res

    # by class of the dense split launch: free variables nf = 3N + k * stance
    nst = (inst['C'] != 0).sum(axis=1)
    nf = 3 * N + (3 if var == '3f' else 2) * nst
    cmp_nv = int(os.environ.get('CMP_NV', '48'))
    # (round 5: the all-swing windows run two per wave in hmpc_swing.hip --
    # a pair shares its stamps, so its cycles are per wave = per 2 instances)
    sw = (nst == 0) if prec == 'f64' else np.zeros(B, bool)   # (no swing class in the fp32 builds)
    res = {'precision': prec, 'stamped': int(stamped.sum()), 'B': B,
           'all': summary(np.ones(B, bool)), 'swing_pair_per_wave': summary(sw),
           'compacted': summary((nf <= cmp_nv) & ~sw), 'full': summary(nf > cmp_nv)}
    for s_ in np.unique(nst):
        res[f'stance{int(s_)}_nf{int(3 * N + (3 if var == "3f" else 2) * s_)}'] = summary(nst == s_)
    # the slowest instances (the small-batch step is as long as its slowest one)
    p99 = np.quantile(tot[stamped], 0.99) if stamped.any() else 0
    res['slowest_1pct'] = summary(tot >= p99)
    res['slowest_1pct']['nst_mean'] = float(nst[(tot >= p99) & stamped].mean()) if stamped.any() else 0.0
    # per-instance latency quantiles (s_memtime runs per XCD, so start times
    # of different instances are not comparable; latencies are)
    q = [0.0, 0.5, 0.9, 0.99, 1.0]
    res['latency_quantiles'] = {'q': q, 'cycles': [float(np.quantile(tot[stamped], x)) for x in q]}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
