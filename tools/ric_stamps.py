"""Per-phase cycle breakdown of the Riccati kernel (diagnostic build).

Build:  OUT=libhmpc_stamps.so BDIR=build_stamps HORIZONS=10 \\
        hopper-mpc-inertial_amd/build.sh -DHMPC_STAMPS
Run:    HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so \\
        python tools/ric_stamps.py variant N B [mu] [curve]
The stamped kernel writes accumulated s_memtime cycles over each instance's
x* row (slots in hmpc_ric.hip: RS_ACC).  Add -DHMPC_RIC_GROUPS_PER_CU=4 to the
build to run the persistent grid at one workgroup per SIMD (round 4: 378 k vs
410 k cycles per N = 20 instance at one vs two waves per SIMD).  Horizons
above 24 factorise in a kernel of their own (ric_factor_kernel), whose phase
is not stamped.
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

NAMES = ['load_dynamics', 'gradient', 'riccati_factor', 'unconstrained', 'gi_scan', 'gi_s_hinv',
         'gi_c_y_r', 'gi_z_hinv', 'gi_step_add_drop', 'outputs', 'total', 'fac_a_T_M1', 'fac_b_G_F',
         'fac_c_chol_K', 'fac_d_Ginv_P']


def main():
    var, N, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    flags = sys.argv[4:]
    inst = hmpc_plan.sample_instances(B, N, curve='curve' in flags, seed=2024,
                                      mu_sweep=(0.3, 1.2) if 'mu' in flags else None)
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda()
         for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}
    c = ho.runner_constants()
    ctx = hmpc.Context(var, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                       precision='f64_riccati')
    for _ in range(3):
        out = ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    torch.cuda.synchronize()
    raw = out['x'].view(torch.int64).reshape(B, -1)[:, :16].cpu().numpy()
    st = raw[:, :len(NAMES)].astype(np.float64)
    names = NAMES if N <= 24 else NAMES[:11] + ['count_s_sweep_pairs', 'count_mrhs_cache_hits',
                                                 'count_z_fallback_sweeps', 'count_rhs_in_sweep_pairs']
    res = {n: float(st[:, i].mean()) for i, n in enumerate(names)}
    if N > 24:   # the factorisation kernel ran separately: slots 11-14 are event counts
        res['count_z_fallback_sweeps_max'] = float(st[:, 13].max())
    res['count_drops'] = float((raw[:, 15] >> 32).mean())
    res['count_columns_shifted'] = float((raw[:, 15] & 0xffffffff).mean())
    res['iters_mean'] = float(out['iters'].float().mean())
    res['config'] = f'{var} N={N} B={B} {" ".join(flags)}'
    print(json.dumps(res))


if __name__ == '__main__':
    main()
