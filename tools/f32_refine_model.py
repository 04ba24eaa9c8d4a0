"""configs[4]: can fp32 factors + fp64 iterative refinement meet the 1e-6
tolerance faster than the fp64 kernel?  

Numerical half of the answer, on the CPU: for sampled configs[2] instances
(3f, N = 10, --curve), condense the reference-built QP (oracle/hmpc_oracle
build_qp; the same condensed problem the dense kernel factors: H over the
free inputs), take the optimal active set A (exact solve), and run the
range-space refinement a fp32 kernel would run on its own final active set:

    start  u0 = the fp32 solution (every operation in float32: H = L L'
           and S = N_A' H^-1 N_A = R'R factored in float32)
    iterate  r1 = -(H u + h) + N_A lam,  r2 = b_A - N_A' u       (float64)
             dlam = S^-1 (r2 - N_A' H^-1 r1),  du = H^-1 (r1 + N_A dlam)
                                                    (float32 factors)
until max|u - u*| <= 1e-6.  Reports the error after each iteration and the
iterations each instance needs (the contraction rate).  The GPU half (what one
iteration costs against the fp64 kernel) is in DESIGN.md section 5 next to
the measured fp32 / fp64 throughput.

    python tools/f32_refine_model.py [B]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import hmpc_plan  # noqa: E402
from oracle import hmpc_oracle as ho  # noqa: E402


def condensed(p, inst, i):
    """H, h, Nrows (G, lo, hi over the free inputs), free index list, the
    exact u* and its active rows."""
    N = p.N
    Ad, Bd = ho.gen_dt_dynamics(p, inst['x_lin'][i], inst['pf'][i])
    _, _, Gd = ho.constant_matrices(p)
    C = inst['C'][i]
    qp = ho.build_qp(p, inst['x_in'][i], inst['x_ref'][i], Ad, Bd, Gd, C)
    nxz = (N + 1) * 12
    free = [6 * k + c for k in range(N) for c in range(6)
            if not ((c < 3 and C[k] == 0) or (p.variant == '2f' and c == 1))]
    u0 = np.zeros((N, 6))
    x0 = ho.rollout(p, inst['x_in'][i], u0, Ad, Bd, Gd)
    z0 = np.concatenate([x0.ravel(), u0.ravel()])
    T = np.zeros((len(z0), len(free)))
    for j, f in enumerate(free):
        u = np.zeros(N * 6)
        u[f] = 1.0
        x = ho.rollout(p, inst['x_in'][i], u.reshape(N, 6), Ad, Bd, Gd)
        T[:nxz, j] = x.ravel() - x0.ravel()
        T[nxz + f, j] = 1.0
    H = T.T @ qp['P'] @ T
    h = T.T @ (qp['P'] @ z0 + qp['q'])
    ineq = qp['l'] != qp['u']
    G = qp['A'][ineq] @ T
    off = qp['A'][ineq] @ z0
    lo, hi = qp['l'][ineq] - off, qp['u'][ineq] - off
    ref = ho.solve_instance(p, inst['x_in'][i], inst['x_lin'][i], inst['x_ref'][i], inst['pf'][i], C)
    ustar = ref['u'].ravel()[free]
    g = G @ ustar
    # active rows as n'u = b with the sign that makes them >= rows
    act_lo = np.isfinite(lo) & (np.abs(g - lo) < 1e-7)
    act_hi = np.isfinite(hi) & (np.abs(g - hi) < 1e-7)
    NA = np.vstack([G[act_lo], -G[act_hi]]).T
    bA = np.concatenate([lo[act_lo], -hi[act_hi]])
    return H, h, NA, bA, ustar


def f32_solve_setup(H, NA):
    L = np.linalg.cholesky(H.astype(np.float32))
    def hinv(v):   # float32 triangular solves
        y = np.linalg.solve(L, v.astype(np.float32))
        return np.linalg.solve(L.T, y).astype(np.float32)
    if NA.shape[1]:
        HN = np.stack([hinv(NA[:, j]) for j in range(NA.shape[1])], axis=1)
        S = (NA.astype(np.float32).T @ HN).astype(np.float32)
        R = np.linalg.cholesky(S)
        def sinv(v):
            y = np.linalg.solve(R, v.astype(np.float32))
            return np.linalg.solve(R.T, y).astype(np.float32)
    else:
        sinv = None
    return hinv, sinv


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    p = ho.MpcParams.runner('3f', 10)
    inst = hmpc_plan.sample_instances(B, 10, curve=True, seed=2024)
    hist, need = [], []
    for i in range(B):
        H, h, NA, bA, ustar = condensed(p, inst, i)
        hinv, sinv = f32_solve_setup(H, NA)
        q = NA.shape[1]
        NA32 = NA.astype(np.float32)
        # the fp32 solve itself (range-space EQP on the optimal active set,
        # every operation in float32)
        r1 = (-h).astype(np.float32)
        if q:
            lam = sinv(bA.astype(np.float32) - NA32.T @ hinv(r1))
            u = hinv(r1 + NA32 @ lam).astype(np.float64)
            lam = lam.astype(np.float64)
        else:
            u, lam = hinv(r1).astype(np.float64), np.zeros(0)
        errs = [float(np.abs(u - ustar).max())]
        for it in range(12):
            r1 = -(H @ u + h) + (NA @ lam if q else 0.0)          # float64 residuals
            if q:
                r2 = bA - NA.T @ u
                dlam = sinv(r2 - NA32.T @ hinv(r1)).astype(np.float64)
                du = hinv(r1 + NA @ dlam).astype(np.float64)
                lam = lam + dlam
            else:
                du = hinv(r1).astype(np.float64)
            u = u + du
            errs.append(float(np.abs(u - ustar).max()))
        hist.append(errs)
        ok = [k for k, e in enumerate(errs) if e <= 1e-6]
        need.append(ok[0] if ok else None)
    hist = np.array(hist)
    res = {
        'instances': B,
        'workload': 'configs[2] instances (3f, N=10, --curve), condensed over the free inputs, optimal active set',
        'fp32_solution_max_abs_du': float(hist[:, 0].max()),
        'median_abs_du_by_iteration': [float(np.median(hist[:, k])) for k in range(hist.shape[1])],
        'max_abs_du_by_iteration': [float(hist[:, k].max()) for k in range(hist.shape[1])],
        'iterations_to_1e-6': {'max': max((n for n in need if n is not None), default=None),
                               'median': float(np.median([n for n in need if n is not None])),
                               'never': int(sum(n is None for n in need))},
    }
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
