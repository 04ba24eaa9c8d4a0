"""TEST INFRASTRUCTURE ONLY -- exact fp64 solve of a strictly convex QP by a
PRIMAL active-set method.

    minimise 1/2 z'Pz + q'z      s.t.   l <= A z <= u      (P positive definite)

The CasADi variant's QP (oracle/cas_oracle.py, ``src/mpc_cas_euler_3f.py``)
is degenerate for an interior-point method: most of its one-sided dynamics
rows, the fx rows repeated inside fy1 / fy2 and the force bounds are active
together at the optimum (median 70 rows), so ``qp_exact``'s IPM stalls or
overflows (lambda / s) on about one in six instances.  A primal active-set
method does not see that degeneracy: it walks from a feasible point along
exact equality-constrained steps, keeping its working set linearly
independent by construction (a blocking row of a nonzero step is never in
the span of the working set), and stops where the multipliers of the working
set are non-negative.  That is the exact optimum, certified by
``qp_exact.certificate``.

This is independent of the GPU kernel (hmpc_cas.hip), which runs a DUAL
(Goldfarb-Idnani, range-space) active-set method from the unconstrained
optimum: different iterates, different working sets, same optimum.

Feasible start: the caller's (cas_oracle: zero inputs and the simulated
trajectory, which meets every row of that QP), else HiGHS's least-violation
LP point (``qp_exact.min_violation``), whose certificate is then the only
ground for reporting primal infeasibility.
"""
from __future__ import annotations

import numpy as np

from oracle import qp_exact


def solve(P, q, A, l, u, z0=None, tol=1e-9, max_iter=2000):
    """Returns dict(x, y, status, cert, iters, n_active) like qp_exact.solve.
    z0: a feasible starting point (else HiGHS's least-violation LP point)."""
    P = np.asarray(P, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64)
    A = np.asarray(A, dtype=np.float64)
    l = np.asarray(l, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    n = P.shape[0]
    E, e, G, g, src = qp_exact._split(A, l, u)
    me = E.shape[0]
    if z0 is not None:
        z = np.array(z0, dtype=np.float64)
    else:
        t, z = qp_exact.min_violation(A, l, u)
        if z is None or not np.isfinite(t) or t > 1e-7:
            st = 'primal_infeasible' if (np.isfinite(t) and t > 1e-7) else 'failed'
            return dict(x=None, y=None, status=st, cert=None, iters=0, min_violation=t)
    scale = 1.0 + max(np.abs(g).max(initial=0.0), np.abs(e).max(initial=0.0))
    # starting working set: the rows tight at the start point, greedily kept
    # linearly independent of the equalities and each other (QR residual)
    W = []
    basis = np.zeros((0, n))
    if me:
        Q, _ = np.linalg.qr(E.T)
        basis = Q.T
    slack = g - G @ z
    for i in np.argsort(slack):
        if slack[i] > 1e-9 * scale:
            break
        r = G[i] - basis.T @ (basis @ G[i])
        nr = np.linalg.norm(r)
        if nr > 1e-8 * np.linalg.norm(G[i]):
            basis = np.vstack([basis, r / nr])
            W.append(int(i))
    it = 0
    zero_steps = 0
    mu = np.zeros(0)
    for it in range(1, max_iter + 1):
        AW = np.vstack([E, G[W]]) if W else E
        m = AW.shape[0]
        K = np.zeros((n + m, n + m))
        K[:n, :n] = P
        K[:n, n:] = AW.T
        K[n:, :n] = AW
        rhs = np.concatenate([-(P @ z + q), np.zeros(m)])
        sol = np.linalg.solve(K, rhs)
        p, mu = sol[:n], sol[n:]
        if np.abs(p).max(initial=0.0) <= 1e-13 * (1.0 + np.abs(z).max(initial=0.0)):
            lam = mu[me:]
            if lam.size == 0 or lam.min() >= -tol:
                break
            # drop the most negative multiplier (Bland's smallest index after
            # a run of zero steps: no cycling on degenerate vertices)
            neg = np.where(lam < -tol)[0]
            k = neg[np.argmin([W[j] for j in neg])] if zero_steps > 50 else int(np.argmin(lam))
            W.pop(int(k))
            continue
        Gp = G @ p
        slack = g - G @ z
        cand = [(max(slack[i], 0.0) / Gp[i], i) for i in range(G.shape[0])
                if i not in W and Gp[i] > 1e-14 * (1.0 + np.abs(G[i]).max())]
        alpha, block = 1.0, None
        for a_i, i in cand:
            if a_i < alpha or (a_i == alpha and block is not None and i < block):
                alpha, block = a_i, i
        z = z + alpha * p
        zero_steps = zero_steps + 1 if alpha == 0.0 else 0
        if block is not None and alpha < 1.0:
            W.append(int(block))
    else:
        return dict(x=None, y=None, status='failed', cert=None, iters=it)
    y = mu[:me]
    lam = np.zeros(G.shape[0])
    lam[W] = mu[me:]
    cert = qp_exact.certificate(P, q, E, e, G, g, z, y, lam)
    ok = (cert['primal_eq'] < tol and cert['primal_ineq'] < tol and cert['dual_neg'] < tol
          and cert['stationarity'] < tol)
    yA = np.zeros(len(l))
    ie = np.where(np.isfinite(l) & np.isfinite(u) & (l == u))[0]
    yA[ie] = y
    for k, (i, sgn) in enumerate(src):
        yA[i] += sgn * lam[k]
    return dict(x=z, y=yA, status='solved' if ok else 'solved_inaccurate', cert=cert, iters=it,
                n_active=int(np.sum(lam > 1e-9)))
