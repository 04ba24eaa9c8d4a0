"""TEST INFRASTRUCTURE ONLY -- exact fp64 solve of an OSQP-form QP.

    minimise 1/2 z'Pz + q'z      s.t.   l <= A z <= u

Stands in for cvxpy+OSQP (``src/mpc_cvx_euler_3f.py:156-157``), which is not
installed here.  OSQP itself stops ADMM at eps=1e-5 and then *polishes*: it
guesses the active set and solves the reduced KKT system exactly.  This module
reaches the same exact point by a different, independent route from the GPU
kernel (which condenses and runs a dual active-set method):

1. Mehrotra predictor-corrector interior point on the sparse (non-condensed)
   KKT system, run to complementarity ~1e-13;
2. polish: take the active set {lambda_i > s_i}, solve the equality-
   constrained KKT system with iterative refinement, and repair the active
   set (add violated rows / drop negative multipliers) until
3. a KKT certificate holds: primal violation, negative duals and
   stationarity residual all below 1e-9 (scaled).

Status strings: 'solved' (certificate holds), 'solved_inaccurate' (IPM only),
'primal_infeasible' (certified: the LP min_violation -- the least t with
l - t <= A z <= u + t -- is > 1e-7), 'failed' (no convergence, no certificate).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


def _split(A, l, u):
    A = np.asarray(A, dtype=np.float64)
    eq = np.isfinite(l) & np.isfinite(u) & (l == u)
    E, e = A[eq], l[eq]
    G_rows, g = [], []
    src = []          # (row index in A, sign) for each inequality
    for i in np.where(~eq)[0]:
        if np.isfinite(u[i]):
            G_rows.append(A[i]); g.append(u[i]); src.append((i, +1))
        if np.isfinite(l[i]):
            G_rows.append(-A[i]); g.append(-l[i]); src.append((i, -1))
    G = np.array(G_rows).reshape(len(G_rows), A.shape[1])
    return E, np.asarray(e), G, np.asarray(g), src


def _kkt_solve(Hs, E, rhs_x, rhs_e):
    n = Hs.shape[0]
    K = sp.bmat([[Hs, sp.csr_matrix(E).T], [sp.csr_matrix(E), None]], format='csc')
    lu = spla.splu(K)
    sol = lu.solve(np.concatenate([rhs_x, rhs_e]))
    return sol[:n], sol[n:], lu


def ipm(P, q, E, e, G, g, tol=1e-12, max_iter=200):
    n, me, mi = P.shape[0], E.shape[0], G.shape[0]
    Ps = sp.csr_matrix(P)
    Gs = sp.csr_matrix(G)
    # initial point: the equality-constrained optimum (inequalities dropped),
    # slacks max(g - G z, 1), unit multipliers.  (A cold start from z = 0
    # diverges on the Runner's N = 60 run at its last call, where x_in sits
    # ~1 m above the plan.)
    try:
        z, y, _ = _kkt_solve((Ps + 1e-9 * sp.eye(n)).tocsc(), E, -q, e)
    except RuntimeError:
        z, y = np.zeros(n), np.zeros(me)
    if not np.all(np.isfinite(z)):
        z, y = np.zeros(n), np.zeros(me)
    s = np.maximum(g - Gs @ z, 1.0)
    lam = np.ones(mi)
    for it in range(max_iter):
        rd = Ps @ z + q + E.T @ y + Gs.T @ lam
        re = E @ z - e
        ri = Gs @ z + s - g
        mu = (s @ lam) / max(mi, 1)
        scale = 1.0 + max(np.abs(q).max(initial=0), np.abs(g).max(initial=0), np.abs(e).max(initial=0))
        if (np.abs(rd).max(initial=0) < tol * scale and np.abs(re).max(initial=0) < tol * scale
                and np.abs(ri).max(initial=0) < tol * scale and mu < tol * 1e-2):
            return z, y, s, lam, 'solved', it
        D = lam / s
        H = (Ps + Gs.T @ sp.diags(D) @ Gs).tocsc()
        K = sp.bmat([[H, sp.csr_matrix(E).T], [sp.csr_matrix(E), None]], format='csc')
        try:
            with np.errstate(all='ignore'):
                lu = spla.splu(K)
        except RuntimeError:       # singular: iterates diverged (infeasible)
            break
        if not (np.all(np.isfinite(s)) and np.all(np.isfinite(lam)) and s.max() < 1e30):
            break

        def newton(rc):
            # lam o ds + s o dlam = -rc ; ds = -ri - G dz
            rhs_x = -rd - Gs.T @ ((-rc + lam * ri) / s)
            sol = lu.solve(np.concatenate([rhs_x, -re]))
            dz, dy = sol[:n], sol[n:]
            ds = -ri - Gs @ dz
            dlam = (-rc - lam * ds) / s
            return dz, dy, ds, dlam

        def maxstep(v, dv):
            neg = dv < 0
            return min(1.0, np.min(-v[neg] / dv[neg])) if np.any(neg) else 1.0

        with np.errstate(all='ignore'):
            dz, dy, ds, dl = newton(s * lam)
        a_aff = min(maxstep(s, ds), maxstep(lam, dl))
        mu_aff = ((s + a_aff * ds) @ (lam + a_aff * dl)) / max(mi, 1)
        sigma = (mu_aff / mu) ** 3 if mu > 0 else 0.0
        with np.errstate(all='ignore'):
            dz, dy, ds, dl = newton(s * lam + ds * dl - sigma * mu)
        if not (np.all(np.isfinite(dz)) and np.all(np.isfinite(ds))):
            break
        a = min(1.0, 0.995 * min(maxstep(s, ds), maxstep(lam, dl)))
        z += a * dz; y += a * dy; s += a * ds; lam += a * dl
        s = np.maximum(s, 1e-300); lam = np.maximum(lam, 1e-300)
    with np.errstate(all='ignore'):
        rp = max(np.abs(E @ z - e).max(initial=0), np.maximum(Gs @ z - g, 0).max(initial=0))
    bad = not np.isfinite(rp) or rp > 1e-6
    return z, y, s, lam, ('failed' if bad else 'solved_inaccurate'), it


def min_violation(A, l, u):
    """Certificate of (in)feasibility of l <= A z <= u: the LP
    min t  s.t.  l - t <= A z <= u + t,  t >= 0  (scipy HiGHS).  Returns
    (t*, z): t* = 0 (to the LP's tolerance) with a feasible z, or t* > 0 --
    no point violates every row by less than t*, i.e. the QP is primal
    infeasible."""
    from scipy.optimize import linprog
    A = np.asarray(A, dtype=np.float64)
    m, n = A.shape
    rows, rhs = [], []
    fu, fl = np.isfinite(u), np.isfinite(l)
    # A z - t <= u ;  -A z - t <= -l
    Au = np.hstack([A[fu], -np.ones((fu.sum(), 1))])
    Al = np.hstack([-A[fl], -np.ones((fl.sum(), 1))])
    c = np.zeros(n + 1)
    c[-1] = 1.0
    res = linprog(c, A_ub=sp.vstack([sp.csr_matrix(Au), sp.csr_matrix(Al)]),
                  b_ub=np.concatenate([u[fu], -l[fl]]),
                  bounds=[(None, None)] * n + [(0, None)], method='highs')
    if res.status != 0:
        return np.nan, None
    return float(res.x[-1]), res.x[:n]


def _polish(P, q, E, e, G, g, active, refine=6, delta=1e-11):
    """Exact KKT solve with the inequalities in ``active`` held at equality."""
    n = P.shape[0]
    Ea = np.vstack([E, G[active]]) if np.any(active) else E
    ea = np.concatenate([e, g[active]])
    K0 = sp.bmat([[sp.csr_matrix(P), sp.csr_matrix(Ea).T], [sp.csr_matrix(Ea), None]], format='csc')
    Kr = (K0 + sp.diags(np.concatenate([np.full(n, delta), np.full(Ea.shape[0], -delta)]))).tocsc()
    lu = spla.splu(Kr)
    rhs = np.concatenate([-q, ea])
    sol = np.zeros(n + Ea.shape[0])
    for _ in range(refine):
        res = rhs - K0 @ sol
        sol += lu.solve(res)
    z = sol[:n]
    yy = sol[n:]
    y = yy[:E.shape[0]]
    lam = np.zeros(G.shape[0])
    lam[active] = yy[E.shape[0]:]
    return z, y, lam


def certificate(P, q, E, e, G, g, z, y, lam):
    gs = 1.0 + np.abs(q).max(initial=0)
    stat = P @ z + q + E.T @ y + G.T @ lam
    return dict(
        primal_eq=float(np.abs(E @ z - e).max(initial=0)),
        primal_ineq=float(np.maximum(G @ z - g, 0).max(initial=0)),
        dual_neg=float(np.maximum(-lam, 0).max(initial=0)),
        stationarity=float(np.abs(stat).max(initial=0) / gs),
        complementarity=float(np.abs(lam * (G @ z - g)).max(initial=0)),
    )


def solve(P, q, A, l, u, tol=1e-9, max_repair=20):
    """Exact solve.  Returns dict(x, y, status, cert, iters)."""
    P = np.asarray(P, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64)
    l = np.asarray(l, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    E, e, G, g, src = _split(A, l, u)
    z, y, s, lam, st, its = ipm(P, q, E, e, G, g)
    if st == 'failed':
        # no convergence: primal_infeasible only with a certificate
        t, _ = min_violation(A, l, u)
        st = 'primal_infeasible' if (np.isfinite(t) and t > 1e-7) else 'failed'
        return dict(x=None, y=None, status=st, cert=None, iters=its, min_violation=t)
    best = (z, y, lam, certificate(P, q, E, e, G, g, z, y, lam), 'solved_inaccurate')
    active = lam > s
    for rep in range(max_repair):
        zp, yp, lp = _polish(P, q, E, e, G, g, active)
        c = certificate(P, q, E, e, G, g, zp, yp, lp)
        ok = (c['primal_eq'] < tol and c['primal_ineq'] < tol and c['dual_neg'] < tol
              and c['stationarity'] < tol)
        if ok:
            best = (zp, yp, lp, c, 'solved')
            break
        viol = G @ zp - g
        worst_p = np.argmax(np.where(active, -np.inf, viol))
        worst_d = np.argmin(np.where(active, lp, np.inf))
        if not active[worst_p] and viol[worst_p] > tol:
            active[worst_p] = True
        elif active[worst_d] and lp[worst_d] < -tol:
            active[worst_d] = False
        else:
            break
    z, y, lam, cert, status = best
    # map inequality multipliers back onto rows of A (OSQP sign convention:
    # y_i > 0 at an active upper bound, < 0 at an active lower bound)
    yA = np.zeros(len(l))
    ie = np.where(np.isfinite(l) & np.isfinite(u) & (l == u))[0]
    yA[ie] = y
    for k, (i, sgn) in enumerate(src):
        yA[i] += sgn * lam[k]
    nact = int(np.sum(lam > 1e-9))
    return dict(x=z, y=yA, status=status, cert=cert, iters=its, n_active=nact)
