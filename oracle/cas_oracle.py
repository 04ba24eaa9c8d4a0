"""TEST INFRASTRUCTURE ONLY -- the reference's CasADi variant restated.

``src/mpc_cas_euler_3f.py`` builds its QP once symbolically (``:14-110``) and
solves it with qpOASES per call (``:112-152``).  casadi and qpOASES are absent
here, so this module restates *what the reference constructs* -- bugs
included -- in numpy, and solves it exactly:

* second-order discretisation ``M = I + A_bar t + 1/2 t^2 A_bar^2`` of the
  augmented [A B G] system (``:44-50``), yaw of ``x_in`` for every stage
  (``:139``), the foot vector fixed at rf = [0, 0, -0.2] (``:39-41``; the
  ``rf`` argument of ``mpcontrol`` is unused);
* cost sum_{k<N} |x_k - x_ref_k|^2 + 0.01 |u_k - 2 m g 1|^2 (``:58-70``: the
  scalar u_ref is subtracted from all six inputs, x_N is not costed);
* constraint rows g = [x_0 - x_in; x_{k+1} - (Ad x_k + Bd u_k + Gd);
  fx1; fx2; fy1; fy2] (``:61-85``) where fy1 / fy2 are fx1 followed by ONE
  y row of the last stage (``:75-76`` re-read constr_fricx1); bounds
  lbg = 0 on the first N + 1 rows only and -1e10 elsewhere, ubg = 0 (``:97-99``):
  the initial condition is an equality only for its first N + 1 components
  and every dynamics row is one-sided;
* input bounds fx, fy in [-200 C, 200 C], fz in [0, 400 C] (``:121-134``),
  torques and states free (+-1e10).

z = [vec(x) (column-major, x is 12 x (N+1)); vec(u)] as in ``:87``.

The QP leaves x_N uncosted and only bounded above by its one-sided dynamics
row, so the solution set is a ray in x_N.  u* and x_{<N} are unique (the
rest of the Hessian is diagonal positive).  ``solve`` drops x_N and its
rows, solves the rest exactly with ``qp_exact`` and reports x_N on its
dynamics bound (exact primal active-set method, oracle/qp_primal.py).
qpOASES's own answer is not reproducible here:
parity for this variant is unpinned against qpOASES; the problem data is
pinned to the reference's own construction (tests/golden/cas_N10.npz,
recorded through a casadi stub, tests/golden/_stubs/casadi).
"""
from __future__ import annotations

import numpy as np

from oracle import qp_exact, qp_primal  # noqa: F401

BIG = 1e10


def rz(psi):
    """src/utils.py:46-51"""
    c, s = np.cos(psi), np.sin(psi)
    return np.array([[c, s, 0.0], [-s, c, 0.0], [0.0, 0.0, 1.0]])


def hat(w):
    """src/utils.py:21-25"""
    return np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])


def discretise(t, m, g, Jinv, rh, psi):
    """Ad, Bd, Gd of src/mpc_cas_euler_3f.py:25-50 for the yaw psi."""
    n_x, n_u = 12, 6
    R = rz(psi)
    A = np.zeros((n_x, n_x))
    A[0:3, 6:9] = np.eye(3)
    A[3:6, 9:] = R
    B = np.zeros((n_x, n_u))
    B[6:9, 0:3] = np.eye(3) / m
    Jw = R @ Jinv @ R.T
    rf = np.array([0.0, 0.0, -0.2])
    B[9:12, 0:3] = Jw @ hat(rh + rf)
    B[9:12, 3:] = Jw @ R.T
    G = np.zeros((n_x, 1))
    G[8] = -g
    Ab = np.hstack([np.hstack([A, B]), G])
    Ab = np.vstack([Ab, np.zeros((n_u + 1, n_x + n_u + 1))])
    M = np.eye(n_x + n_u + 1) + Ab * t + 0.5 * (t ** 2) * Ab @ Ab
    return M[0:n_x, 0:n_x], M[0:n_x, n_x:n_x + n_u], M[0:n_x, -1]


def build_qp(t, N, m, g, mu, Jinv, rh, x_in, x_ref_in, C):
    """The QP data the reference hands qpOASES for mpcontrol(x_in, x_ref_in,
    rf, C): dict(P, q, r, A, g0, lbg, ubg, lbx, ubx), g(z) = A z + g0."""
    n_x, n_u = 12, 6
    nX, n = n_x * (N + 1), n_x * (N + 1) + n_u * N
    Ad, Bd, Gd = discretise(t, m, g, Jinv, rh, x_in[5])
    xi = lambda k, i: n_x * k + i          # noqa: E731
    ui = lambda k, c: nX + n_u * k + c      # noqa: E731
    P = np.zeros((n, n))
    q = np.zeros(n)
    r = 0.0
    ur = m * g * 2
    for k in range(N):
        for i in range(n_x):
            P[xi(k, i), xi(k, i)] = 2.0
            q[xi(k, i)] = -2.0 * x_ref_in[k, i]
            r += x_ref_in[k, i] ** 2
        for c in range(n_u):
            P[ui(k, c), ui(k, c)] = 0.02
            q[ui(k, c)] = -0.02 * ur
            r += 0.01 * ur * ur
    rows, g0 = [], []

    def row():
        rows.append(np.zeros(n))
        g0.append(0.0)
        return rows[-1]

    for i in range(n_x):                     # x_0 - x_in
        a = row()
        a[xi(0, i)] = 1.0
        g0[-1] = -x_in[i]
    for k in range(N):                       # x_{k+1} - (Ad x_k + Bd u_k + Gd)
        for i in range(n_x):
            a = row()
            a[xi(k + 1, i)] += 1.0
            for j in range(n_x):
                a[xi(k, j)] -= Ad[i, j]
            for c in range(n_u):
                a[ui(k, c)] -= Bd[i, c]
            g0[-1] = -Gd[i]
    fx1 = [(k, 0, 1.0) for k in range(N)]
    fx2 = [(k, 0, -1.0) for k in range(N)]
    fy1 = fx1 + [(N - 1, 1, 1.0)]            # :75 re-reads constr_fricx1
    fy2 = fx1 + [(N - 1, 1, -1.0)]           # :76
    for blk in (fx1, fx2, fy1, fy2):
        for k, c, sgn in blk:
            a = row()
            a[ui(k, c)] = sgn
            a[ui(k, 2)] = -mu
    A = np.array(rows)
    nc = A.shape[0]
    lbg = np.full(nc, -BIG)
    lbg[0:N + 1] = 0.0
    ubg = np.zeros(nc)
    lbx = np.full(n, -BIG)
    ubx = np.full(n, BIG)
    C = np.asarray(C, dtype=np.float64)
    ubx[nX + 0::n_u] = 200 * C
    ubx[nX + 1::n_u] = 200 * C
    lbx[nX + 0::n_u] = -200 * C
    lbx[nX + 1::n_u] = -200 * C
    ubx[nX + 2::n_u] = 400 * C
    lbx[nX + 2::n_u] = 0.0
    return dict(P=P, q=q, r=r, A=A, g0=np.array(g0), lbg=lbg, ubg=ubg, lbx=lbx, ubx=ubx,
                Ad=Ad, Bd=Bd, Gd=Gd, x_in=np.array(x_in, dtype=np.float64))


def solve(qp, N):
    """Exact solve of a recorded / restated CasADi QP: x_N and the rows that
    touch it dropped (its solution set is a ray), the rest by qp_exact.
    Returns dict(z, u (N,6), x (N+1,12), status, obj)."""
    n_x, n_u = 12, 6
    nX = n_x * (N + 1)
    n = nX + n_u * N
    keep = np.ones(n, bool)
    keep[n_x * N:nX] = False
    A = qp['A']
    rows = ~np.any(A[:, ~keep] != 0.0, axis=1)
    inf = lambda v: np.where(v >= BIG, np.inf, np.where(v <= -BIG, -np.inf, v))   # noqa: E731
    Ar = np.vstack([A[rows][:, keep], np.eye(int(keep.sum()))])
    lo = np.concatenate([inf(qp['lbg'][rows]) - qp['g0'][rows], inf(qp['lbx'][keep])])
    hi = np.concatenate([inf(qp['ubg'][rows]) - qp['g0'][rows], inf(qp['ubx'][keep])])
    free_rows = np.isinf(lo) & np.isinf(hi)
    Ar, lo, hi = Ar[~free_rows], lo[~free_rows], hi[~free_rows]
    # fy1 / fy2 repeat the fx1 rows (:75-76): drop exact duplicates (the
    # same constraint twice is degenerate for the polish's KKT system)
    _, first = np.unique(np.hstack([Ar, lo[:, None], hi[:, None]]), axis=0, return_index=True)
    first = np.sort(first)
    Ar, lo, hi = Ar[first], lo[first], hi[first]
    P = qp['P'][np.ix_(keep, keep)]
    q = qp['q'][keep]
    # exact primal active-set solve (qp_primal) from a feasible point: zero
    # inputs and the trajectory simulated through the dynamics rows meet every
    # row (x_0 = x_in, each dynamics row at 0, forces 0 inside their bounds and
    # friction cones).  qp_exact's IPM stalls on this degenerate QP (many
    # one-sided dynamics rows active together) about once in six.
    z0 = None
    if 'Ad' in qp and 'x_in' in qp:
        xs = np.zeros((N + 1, n_x))
        xs[0] = qp['x_in']
        for k in range(N):
            xs[k + 1] = qp['Ad'] @ xs[k] + qp['Gd']
        z0 = np.concatenate([xs.ravel(), np.zeros(n_u * N)])[keep]
    res = qp_primal.solve(P, q, Ar, lo, hi, z0=z0)
    if res['x'] is None:
        return dict(z=None, u=None, x=None, status=res['status'], obj=np.nan)
    z = np.zeros(n)
    z[keep] = res['x']
    # x_N on its dynamics bound: the reference's predicted state
    xs = z[:nX].reshape(N + 1, n_x)
    us = z[nX:].reshape(N, n_u)
    if 'Ad' in qp:
        xs[N] = qp['Ad'] @ xs[N - 1] + qp['Bd'] @ us[N - 1] + qp['Gd']
        z[:nX] = xs.ravel()
    obj = 0.5 * z @ qp['P'] @ z + qp['q'] @ z + qp['r']
    return dict(z=z, u=us.copy(), x=xs.copy(), status=res['status'], obj=obj)


def kkt_residual(qp, z, N, act_tol=1e-7):
    """Optimality certificate of a candidate z for the x_N-reduced QP,
    independent of any solver: the active rows and bounds at z, multipliers
    of the right sign from non-negative least squares on the stationarity
    condition P z + q + sum lam_i a_i = 0 (a_i = +n_i at an upper bound, -n_i
    at a lower one, both for an equality).  For a feasible z of this convex
    QP a small residual proves global optimality.  Returns the scaled
    residual max|P z + q + A_act' lam| / (1 + max|q|)."""
    from scipy.optimize import nnls
    n_x = 12
    nX = n_x * (N + 1)
    n = len(z)
    keep = np.ones(n, bool)
    keep[n_x * N:nX] = False
    A = qp['A']
    rows = ~np.any(A[:, ~keep] != 0.0, axis=1)
    cols = []
    g = A @ z + qp['g0']
    for i in np.where(rows)[0]:
        up = g[i] >= qp['ubg'][i] - act_tol
        lo = qp['lbg'][i] > -BIG and g[i] <= qp['lbg'][i] + act_tol
        if up:
            cols.append(A[i, keep])
        if lo:
            cols.append(-A[i, keep])
    kz = np.where(keep)[0]
    for j, v in enumerate(kz):
        e = np.zeros(len(kz))
        e[j] = 1.0
        if qp['ubx'][v] < BIG and z[v] >= qp['ubx'][v] - act_tol:
            cols.append(e)
        if qp['lbx'][v] > -BIG and z[v] <= qp['lbx'][v] + act_tol:
            cols.append(-e)
    grad = qp['P'][np.ix_(keep, keep)] @ z[keep] + qp['q'][keep]
    if not cols:
        return float(np.abs(grad).max()) / (1.0 + float(np.abs(qp['q']).max()))
    Am = np.array(cols).T
    lam, res = nnls(Am, -grad, maxiter=20 * Am.shape[1])
    r = grad + Am @ lam
    return float(np.abs(r).max()) / (1.0 + float(np.abs(qp['q']).max()))
