"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's MPC problem.

Never imported by the product path.  Each function cites the reference lines
it restates (paths relative to the upstream repository root).

The standard form produced here is exactly the problem that cvxpy hands to
OSQP for ``Mpc.solve_qp`` (``src/mpc_cvx_euler_3f.py:155-160``):

    minimise  1/2 z'Pz + q'z + r      subject to  l <= A z <= u

with the decision vector laid out row-major as
``z = [x[0,:], ..., x[N,:], u[0,:], ..., u[N-1,:]]``.  Constraint rows are
emitted in the order of the reference's ``constr`` list (``:110-150``); every
relation ``lhs OP rhs`` becomes the row ``lhs - rhs`` with bounds taken from
OP, which is how the recording stub in ``tests/golden`` reads the reference.
"""
from __future__ import annotations

import dataclasses

import numpy as np

NX = 12
NU = 6


# --------------------------------------------------------------------------
# constants -- src/robotrunner.py:37-48,68,76 and src/mpc_cvx_euler_3f.py:12-39
# --------------------------------------------------------------------------
def runner_constants():
    """Physical constants the Runner passes to ``Mpc`` (src/robotrunner.py:37-48)."""
    m = 7.5
    J = np.array([[76148072.89, 70089.52, 2067970.36],
                  [70089.52, 45477183.53, -87045.58],
                  [2067970.36, -87045.58, 76287220.47]]) * (10 ** (-9))
    Jinv = np.linalg.inv(J)
    rh = -np.array([0.02663114, 0.04435752, 6.61082088]) / 1000
    return dict(t=0.02, m=m, g=9.807, mu=1, J=J, Jinv=Jinv, rh=rh)


Q_DIAG = np.array([50., 50., 2., 1., 1., 50., 1., 1., 1., 10., 10., 10.])   # :35
R_DIAG = np.array([0.001, 0.001, 0.001, 0.001, 0.001, 0.001])               # :37
F_MAX = np.array([352, 0, 206])                                              # :20
TAU_MAX = (7.78, 7.78, 4)                                                    # :123-128
Z_MIN = 0.1                                                                  # :129


def rz(phi):
    """src/utils.py:46-51 (transposed yaw rotation)."""
    return np.array([[np.cos(phi), np.sin(phi), 0.0],
                     [-np.sin(phi), np.cos(phi), 0.0],
                     [0.0, 0.0, 1.0]])


def hat(w):
    """src/utils.py:21-25."""
    return np.array([[0, - w[2], w[1]],
                     [w[2], 0, - w[0]],
                     [-w[1], w[0], 0]])


@dataclasses.dataclass
class MpcParams:
    variant: str       # '3f' or '2f'
    N: int
    t: float
    m: float
    g: float
    mu: float
    Jinv: np.ndarray
    rh: np.ndarray

    @classmethod
    def runner(cls, variant='3f', N=10, mu=None):
        c = runner_constants()
        return cls(variant=variant, N=N, t=c['t'], m=c['m'], g=c['g'],
                   mu=c['mu'] if mu is None else mu, Jinv=c['Jinv'], rh=c['rh'])


def constant_matrices(p: MpcParams):
    """A, B, G scratch and Gd of Mpc.__init__ (3f :24-33, 2f :24-32)."""
    A = np.zeros((NX, NX))
    B = np.zeros((NX, NU))
    G = np.zeros(NX)
    A[0:3, 6:9] = np.eye(3)
    if p.variant == '3f':
        B[6:9, 0:3] = np.eye(3) / p.m
    G[8] = -p.g
    Gd = G * p.t
    return A, B, Gd


def gen_dt_dynamics(p: MpcParams, x, pf):
    """Per-stage forward-Euler discretisation.

    3f: src/mpc_cvx_euler_3f.py:71-94; 2f: src/mpc_cvx_euler_2f.py:70-94.
    ``x`` is the (N+1, 12) linearisation trajectory (rows 0..N-1 used),
    ``pf`` the (N, 3) footstep plan.  Returns Ad (N,12,12), Bd (N,12,6).
    """
    A, B, _ = constant_matrices(p)
    dt = p.t
    Ad = np.zeros((p.N, NX, NX))
    Bd = np.zeros((p.N, NX, NU))
    for k in range(p.N):
        rz_phi = rz(x[k, 5])
        rf = p.rh + rz_phi @ (pf[k, :] - x[k, 0:3])
        J_w_inv = rz_phi @ p.Jinv @ rz_phi.T
        A[3:6, 9:] = rz_phi
        if p.variant == '3f':
            rhat = hat(rz_phi.T @ rf)                       # 3f :85
            B[9:12, 0:3] = J_w_inv @ rhat                   # 3f :88
        else:
            rhat = hat(rf)                                  # 2f :84
            B[6:9, 0:3] = rz_phi.T / p.m                    # 2f :87
            B[9:12, 0:3] = J_w_inv @ rz_phi.T @ rhat        # 2f :88
        B[9:12, 3:] = J_w_inv @ rz_phi.T
        Ad[k, :, :] = np.eye(NX) + A * dt
        Bd[k, :, :] = B * dt
    return Ad, Bd


def effective_uref(p: MpcParams, C, k, uref_mode='aliased'):
    """u_ref seen by stage k's cost term.

    The reference mutates ONE ``u_ref`` array inside the stage loop
    (3f :107,131,138) and cvxpy keeps constants by reference, so when the
    problem is canonicalised every stage sees the value written by the LAST
    stage: u_ref[2] = 2mg*C[N-1] ("aliased", the reference-effective
    behaviour).  ``per_stage`` is the intended value
    u_ref[2] = 2mg*C[k].
    """
    u_ref = np.zeros(NU)
    kk = p.N - 1 if uref_mode == 'aliased' else k
    u_ref[2] = p.m * p.g * 2 if C[kk] != 0 else 0
    return u_ref


def _vx(N, k):
    return k * NX


def _vu(N, k):
    return (N + 1) * NX + k * NU


def build_qp(p: MpcParams, x_in, x_ref, Ad, Bd, Gd, C, uref_mode='aliased'):
    """OSQP standard form of ``Mpc.build_qp`` (3f :96-153, 2f :96-151).

    Returns dict(P, q, r, A, l, u) with dense numpy arrays (small N only
    matter here: N=10 gives 192 variables).
    """
    N = p.N
    nz = (N + 1) * NX + N * NU
    P = np.zeros((nz, nz))
    q = np.zeros(nz)
    r = 0.0
    rows, lo, hi = [], [], []

    def row(coefs, lower, upper):
        a = np.zeros(nz)
        for idx, c in coefs:
            a[idx] += c
        rows.append(a)
        lo.append(lower)
        hi.append(upper)

    Q = np.diag(Q_DIAG)
    R = np.diag(R_DIAG)
    inf = np.inf
    mu = p.mu
    for k in range(N):
        kf = 100 if k == N - 1 else 1       # :113
        kuf = 0 if k == N - 1 else 1        # :114
        iz = _vx(N, k) + 2
        iu = _vu(N, k)
        # torque box (:123-128), relation "lhs - rhs OP 0"
        row([(iu + 3, 1.0)], -inf, TAU_MAX[0])
        row([(iu + 3, 1.0)], -TAU_MAX[0], inf)
        row([(iu + 4, 1.0)], -inf, TAU_MAX[1])
        row([(iu + 4, 1.0)], -TAU_MAX[1], inf)
        row([(iu + 5, 1.0)], -inf, TAU_MAX[2])
        row([(iu + 5, 1.0)], -TAU_MAX[2], inf)
        if p.variant == '2f':
            row([(iu + 1, 1.0)], 0.0, 0.0)                  # 2f :129 fy == 0
        row([(iz, 1.0)], Z_MIN, inf)                        # :129 z >= 0.1
        # cost (:132/:139): quad_form(x[k+1]-x_ref[k], Q*kf) + quad_form(u[k]-u_ref, R*kuf)
        Wx = Q * kf
        Wu = R * kuf
        ix1 = _vx(N, k + 1)
        P[ix1:ix1 + NX, ix1:ix1 + NX] += 2 * Wx
        q[ix1:ix1 + NX] += 2 * Wx @ (-x_ref[k, :])
        r += x_ref[k, :] @ Wx @ x_ref[k, :]
        u_ref = effective_uref(p, C, k, uref_mode)
        P[iu:iu + NU, iu:iu + NU] += 2 * Wu
        q[iu:iu + NU] += 2 * Wu @ (-u_ref)
        r += u_ref @ Wu @ u_ref
        # dynamics x[k+1] == Ak x[k] + Bk u[k] + Gd  (:133/:140)
        ix0 = _vx(N, k)
        for i in range(NX):
            coefs = [(ix1 + i, 1.0)]
            coefs += [(ix0 + j, -Ad[k, i, j]) for j in range(NX) if Ad[k, i, j] != 0]
            coefs += [(iu + j, -Bd[k, i, j]) for j in range(NU) if Bd[k, i, j] != 0]
            row(coefs, Gd[i], Gd[i])
        if C[k] == 0:
            if p.variant == '3f':                           # 3f :134-136
                row([(iu + 0, 1.0)], 0.0, 0.0)
                row([(iu + 1, 1.0)], 0.0, 0.0)
                row([(iu + 2, 1.0)], 0.0, 0.0)
            else:                                           # 2f :135-136
                row([(iu + 0, 1.0)], 0.0, 0.0)
                row([(iu + 2, 1.0)], 0.0, 0.0)
        else:
            row([(iu + 0, 1.0), (iu + 2, -mu)], -inf, 0.0)   # 0 >= fx - mu fz
            row([(iu + 0, -1.0), (iu + 2, -mu)], -inf, 0.0)  # 0 >= -fx - mu fz
            if p.variant == '3f':
                row([(iu + 1, 1.0), (iu + 2, -mu)], -inf, 0.0)
                row([(iu + 1, -1.0), (iu + 2, -mu)], -inf, 0.0)
            row([(iu + 2, 1.0)], 0.0, inf)                  # fz >= 0
            row([(iu + 2, 1.0)], -inf, float(F_MAX[2]))     # fz <= f_max[2]
    for i in range(NX):                                     # :150 x[0] == x_in
        row([(_vx(N, 0) + i, 1.0)], x_in[i], x_in[i])
    return dict(P=P, q=q, r=r, A=np.array(rows), l=np.array(lo), u=np.array(hi))


def unpack(p: MpcParams, z):
    N = p.N
    x = z[:(N + 1) * NX].reshape(N + 1, NX)
    u = z[(N + 1) * NX:].reshape(N, NU)
    return x, u


def objective(p: MpcParams, x, u, x_ref, C, uref_mode='aliased'):
    """The reference cost (:132/:139) evaluated directly on a trajectory."""
    N = p.N
    obj = 0.0
    for k in range(N):
        kf = 100 if k == N - 1 else 1
        kuf = 0 if k == N - 1 else 1
        e = x[k + 1] - x_ref[k]
        du = u[k] - effective_uref(p, C, k, uref_mode)
        obj += e @ (Q_DIAG * kf * e) + du @ (R_DIAG * kuf * du)
    return obj


def rollout(p: MpcParams, x_in, u, Ad, Bd, Gd):
    """x[k+1] = Ad_k x[k] + Bd_k u[k] + Gd from x[0] = x_in."""
    x = np.zeros((p.N + 1, NX))
    x[0] = x_in
    for k in range(p.N):
        x[k + 1] = Ad[k] @ x[k] + Bd[k] @ u[k] + Gd
    return x


def solve_instance(p: MpcParams, x_in, x_lin, x_ref, pf, C, uref_mode='aliased', **kw):
    """gen_dt_dynamics + build_qp + exact solve for ONE linearisation x_lin.

    Returns dict(u, x, obj, status, ...) -- one "QP solve" of SURVEY.md 8d.
    """
    from . import qp_exact
    _, _, Gd = constant_matrices(p)
    Ad, Bd = gen_dt_dynamics(p, x_lin, pf)
    qp = build_qp(p, x_in, x_ref, Ad, Bd, Gd, C, uref_mode)
    sol = qp_exact.solve(qp['P'], qp['q'], qp['A'], qp['l'], qp['u'], **kw)
    out = dict(status=sol['status'], info=sol)
    if sol['x'] is None:
        out.update(u=None, x=None, obj=None)
        return out
    x, u = unpack(p, sol['x'])
    out.update(u=u, x=x, obj=0.5 * sol['x'] @ qp['P'] @ sol['x'] + qp['q'] @ sol['x'] + qp['r'],
               Ad=Ad, Bd=Bd, qp=qp)
    return out


class OracleMpc:
    """Stateful restatement of ``Mpc.mpcontrol`` (3f :41-69, 2f :40-68)."""

    def __init__(self, p: MpcParams, uref_mode='aliased'):
        self.p = p
        self.uref_mode = uref_mode
        self.x_value = None
        self.nsolves = 0

    def mpcontrol(self, x_in, x_ref_in, pf, C, init):
        N = self.p.N
        x_guess = np.zeros((N + 1, NX))
        if init is True:
            x_guess[0, :] = x_in
            x_guess[1:, :] = x_ref_in
            s = solve_instance(self.p, x_in, x_guess, x_ref_in, pf, C, self.uref_mode)
            self.nsolves += 1
            if s['u'] is None:
                raise Exception("\n *** QP FAILED *** \n")
            x_guess = s['x']
        else:
            x_guess[0, :] = x_in
            x_guess[1:-1, :] = self.x_value[2:, :]
            x_guess[-1, :] = self.x_value[-1, :]
        s = solve_instance(self.p, x_in, x_guess, x_ref_in, pf, C, self.uref_mode)
        self.nsolves += 1
        if s['u'] is None:
            raise Exception("\n *** QP FAILED *** \n")
        self.x_value = s['x']
        return s['u']
