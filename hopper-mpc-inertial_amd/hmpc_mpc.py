"""The reference's ``Mpc`` class, re-implemented on the MI355X solve path.

Same constructor ``Mpc(t, N, m, g, mu, Jinv, rh, **kwargs)`` and the same
``mpcontrol(x_in, x_ref_in, pf, C, init) -> u (N, 6)`` as
src/mpc_cvx_euler_3f.py:12-69 / src/mpc_cvx_euler_2f.py:12-68, including the
two-solve ``init=True`` path, the time-shifted warm linearisation of later
calls, the ``self.x.value`` / ``self.u.value`` attributes (cvxpy-Variable
look-alikes) and the ``Exception("\\n *** QP FAILED *** \\n")`` failure mode.

Every QP is solved by libhmpc.so on the GPU (``hmpc_solve_batch_host`` with
B = 1); there is no CPU fallback.

Extra keyword arguments: ``uref_mode`` ('aliased' = what the reference's
cvxpy problem actually contains, the default; 'per_stage' = the intended
u_ref) and ``device`` (HIP ordinal).
"""
from __future__ import annotations

import numpy as np

import hmpc


class _Value:
    """Stand-in for a cvxpy Variable: only ``.value`` is used by callers."""

    def __init__(self):
        self.value = None


class MpcBase:
    variant = '3f'

    def __init__(self, t, N, m, g, mu, Jinv, rh, **kwargs):
        self.t = t
        self.N = N
        self.m = m
        self.g = g
        self.mu = mu
        self.Jinv = Jinv
        self.rh = rh
        self.f_max = np.array([352, 0, 206])
        self.f_min = -self.f_max
        self.n_x = 12
        self.n_u = 6
        self.Q = np.diag([50., 50., 2., 1., 1., 50., 1., 1., 1., 10., 10., 10.])
        self.R = np.diag([0.001] * 6)
        self.x = _Value()
        self.u = _Value()
        self.objective = None
        self.solves = 0
        self.uref_mode = kwargs.get('uref_mode', 'aliased')
        self._ctx = hmpc.Context(self.variant, N, t=t, m=m, g=g, mu=mu, Jinv=Jinv, rh=rh,
                                 uref_mode=self.uref_mode, device=kwargs.get('device', 0))

    def mpcontrol(self, x_in, x_ref_in, pf, C, init):
        N = self.N
        x_guess = np.zeros((N + 1, self.n_x))
        if init is True:
            x_guess[0, :] = x_in
            x_guess[1:, :] = x_ref_in
            self._solve(x_in, x_guess, x_ref_in, pf, C)
            x_guess = self.x.value
        else:
            x_guess[0, :] = x_in
            x_guess[1:-1, :] = self.x.value[2:, :]
            x_guess[-1, :] = self.x.value[-1, :]
        self._solve(x_in, x_guess, x_ref_in, pf, C)
        return self.u.value

    def _solve(self, x_in, x_lin, x_ref, pf, C):
        r = self._ctx.solve_host(np.asarray(x_in, dtype=np.float64)[None],
                                 np.asarray(x_lin, dtype=np.float64)[None],
                                 np.asarray(x_ref, dtype=np.float64)[None],
                                 np.asarray(pf, dtype=np.float64)[None],
                                 np.asarray(C, dtype=np.float64)[None], mu=self.mu)
        self.solves += 1
        self.status = int(r['status'][0])
        if self.status != 0:
            self.x.value = None
            self.u.value = None
            raise Exception("\n *** QP FAILED *** \n")
        self.x.value = r['x'][0]
        self.u.value = r['u'][0]
        self.objective = float(r['obj'][0])
