"""Drop-in for the reference module src/mpc_cas_euler_3f.py (the CasADi /
qpOASES variant).  Same constructor ``Mpc(t, N, Jinv, rh, m, g, mu, **kwargs)``
(:14) and ``mpcontrol(x_in, x_ref_in, rf, C) -> u (N, 6)`` (:112); the QP the
reference builds -- second-order discretisation at the yaw of x_in, scalar
u_ref on all six inputs, one-sided dynamics rows, the fixed foot vector
(``rf`` is ignored, as in the reference) -- is solved exactly on the MI355X
(``hmpc::cas_kernel``, HMPC_VARIANT_CAS).  The reference passes the solver's
result back without checking it (``error_on_fail: 0``); this mirror does the
same, and keeps the per-solve status in ``self.status``.

1 <= N <= 11 (the reference's equality block covers the initial condition
only there).  There is no CPU fallback.
"""
from __future__ import annotations

import numpy as np

import hmpc


class Mpc:

    def __init__(self, t, N, Jinv, rh, m, g, mu, **kwargs):
        self.t = t
        self.N = N
        self.Jinv = Jinv
        self.rhat = rh
        self.m = m
        self.g = g
        self.mu = mu
        self.n_x = 12
        self.n_u = 6
        self.status = None
        self._ctx = hmpc.Context('cas', N, t=t, m=m, g=g, mu=mu, Jinv=Jinv, rh=rh,
                                 device=kwargs.get('device', 0))

    def mpcontrol(self, x_in, x_ref_in, rf, C):
        N = self.N
        x_in = np.asarray(x_in, dtype=np.float64).reshape(1, 12)
        x_ref = np.asarray(x_ref_in, dtype=np.float64).reshape(1, N, 12)
        C = np.asarray(C, dtype=np.float64).reshape(1, N)
        x_lin = np.zeros((1, N + 1, 12))     # unused by this variant
        pf = np.zeros((1, N, 3))             # unused (rf is fixed, :39)
        r = self._ctx.solve_host(x_in, x_lin, x_ref, pf, C)
        self.status = int(r['status'][0])
        self.x_opt = r['x'][0]
        self.objective = float(r['obj'][0])
        return r['u'][0]
