"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the Runner's plant and
closed loop.  Never imported by the product path.

* ``quat2euler``     -- src/utils.py:54-62 over transforms3d's
                        ``euler.quat2euler(q, axes='rzyx')`` (transforms3d is
                        absent here; its published quat2mat + mat2euler
                        algorithm is restated, as in tests/golden/_stubs)
* ``rot``            -- H' L(q) R(q)' H, src/utils.py:28-43 with H of :4-5
* ``convert``        -- src/robotrunner.py:19-28
* ``dynamics_ct``    -- src/robotrunner.py:126-152
* ``rk4_normalized`` -- src/robotrunner.py:154-164
* ``run_closed_loop``-- src/robotrunner.py:81-113 (Runner.run without plots),
                        with the oracle's exact Mpc (hmpc_oracle.OracleMpc)

Pinned by tests/golden/plant.npz (dX, Xn, x_conv of the reference's own
functions) and tests/golden/loop_3f_N10.npz (the reference loop's states).
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

_EPS4 = np.finfo(np.float64).eps * 4.0


def quat2euler(q):
    """[roll, pitch, yaw] of the unit quaternion q = [w, x, y, z]
    (src/utils.py:54-62: the 'rzyx' angles, reordered)."""
    w, x, y, z = q
    nq = w * w + x * x + y * y + z * z
    if nq < np.finfo(np.float64).eps:
        M = np.eye(3)
    else:
        s = 2.0 / nq
        X, Y, Z = x * s, y * s, z * s
        wX, wY, wZ = w * X, w * Y, w * Z
        xX, xY, xZ = x * X, x * Y, x * Z
        yY, yZ, zZ = y * Y, y * Z, z * Z
        M = np.array([[1.0 - (yY + zZ), xY - wZ, xZ + wY],
                      [xY + wZ, 1.0 - (xX + zZ), yZ - wX],
                      [xZ - wY, yZ + wX, 1.0 - (xX + yY)]])
    cy = math.sqrt(M[0, 0] * M[0, 0] + M[1, 0] * M[1, 0])
    if cy > _EPS4:
        ax = math.atan2(M[2, 1], M[2, 2])
        ay = math.atan2(-M[2, 0], cy)
        az = math.atan2(M[1, 0], M[0, 0])
    else:
        ax = math.atan2(-M[1, 2], M[1, 1])
        ay = math.atan2(-M[2, 0], cy)
        az = 0.0
    # 'rzyx' returns (z, y, x) = (az, ay, ax); utils.quat2euler reorders to xyz
    return np.array([ax, ay, az])


def rot(q):
    """Body-to-world rotation H' L(q) R(q)' H (src/utils.py:28-43)."""
    w, x, y, z = q
    return np.array([
        [w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z]])


def convert(X):
    """SE(3) simulator state -> Euler MPC state (src/robotrunner.py:19-28)."""
    x0 = np.zeros(12)
    x0[0:3] = X[0:3]
    q = X[3:7]
    x0[3:6] = quat2euler(q)
    Rm = rot(q)
    x0[6:9] = Rm @ X[7:10]
    x0[9:12] = Rm @ X[10:13]
    return x0


def dynamics_ct(X, U, pf, m, g, J, rh):
    """SE(3) rigid-body dynamics (src/robotrunner.py:126-152)."""
    p, q, v, w = X[0:3], X[3:7], X[7:10], X[10:13]
    Fw, tau = U[0:3], U[3:6]
    Rm = rot(q)
    Fgw = np.array([0.0, 0.0, -g]) * m
    Ftb = Rm.T @ (Fgw + Fw)
    r = rh + Rm.T @ (pf - p)
    Fb = Rm.T @ Fw
    tautb = tau + np.cross(r, Fb)
    dp = Rm @ v
    # 0.5 L(q) H w
    dq = 0.5 * np.array([-q[1] * w[0] - q[2] * w[1] - q[3] * w[2],
                         q[0] * w[0] - q[3] * w[1] + q[2] * w[2],
                         q[3] * w[0] + q[0] * w[1] - q[1] * w[2],
                         -q[2] * w[0] + q[1] * w[1] + q[0] * w[2]])
    dv = Ftb / m - np.cross(w, v)
    dw = np.linalg.solve(J, tautb - np.cross(w, J @ w))
    return np.concatenate([dp, dq, dv, dw])


def rk4_normalized(X, U, pf, h, m, g, J, rh):
    """Classic RK4 + quaternion renormalisation (src/robotrunner.py:154-164)."""
    f1 = dynamics_ct(X, U, pf, m, g, J, rh)
    f2 = dynamics_ct(X + 0.5 * h * f1, U, pf, m, g, J, rh)
    f3 = dynamics_ct(X + 0.5 * h * f2, U, pf, m, g, J, rh)
    f4 = dynamics_ct(X + h * f3, U, pf, m, g, J, rh)
    Xn = X + (h / 6.0) * (f1 + 2 * f2 + 2 * f3 + f4)
    Xn[3:7] = Xn[3:7] / np.linalg.norm(Xn[3:7])
    return Xn


def run_closed_loop(N=10, N_run=1000, curve=False, variant='3f', n_periods=None, X0=None):
    """Runner.run (src/robotrunner.py:81-113) with the oracle's exact Mpc.
    Returns X_traj (N_run+1, 13), f_hist (N_run, 6) and the per-call records."""
    here = os.path.dirname(os.path.abspath(__file__))
    pkg = os.path.join(os.path.dirname(here), 'hopper-mpc-inertial_amd')
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    import hmpc_plan as hp
    from oracle import hmpc_oracle as ho

    cfg = hp.RunnerConfig(N_run=N_run, curve=curve, N=N)
    c = ho.runner_constants()
    J = c['J']
    mpc = ho.OracleMpc(ho.MpcParams.runner(variant, N))
    X_traj = np.tile(np.array([0, 0, 0.27, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0], float), (N_run + 1, 1))
    if X0 is not None:
        X_traj[0] = X0
    # the plan from the robot's own start (src/robotrunner.py:91):
    # path_plan_init(convert(X_traj[0]), convert(X_f)), X_f = [dist, 0, 0.27, 1, 0...] (:58)
    X_f = np.hstack([cfg.dist, 0, 0.27, 1, np.zeros(9)])
    x_ref, pf_ref = hp.path_plan_init(cfg, convert(X_traj[0]), convert(X_f))
    f_hist = np.zeros((N_run, 6))
    t = cfg.t_start
    mf = cfg.mpc_factor
    counter = mf
    U = np.zeros((N, 6))
    init = True
    calls = []
    steps = N_run if n_periods is None else min(N_run, n_periods * mf)
    for k in range(steps):
        t = t + cfg.dt
        if counter == mf:
            counter = 0
            C = hp.gait_map(cfg, N, cfg.mpc_dt, t, 0)
            x_in = convert(X_traj[k])
            U = mpc.mpcontrol(x_in, hp.path_plan_grab(cfg, x_ref, k), hp.path_plan_grab(cfg, pf_ref, k),
                              C, init)
            calls.append(dict(k=k, x_in=x_in, C=C, U=U))
            init = False
        counter += 1
        f_hist[k] = U[0]
        X_traj[k + 1] = rk4_normalized(X_traj[k], f_hist[k], pf_ref[k], cfg.dt, c['m'], c['g'], J,
                                       c['rh'])
    return dict(X_traj=X_traj[:steps + 1], f_hist=f_hist[:steps], calls=calls, x_ref=x_ref,
                pf_ref=pf_ref, cfg=cfg)
