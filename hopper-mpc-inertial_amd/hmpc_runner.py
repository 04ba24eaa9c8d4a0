"""Batched, device-resident mirror of the reference Runner
(src/robotrunner.py:31-113): B robots follow the Runner's plan under MPC,
every per-step quantity stays on the GPU.

Per MPC period (mpc_factor low-level steps, src/robotrunner.py:92-113):

* ``hmpc_mpcontrol_plan_batch`` -- ``Mpc.mpcontrol`` on path_plan_grab
  windows read in place from the device-resident plan (:98-107), warm start
  (x* of the previous period) kept on the device;
* ``hmpc_plant_batch``          -- mpc_factor ``rk4_normalized`` steps with
  the first input row held (:109-111), then ``convert`` for the next solve.

The plan (``path_plan_init``, one per robot from its own start state, or one
shared plan when all robots start alike) and the gait schedule (``gait_map``
per MPC call, ``gait_scheduler`` per step) are made on the device too
(``hmpc_plan_batch`` / ``hmpc_gait_batch``), so a period is two kernel
launches and no host work.
Plots are out of scope.

There is no CPU fallback: without libhmpc.so or a GPU this raises.
"""
from __future__ import annotations

import numpy as np

import hmpc
import hmpc_plan as hp

X0_DEFAULT = np.array([0, 0, 0.27, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0], dtype=np.float64)   # :57


class Runner:
    """``Runner(dt, dyn, curve, N_run)`` (src/robotrunner.py:31) for ``batch``
    robots at once.  ``N`` is the MPC horizon (the reference fixes 60,
    :46); ``X0`` (13,) or (batch, 13) overrides the start state X_0 (:57)."""

    def __init__(self, dt=1e-3, dyn='2f', curve=False, N_run=5000, N=60, batch=1, X0=None, mu=1.0,
                 uref_mode='aliased', device=0):
        import torch
        self.cfg = hp.RunnerConfig(dt=dt, N_run=N_run, curve=curve, N=N)
        self.dyn = dyn
        self.B = int(batch)
        self.device = torch.device('cuda', device)
        c = hp.runner_constants()                                              # :37-48
        m, g = c['m'], c['g']
        self.J = c['J']
        self.Jinv = c['Jinv']
        self.rh = c['rh']
        self.ctx = hmpc.Context(dyn, N, t=self.cfg.mpc_dt, m=m, g=g, mu=mu, Jinv=self.Jinv,
                                rh=self.rh, uref_mode=uref_mode, device=device)
        X0 = X0_DEFAULT if X0 is None else np.asarray(X0, dtype=np.float64)
        self.X0 = np.ascontiguousarray(np.broadcast_to(X0, (self.B, 13)))
        # X_f = [dist, 0, 0.27, 1, 0 ...] (:58)
        self.X_f = np.hstack([self.cfg.dist, 0, 0.27, 1, np.zeros(9)]).astype(np.float64)

    def close(self):
        self.ctx.close()

    def run(self, n_periods=None, record=True):
        """Runner.run (src/robotrunner.py:81-113) without plots.

        Runs the first ``n_periods`` MPC periods (all of N_run when None).
        Returns numpy arrays X_traj (B, steps+1, 13), f_hist (B, steps, 6),
        s_hist (steps,), plus per-call status (n_calls, B) and the plan."""
        import torch
        cfg, B, dev = self.cfg, self.B, self.device
        N, mf, dt = cfg.N, cfg.mpc_factor, cfg.dt
        steps = cfg.N_run if n_periods is None else min(cfg.N_run, int(n_periods) * mf)
        f64 = dict(dtype=torch.float64, device=dev)
        X = torch.from_numpy(self.X0.copy()).to(dev)
        x_in = torch.empty((B, 12), **f64)
        self.ctx.convert_device(X, x_in)                                         # :102
        # plan on the device: path_plan_init(convert(X_0), convert(X_f)) (:91),
        # one plan per robot -- or one shared plan when every robot starts alike
        shared = bool((self.X0 == self.X0[:1]).all())
        Bp = 1 if shared else B
        Xf = torch.from_numpy(np.tile(self.X_f, (Bp, 1))).to(dev)
        xf = torch.empty((Bp, 12), **f64)
        self.ctx.convert_device(Xf, xf)
        x0p = x_in[:1].clone() if shared else x_in.clone()
        plan_x, plan_pf, _ = self.ctx.plan_device(x0p, xf, cfg.N_run, cfg.N_k, dt, cfg.curve, cfg.t_p,
                                                  cfg.phi_switch, cfg.t_start, cfg.step_adjustment)
        T = plan_x.shape[1]
        if shared:
            plan_x, plan_pf = plan_x[0], plan_pf[0]
        # gait schedule per low-level step and per MPC call, on the device
        # (the reference's float64 time accumulation, :92-101)
        C_all, s_hist_d = self.ctx.gait_device(steps, mf, N, dt, cfg.mpc_dt, cfg.t_p, cfg.phi_switch,
                                               cfg.t_start, 0.0)
        call_k = list(range(0, steps, mf))
        pf_flat = plan_pf.reshape(-1)
        pf_bs = 0 if shared else 3 * T
        x_prev = torch.zeros((B, N + 1, 12), **f64)
        out = dict(u=torch.empty((B, N, 6), **f64), obj=torch.empty(B, **f64),
                   status=torch.empty(B, dtype=torch.int32, device=dev),
                   iters=torch.empty(B, dtype=torch.int32, device=dev))
        X_traj = torch.empty((B, steps + 1, 13), **f64) if record else None
        f_hist = torch.empty((B, steps, 6), **f64) if record else None
        hist = torch.empty((B, mf, 13), **f64) if record else None
        if record:
            X_traj[:, 0] = X
        status = torch.empty((len(call_k), B), dtype=torch.int32, device=dev)
        for p, k in enumerate(call_k):
            self.ctx.mpcontrol_plan_device(p == 0, x_in, plan_x, plan_pf, k, mf, C_all[p], x_prev,
                                           out=out)                             # :98-103
            status[p] = out['status']
            n = min(mf, steps - k)
            self.ctx.plant_device(X, out['u'], 6 * N, pf_flat[3 * k:], pf_bs, 3, n, dt, self.J,
                                  X_hist=hist if record else None, x_out=x_in)   # :109-111
            if record:
                X_traj[:, k + 1:k + 1 + n] = hist[:, :n]
                f_hist[:, k:k + n] = out['u'][:, 0:1, :]
        torch.cuda.synchronize(dev)
        st = status.cpu().numpy()
        if (st != 0).any():
            bad = np.argwhere(st != 0)[0]
            raise Exception(f"\n *** QP FAILED *** \n (call {bad[0]}, robot {bad[1]}: "
                            f"{hmpc.STATUS.get(int(st[bad[0], bad[1]]), st[bad[0], bad[1]])})")
        res = dict(X_final=X.cpu().numpy(), s_hist=s_hist_d.cpu().numpy(), status=st,
                   x_ref=plan_x.cpu().numpy(), pf_ref=plan_pf.cpu().numpy(), call_k=np.array(call_k))
        if record:
            res['X_traj'] = X_traj.cpu().numpy()
            res['f_hist'] = f_hist.cpu().numpy()
        return res
