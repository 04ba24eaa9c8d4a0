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
launches and no host work; ``run(graph=True)`` replays the whole run as
one captured HIP graph.
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
        self._graphs = {}     # (steps, record) -> (graph, buffers, stream)
        self._x0_ver = 0

    def close(self):
        self.ctx.close()

    def run(self, n_periods=None, record=True, graph=False):
        """Runner.run (src/robotrunner.py:81-113) without plots.

        Runs the first ``n_periods`` MPC periods (all of N_run when None).
        Returns numpy arrays X_traj (B, steps+1, 13), f_hist (B, steps, 6),
        s_hist (steps,), plus per-call status (n_calls, B) and the plan.

        ``graph=True``: the periods (every mpcontrol, plant step and record
        copy: 5-8 launches per period) are captured once into a HIP graph on
        the Runner's own stream and replayed by later ``graph=True`` runs of
        the same length -- one graph launch per run instead of one host
        launch per kernel.  The first such call runs eagerly (it allocates
        the context's workspaces, which a capture cannot) and captures; a
        replay first re-plans on the device when the start states changed
        (``set_start``).  Results equal the eager run's bit for bit."""
        import torch
        steps = self._steps(n_periods)
        if not graph:
            S = self._setup(steps, record)
            self._enqueue(S)
            return self._finish(S)
        key = (steps, bool(record))
        g = self._graphs.get(key)
        if g is None:
            stream = torch.cuda.Stream(self.device)
            stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(stream):
                S = self._setup(steps, record)
                self._enqueue(S)          # eager: workspaces allocated, results valid
            stream.synchronize()
            res = self._finish(S)
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg, stream=stream):
                self._enqueue(S)
            self._graphs[key] = (cg, S, stream)
            return res
        cg, S, stream = g
        with torch.cuda.stream(stream):
            if S['x0_ver'] != self._x0_ver:
                self._replan(S)
            cg.replay()
        stream.synchronize()
        return self._finish(S)

    def set_start(self, X0):
        """New start states X_0 (13,) or (B, 13) for the next run (graph
        replays re-plan from them on the device)."""
        X0 = np.asarray(X0, dtype=np.float64)
        self.X0 = np.ascontiguousarray(np.broadcast_to(X0, (self.B, 13)))
        self._x0_ver += 1

    def _steps(self, n_periods):
        cfg = self.cfg
        return cfg.N_run if n_periods is None else min(cfg.N_run, int(n_periods) * cfg.mpc_factor)

    def _plan(self, X0buf, x_in):
        """convert(X_0) and path_plan_init on the device (:91,102)."""
        import torch
        cfg, B, dev = self.cfg, self.B, self.device
        f64 = dict(dtype=torch.float64, device=dev)
        self.ctx.convert_device(X0buf, x_in)                                      # :102
        # plan on the device: path_plan_init(convert(X_0), convert(X_f)) (:91),
        # one plan per robot -- or one shared plan when every robot starts alike
        shared = bool((self.X0 == self.X0[:1]).all())
        Bp = 1 if shared else B
        Xf = torch.from_numpy(np.tile(self.X_f, (Bp, 1))).to(dev)
        xf = torch.empty((Bp, 12), **f64)
        self.ctx.convert_device(Xf, xf)
        x0p = x_in[:1].clone() if shared else x_in.clone()
        plan_x, plan_pf, _ = self.ctx.plan_device(x0p, xf, cfg.N_run, cfg.N_k, cfg.dt, cfg.curve, cfg.t_p,
                                                  cfg.phi_switch, cfg.t_start, cfg.step_adjustment)
        if shared:
            plan_x, plan_pf = plan_x[0], plan_pf[0]
        return shared, plan_x, plan_pf

    def _setup(self, steps, record):
        """Device buffers, plan and gait schedule of one run."""
        import torch
        cfg, B, dev = self.cfg, self.B, self.device
        N, mf, dt = cfg.N, cfg.mpc_factor, cfg.dt
        f64 = dict(dtype=torch.float64, device=dev)
        X0buf = torch.from_numpy(self.X0.copy()).to(dev)
        x_in = torch.empty((B, 12), **f64)
        shared, plan_x, plan_pf = self._plan(X0buf, x_in)
        # gait schedule per low-level step and per MPC call, on the device
        # (the reference's float64 time accumulation, :92-101)
        C_all, s_hist_d = self.ctx.gait_device(steps, mf, N, dt, cfg.mpc_dt, cfg.t_p, cfg.phi_switch,
                                               cfg.t_start, 0.0)
        call_k = list(range(0, steps, mf))
        S = dict(steps=steps, record=record, X0buf=X0buf, x_in=x_in, shared=shared, plan_x=plan_x,
                 plan_pf=plan_pf, C_all=C_all, s_hist=s_hist_d, call_k=call_k,
                 x0_ver=self._x0_ver,
                 X=torch.empty((B, 13), **f64),
                 x_prev=torch.zeros((B, N + 1, 12), **f64),
                 out=dict(u=torch.empty((B, N, 6), **f64), obj=torch.empty(B, **f64),
                          status=torch.empty(B, dtype=torch.int32, device=dev),
                          iters=torch.empty(B, dtype=torch.int32, device=dev)),
                 X_traj=torch.empty((B, steps + 1, 13), **f64) if record else None,
                 f_hist=torch.empty((B, steps, 6), **f64) if record else None,
                 hist=torch.empty((B, mf, 13), **f64) if record else None,
                 status=torch.empty((len(call_k), B), dtype=torch.int32, device=dev))
        return S

    def _replan(self, S):
        """A replay with new start states: the plan again, into the captured
        buffers (the planner's error check syncs, so it stays out of the graph)."""
        S['X0buf'].copy_(torch_from(self.X0, S['X0buf']))
        shared, plan_x, plan_pf = self._plan(S['X0buf'], S['x_in'])
        if shared != S['shared']:
            raise ValueError('a graph replay cannot switch between a shared and per-robot plans; '
                             'run with graph=False or use a new Runner')
        S['plan_x'].copy_(plan_x)
        S['plan_pf'].copy_(plan_pf)
        S['x0_ver'] = self._x0_ver

    def _enqueue(self, S):
        """The MPC periods (:92-113) on the current stream, no host work: what
        a graph captures."""
        cfg, B = self.cfg, self.B
        N, mf, dt = cfg.N, cfg.mpc_factor, cfg.dt
        steps, record = S['steps'], S['record']
        X, x_in, x_prev, out = S['X'], S['x_in'], S['x_prev'], S['out']
        X.copy_(S['X0buf'])
        self.ctx.convert_device(X, x_in)                                         # :102
        x_prev.zero_()
        plan_x, plan_pf = S['plan_x'], S['plan_pf']
        T = plan_x.shape[-2]
        pf_flat = plan_pf.reshape(-1)
        pf_bs = 0 if S['shared'] else 3 * T
        X_traj, f_hist, hist = S['X_traj'], S['f_hist'], S['hist']
        if record:
            X_traj[:, 0] = X
        for p, k in enumerate(S['call_k']):
            self.ctx.mpcontrol_plan_device(p == 0, x_in, plan_x, plan_pf, k, mf, S['C_all'][p], x_prev,
                                           out=out)                             # :98-103
            S['status'][p] = out['status']
            n = min(mf, steps - k)
            self.ctx.plant_device(X, out['u'], 6 * N, pf_flat[3 * k:], pf_bs, 3, n, dt, self.J,
                                  X_hist=hist if record else None, x_out=x_in)   # :109-111
            if record:
                X_traj[:, k + 1:k + 1 + n] = hist[:, :n]
                f_hist[:, k:k + n] = out['u'][:, 0:1, :]

    def _finish(self, S):
        import torch
        torch.cuda.synchronize(self.device)
        st = S['status'].cpu().numpy()
        if (st != 0).any():
            bad = np.argwhere(st != 0)[0]
            raise Exception(f"\n *** QP FAILED *** \n (call {bad[0]}, robot {bad[1]}: "
                            f"{hmpc.STATUS.get(int(st[bad[0], bad[1]]), st[bad[0], bad[1]])})")
        res = dict(X_final=S['X'].cpu().numpy(), s_hist=S['s_hist'].cpu().numpy(), status=st,
                   x_ref=S['plan_x'].cpu().numpy(), pf_ref=S['plan_pf'].cpu().numpy(),
                   call_k=np.array(S['call_k']))
        if S['record']:
            res['X_traj'] = S['X_traj'].cpu().numpy()
            res['f_hist'] = S['f_hist'].cpu().numpy()
        return res


def torch_from(a, like):
    """numpy array -> tensor on `like`'s device."""
    import torch
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:   # e.g. a broadcast view (torch wants a writable buffer)
        a = a.copy()
    return torch.from_numpy(a).to(like.device)
