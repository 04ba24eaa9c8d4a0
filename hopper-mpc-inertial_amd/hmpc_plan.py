"""Reference/gait generation and the synthetic instance sampler.

Host-side restatement of the Runner's planner, used to
draw the batched synthetic workload of SURVEY.md 8d:

* ``gait_scheduler`` / ``gait_map``   -- src/robotrunner.py:166-180
* ``path_plan_init``                  -- src/robotrunner.py:182-226, including
  the ``--curve`` quirks (x column overwritten by the *y* spline, yaw-rate
  column differentiating itself)
* ``path_plan_grab``                  -- src/robotrunner.py:228-230

All of it is plain numpy/scipy: it runs once per benchmark outside the timed
region, never on the solve path.
"""
from __future__ import annotations

import dataclasses

import numpy as np
from scipy.interpolate import CubicSpline
from scipy.signal import find_peaks


@dataclasses.dataclass
class RunnerConfig:
    """Runner constants (src/robotrunner.py:32-79)."""
    dt: float = 1e-3
    N_run: int = 2000
    curve: bool = False
    t_p: float = 0.8
    phi_switch: float = 0.5
    N: int = 60
    mpc_dt: float = 0.02
    step_adjustment: int = -115

    @property
    def mpc_factor(self):
        return int(self.mpc_dt / self.dt)

    @property
    def N_k(self):
        return int(self.N * self.mpc_factor)

    @property
    def t_start(self):
        return 0.5 * self.t_p * self.phi_switch

    @property
    def dist(self):
        return 0.4 * (self.N_run * self.dt)


def runner_constants():
    """Physical constants the Runner hands to ``Mpc`` (src/robotrunner.py:37-48,
    68, 76): m, g, the MPC step t = mpc_dt, mu, the body inertia J and its
    inverse, and the hip offset rh."""
    J = np.array([[76148072.89, 70089.52, 2067970.36],
                  [70089.52, 45477183.53, -87045.58],
                  [2067970.36, -87045.58, 76287220.47]]) * (10 ** (-9))   # :38-40
    return dict(t=0.02, m=7.5, g=9.807, mu=1.0, J=J, Jinv=np.linalg.inv(J),
                rh=-np.array([0.02663114, 0.04435752, 6.61082088]) / 1000)   # :43


def gait_scheduler(cfg: RunnerConfig, t, t0):
    phi = np.mod((t - t0) / cfg.t_p, 1)
    return 0 if phi > cfg.phi_switch else 1


def gait_map(cfg: RunnerConfig, N, dt, ts, t0):
    C = np.zeros(N)
    for k in range(0, N):
        C[k] = gait_scheduler(cfg, ts, t0)
        ts += dt
    return C


def initial_states(cfg: RunnerConfig):
    """convert(X_0), convert(X_f) for the identity-orientation start/goal
    (src/robotrunner.py:58-59,91): Euler angles and rates are all zero."""
    x0 = np.zeros(12)
    x0[2] = 0.27
    xf = np.zeros(12)
    xf[0] = cfg.dist
    xf[2] = 0.27
    return x0, xf


def path_plan_init(cfg: RunnerConfig, x_in, xf):
    N_k = cfg.N_k
    N_run = cfg.N_run
    dt = cfg.dt
    t_sit = 0
    t_traj = int(N_run - t_sit)
    t_ref = N_run + N_k
    x_ref = np.linspace(start=x_in, stop=xf, num=t_traj)
    if cfg.curve is True:
        spline_t = np.array([0, t_traj * 0.5, t_traj])
        spline_y = np.array([x_in[1], xf[1] * 0.9, xf[1]])
        csy = CubicSpline(spline_t, spline_y)
        spline_psi = np.array([0, -np.sin(45 * np.pi / 180) * 0.4, -np.sin(45 * np.pi / 180)])
        cspsi = CubicSpline(spline_t, spline_psi)
        for k in range(t_traj):
            x_ref[k, 0] = csy(k)     # sic: the reference writes the y spline into column 0
            x_ref[k, 5] = cspsi(k)
        x_ref[:-1, 11] = [(x_ref[i + 1, 11] - x_ref[i, 11]) / dt for i in range(N_run - 1)]
    x_ref = np.vstack((x_ref, np.tile(xf, (N_k + t_sit, 1))))
    period = cfg.t_p
    amp = cfg.t_p / 4
    phi = np.pi * 3 / 2
    x_ref[:, 2] = [x_in[2] + amp + amp * np.sin(2 * np.pi / period * (i * dt) + phi) for i in range(t_ref)]
    x_ref[:-1, 6:9] = [(x_ref[i + 1, 0:3] - x_ref[i, 0:3]) / dt for i in range(t_ref - 1)]
    C = gait_map(cfg, t_ref, dt, cfg.t_start, 0)
    idx_pf = find_peaks(-x_ref[:, 2])[0] + cfg.step_adjustment
    idx_pf = np.hstack((0, idx_pf))
    idx_pf = np.hstack((idx_pf, t_ref - 1))
    pf_ref = np.zeros((t_ref, 3))
    kf = 0
    n_idx = np.shape(idx_pf)[0]
    for k in range(1, t_ref):
        if C[k - 1] == 1 and C[k] == 0 and kf < n_idx:
            kf += 1
        pf_ref[k, 0:2] = x_ref[idx_pf[kf], 0:2]
    return x_ref, pf_ref


def path_plan_grab(cfg: RunnerConfig, x_ref, k):
    return x_ref[k:(k + cfg.N_k):cfg.mpc_factor, :]


def runner_plan(curve=False, N_run=2000):
    """The Runner's full plan (N=60 horizon padding) -- the source of every
    synthetic instance."""
    cfg = RunnerConfig(N_run=N_run, curve=curve)
    x0, xf = initial_states(cfg)
    x_ref, pf_ref = path_plan_init(cfg, x0, xf)
    return cfg, x_ref, pf_ref


BLOCK = 4096   # instances per independent random stream (sharding granule)


def _draw_block(seed, blk, n, N_run, f, mu_sweep):
    """Random draws of instances [blk*BLOCK, blk*BLOCK + n): a function of
    (seed, blk) only, so any shard of the global batch reproduces them."""
    rng = np.random.default_rng([seed, blk])
    k0 = f * rng.integers(0, N_run // f, size=BLOCK)
    noise = np.concatenate([rng.uniform(-0.02, 0.02, (BLOCK, 3)),
                            rng.uniform(-0.05, 0.05, (BLOCK, 3)),
                            rng.uniform(-0.2, 0.2, (BLOCK, 6))], axis=1)
    if mu_sweep is not None:
        mu = rng.uniform(mu_sweep[0], mu_sweep[1], BLOCK)
    else:
        mu = np.ones(BLOCK)
    return k0[:n], noise[:n], mu[:n]


def sample_instances(B, N, curve=False, seed=0, mu_sweep=None, N_run=2000, start=0):
    """Draw instances [start, start + B) of the synthetic workload of
    SURVEY.md 8d.

    Instance i's random draws depend only on (seed, i): a rank that asks for
    its shard [start, start + B) gets exactly the rows a single process
    drawing the whole batch would (``start`` must be a multiple of BLOCK
    unless B covers from the block start).

    Returns a dict of contiguous float64 arrays:
      x_in (B,12), x_lin (B,N+1,12) = [x_in; x_ref], x_ref (B,N,12),
      pf (B,N,3), C (B,N), mu (B,), k0 (B,) int
    ``mu_sweep=(lo, hi)`` draws mu ~ U(lo, hi), else mu = 1.
    """
    cfg, plan, pf_plan = runner_plan(curve=curve, N_run=N_run)
    f = cfg.mpc_factor
    parts = []
    i = start
    while i < start + B:
        blk, off = divmod(i, BLOCK)
        n = min(BLOCK - off, start + B - i)
        k0, noise, mu = _draw_block(seed, blk, off + n, N_run, f, mu_sweep)
        parts.append((k0[off:], noise[off:], mu[off:]))
        i += n
    if parts:
        k0 = np.concatenate([p[0] for p in parts])
        noise = np.concatenate([p[1] for p in parts])
        mu = np.concatenate([p[2] for p in parts])
    else:
        k0, noise, mu = np.zeros(0, dtype=np.int64), np.zeros((0, 12)), np.zeros(0)
    idx = k0[:, None] + f * np.arange(N)[None, :]
    x_ref = np.ascontiguousarray(plan[idx])
    pf = np.ascontiguousarray(pf_plan[idx])
    x_in = plan[k0] + noise
    # C is a function of k0 only: tabulate per distinct k0
    C = np.zeros((B, N))
    for kk in np.unique(k0):
        C[k0 == kk] = gait_map(cfg, N, cfg.mpc_dt, cfg.t_start + (kk + 1) * cfg.dt, 0)
    x_lin = np.concatenate([x_in[:, None, :], x_ref], axis=1)
    return dict(x_in=np.ascontiguousarray(x_in), x_lin=np.ascontiguousarray(x_lin),
                x_ref=x_ref, pf=pf, C=C, mu=mu, k0=k0)
