"""The Runner's planner on the device: hmpc_plan_batch
(path_plan_init + gait_map, src/robotrunner.py:166-226) and hmpc_gait_batch
(the loop's gait_scheduler / gait_map calls, :92-101).

* the reference's own plans (tests/golden/plan.npz, recorded by importing
  src/robotrunner.py): straight and --curve, from the default start;
* per-robot plans from random start states against the host restatement
  (hmpc_plan.path_plan_init, itself pinned by plan.npz), every robot at once;
* the gait schedule: bit-exact (the float64 time accumulation of the loop is
  reproduced operation for operation), and equal to the reference-recorded
  gait_C10 rows.

Tolerances: gait states and footstep choices exact; x_ref within 1e-12 of
the magnitude (the sine and the spline are within a few ulp of numpy/scipy;
velocity columns divide a difference by dt = 1e-3)."""
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def cx():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    import hmpc_plan
    c = hmpc_plan.runner_constants()
    ctx = hmpc.Context('3f', 10, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    yield ctx
    ctx.close()


def device_plan(cx, cfg, x0, xf):
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    x_ref, pf_ref, C = cx.plan_device(d(x0), d(xf), cfg.N_run, cfg.N_k, cfg.dt, cfg.curve, cfg.t_p,
                                      cfg.phi_switch, cfg.t_start, cfg.step_adjustment)
    torch.cuda.synchronize()
    return x_ref.cpu().numpy(), pf_ref.cpu().numpy(), C.cpu().numpy()


def close(a, b, rel=1e-12):
    scale = max(1.0, float(np.abs(b).max()))
    np.testing.assert_allclose(a, b, rtol=0, atol=rel * scale)


@pytest.mark.parametrize('curve', [False, True])
def test_reference_plan(cx, curve):
    import hmpc_plan as hp
    g = np.load(os.path.join(GOLDEN, 'plan.npz'))
    cfg = hp.RunnerConfig(N_run=2000, curve=curve)
    x0, xf = hp.initial_states(cfg)
    x_ref, pf_ref, C = device_plan(cx, cfg, x0[None], xf[None])
    tag = 'curve' if curve else 'straight'
    assert x_ref.shape == (1,) + g[f'{tag}_x_ref'].shape
    # per column: velocities are differences / dt
    for c in range(12):
        close(x_ref[0][:, c], g[f'{tag}_x_ref'][:, c], 1e-12 if c not in (6, 7, 8, 11) else 1e-10)
    np.testing.assert_array_equal(pf_ref[0], g[f'{tag}_pf_ref'])
    C_host = hp.gait_map(cfg, cfg.N_run + cfg.N_k, cfg.dt, cfg.t_start, 0)
    np.testing.assert_array_equal(C, C_host)


@pytest.mark.parametrize('curve', [False, True])
def test_per_robot_plans(cx, curve):
    import hmpc_plan as hp
    cfg = hp.RunnerConfig(N_run=1000, curve=curve, N=10)
    B = 16
    rng = np.random.default_rng(7)
    x0, xf = hp.initial_states(cfg)
    X0 = np.tile(x0, (B, 1))
    X0[:, 0:3] += rng.uniform(-0.05, 0.05, (B, 3))
    X0[:, 3:6] += rng.uniform(-0.1, 0.1, (B, 3))
    X0[:, 6:12] += rng.uniform(-0.3, 0.3, (B, 6))
    Xf = np.tile(xf, (B, 1))
    Xf[:, 1] += rng.uniform(-0.2, 0.2, B)   # a lateral goal: the --curve y spline is nonzero
    Xf[::2, 2] += 0.01
    x_ref, pf_ref, _ = device_plan(cx, cfg, X0, Xf)
    for b in range(B):
        hx, hpf = hp.path_plan_init(cfg, X0[b], Xf[b])
        for c in range(12):
            close(x_ref[b][:, c], hx[:, c], 1e-12 if c not in (6, 7, 8, 11) else 1e-10)
        close(pf_ref[b], hpf, 1e-13)


def test_gait_schedule(cx):
    import hmpc_plan as hp
    g = np.load(os.path.join(GOLDEN, 'plan.npz'))
    cfg = hp.RunnerConfig(N_run=2000, N=10)
    n_steps, mf = 2000, cfg.mpc_factor
    C, s_hist = cx.gait_device(n_steps, mf, 10, cfg.dt, cfg.mpc_dt, cfg.t_p, cfg.phi_switch, cfg.t_start)
    torch.cuda.synchronize()
    C, s_hist = C.cpu().numpy(), s_hist.cpu().numpy()
    t = cfg.t_start
    rows, s = [], []
    for k in range(n_steps):
        t = t + cfg.dt
        s.append(hp.gait_scheduler(cfg, t, 0))
        if k % mf == 0:
            rows.append(hp.gait_map(cfg, 10, cfg.mpc_dt, t, 0))
    np.testing.assert_array_equal(C, np.array(rows))
    np.testing.assert_array_equal(s_hist, np.array(s, dtype=np.float64))
    # the reference-recorded rows (gait_map(10, mpc_dt, ts, 0) at the loop's times)
    n = len(g['gait_ts'])
    np.testing.assert_array_equal(C[:n], g['gait_C10'])


def test_gait_schedule_before_t0(cx):
    """t < t0: np.mod((t - t0) / t_p, 1) is in [0, 1) (numpy follows the
    divisor's sign), so the device gait must not take fmod's negative phase."""
    import hmpc_plan as hp
    cfg = hp.RunnerConfig(N_run=400, N=10)
    n_steps, mf, t0 = 400, cfg.mpc_factor, 0.37
    C, s_hist = cx.gait_device(n_steps, mf, 10, cfg.dt, cfg.mpc_dt, cfg.t_p, cfg.phi_switch, cfg.t_start,
                               t0=t0)
    torch.cuda.synchronize()
    t = cfg.t_start
    rows, s = [], []
    for k in range(n_steps):
        t = t + cfg.dt
        s.append(hp.gait_scheduler(cfg, t, t0))
        if k % mf == 0:
            rows.append(hp.gait_map(cfg, 10, cfg.mpc_dt, t, t0))
    np.testing.assert_array_equal(C.cpu().numpy(), np.array(rows))
    np.testing.assert_array_equal(s_hist.cpu().numpy(), np.array(s, dtype=np.float64))
    assert (np.array(s) == 0.0).any() and (np.array(s) == 1.0).any()


def test_plan_index_errors_are_reported(cx):
    """Where the reference raises IndexError (a footstep peak pushed outside
    the plan by step_adjustment, src/robotrunner.py:211-216) hmpc_plan_batch
    returns HMPC_ERR_ARG instead of a silently clamped plan.  The error is
    raised only for a peak the footstep counter reads, as in the reference;
    no Runner configuration reaches an out-of-range peak that is never read
    (t_p 0.3-1.6, phi_switch 0.2-0.8 and step_adjustment 0-2000 searched with
    the host planner), so only the read case has a test."""
    import hmpc
    import hmpc_plan as hp
    cfg = hp.RunnerConfig(N_run=2000, N=10)
    x0, xf = hp.initial_states(cfg)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    with pytest.raises(hmpc.HmpcError, match='IndexError'):
        cx.plan_device(d(x0[None]), d(xf[None]), cfg.N_run, cfg.N_k, cfg.dt, cfg.curve, cfg.t_p,
                       cfg.phi_switch, cfg.t_start, 10 ** 6)
    # the same context plans normally afterwards (the error word is per call)
    x_ref, pf_ref, _ = cx.plan_device(d(x0[None]), d(xf[None]), cfg.N_run, cfg.N_k, cfg.dt, cfg.curve,
                                      cfg.t_p, cfg.phi_switch, cfg.t_start, cfg.step_adjustment)
    torch.cuda.synchronize()
    assert np.isfinite(x_ref.cpu().numpy()).all()
