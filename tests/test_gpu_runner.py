"""GPU parity of the Runner's loop on the device:
the plant kernel (dynamics_ct / rk4_normalized / convert,
src/robotrunner.py:19-28,126-164) against the reference's outputs in
tests/golden/plant.npz, the plan-view mpcontrol against the contiguous one,
and the whole batched Runner (hmpc_runner.Runner) against the reference's own
closed loop (tests/golden/loop_3f_N10.npz) and the oracle's.

Tolerances: plant 1e-12 absolute on states (1e-13 relative on derivatives
of size ~1e2; the kernel multiplies by J^-1 where the reference solves with J,
and contracts to FMAs); closed loop 1e-7 on states (the MPC input differs from
the exact optimum by <= 1e-6 N; 1000 RK4 steps of 1 ms keep that well below).
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def hm():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    return hmpc


def ctx(hm, variant='3f', N=10):
    from oracle import hmpc_oracle as ho
    c = ho.runner_constants()
    return hm.Context(variant, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])


def test_plant_kernel_matches_reference(hm):
    from oracle import hmpc_oracle as ho
    from oracle import hmpc_plant as pl
    c = ho.runner_constants()
    d = np.load(os.path.join(GOLDEN, 'plant.npz'))
    B = len(d['X'])
    cx = ctx(hm)
    X = torch.from_numpy(d['X'].copy()).cuda()
    U = torch.from_numpy(d['U'].copy()).cuda()
    pf = torch.from_numpy(d['pf'].copy()).cuda()
    xo = torch.empty((B, 12), dtype=torch.float64, device='cuda')
    cx.plant_device(X, U, 6, pf, 3, 0, 1, 1e-3, c['J'], x_out=xo)
    torch.cuda.synchronize()
    np.testing.assert_allclose(X.cpu().numpy(), d['Xn'], rtol=0, atol=1e-12)
    # convert of the stepped state against the oracle, and of the golden states
    xs = np.array([pl.convert(x) for x in X.cpu().numpy()])
    np.testing.assert_allclose(xo.cpu().numpy(), xs, rtol=0, atol=1e-12)
    Xg = torch.from_numpy(d['X'].copy()).cuda()
    cx.convert_device(Xg, xo)
    torch.cuda.synchronize()
    np.testing.assert_allclose(xo.cpu().numpy(), d['x_conv'], rtol=0, atol=1e-13)
    cx.close()


def test_plant_kernel_many_steps_matches_oracle(hm):
    """20 steps with a per-step foot position and history, 256 robots."""
    from oracle import hmpc_oracle as ho
    from oracle import hmpc_plant as pl
    c = ho.runner_constants()
    rng = np.random.default_rng(3)
    B, S = 256, 20
    X0 = np.zeros((B, 13))
    X0[:, 0:3] = rng.uniform(-1, 1, (B, 3))
    q = rng.normal(size=(B, 4))
    X0[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    X0[:, 7:13] = rng.uniform(-1, 1, (B, 6))
    U = rng.uniform(-50, 150, (B, 6))
    pf = rng.uniform(-0.5, 0.5, (S, 3))   # shared, per step (pf_ref[k + s])
    cx = ctx(hm)
    X = torch.from_numpy(X0.copy()).cuda()
    hist = torch.empty((B, S, 13), dtype=torch.float64, device='cuda')
    cx.plant_device(X, torch.from_numpy(U).cuda(), 6, torch.from_numpy(pf).cuda(), 0, 3, S, 1e-3,
                    c['J'], X_hist=hist)
    torch.cuda.synchronize()
    H = hist.cpu().numpy()
    for b in range(0, B, 17):
        Xr = X0[b].copy()
        for s in range(S):
            Xr = pl.rk4_normalized(Xr, U[b], pf[s], 1e-3, c['m'], c['g'], c['J'], c['rh'])
            np.testing.assert_allclose(H[b, s], Xr, rtol=0, atol=1e-11)
    np.testing.assert_array_equal(X.cpu().numpy(), H[:, -1])
    cx.close()


def test_plan_view_mpcontrol_equals_contiguous(hm):
    """hmpc_mpcontrol_plan_batch reads path_plan_grab windows in place; the
    same windows staged contiguously through hmpc_mpcontrol_batch must give
    bitwise identical results (init and time-shift calls)."""
    import hmpc_plan as hp
    N, B = 10, 64
    cfg, plan, pf_plan = hp.runner_plan(curve=True, N_run=2000)
    cfg = hp.RunnerConfig(N_run=2000, curve=True, N=N)
    cx = ctx(hm, N=N)
    P = torch.from_numpy(np.ascontiguousarray(plan)).cuda()
    PF = torch.from_numpy(np.ascontiguousarray(pf_plan)).cuda()
    res = {}
    for mode in ('view', 'contig'):
        x_prev = torch.zeros((B, N + 1, 12), dtype=torch.float64, device='cuda')
        outs = []
        for call, k in enumerate((400, 420, 440)):
            x_in = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(plan[k], (B, 12)) +
                                                         0.01 * np.sin(np.arange(B * 12).reshape(B, 12) + k))).cuda()
            C = hp.gait_map(cfg, N, cfg.mpc_dt, cfg.t_start + (k + 1) * 1e-3, 0)
            if mode == 'view':
                o = cx.mpcontrol_plan_device(call == 0, x_in, P, PF, k, 20,
                                             torch.from_numpy(C).cuda(), x_prev)
            else:
                xr = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(
                    hp.path_plan_grab(cfg, plan, k), (B, N, 12)))).cuda()
                pr = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(
                    hp.path_plan_grab(cfg, pf_plan, k), (B, N, 3)))).cuda()
                Cb = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(C, (B, N)))).cuda()
                o = cx.mpcontrol_device(call == 0, x_in, xr, pr, Cb, x_prev)
            torch.cuda.synchronize()
            outs.append((o['u'].cpu().numpy().copy(), o['status'].cpu().numpy().copy(),
                         x_prev.cpu().numpy().copy()))
        res[mode] = outs
    for a, b in zip(res['view'], res['contig']):
        assert (a[1] == 0).all()
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[2], b[2])
    cx.close()


def test_plan_view_rejects_window_outside_plan(hm):
    N = 10
    cx = ctx(hm, N=N)
    T = 100
    P = torch.zeros((T, 12), dtype=torch.float64, device='cuda')
    PF = torch.zeros((T, 3), dtype=torch.float64, device='cuda')
    x_in = torch.zeros((2, 12), dtype=torch.float64, device='cuda')
    C = torch.ones(N, dtype=torch.float64, device='cuda')
    x_prev = torch.zeros((2, N + 1, 12), dtype=torch.float64, device='cuda')
    with pytest.raises(hm.HmpcError):
        cx.mpcontrol_plan_device(True, x_in, P, PF, 0, 20, C, x_prev)   # 9*20 >= 100
    cx.close()


def test_runner_on_device_matches_reference_loop(hm):
    import hmpc_runner
    g = np.load(os.path.join(GOLDEN, 'loop_3f_N10.npz'))
    n = int(len(g['k']))
    r = hmpc_runner.Runner(dt=1e-3, dyn='3f', curve=bool(g['curve']), N_run=int(g['N_run']),
                           N=int(g['N']), batch=1)
    out = r.run(n_periods=n)
    r.close()
    X = out['X_traj'][0]
    assert X.shape == (20 * n + 1, 13)
    np.testing.assert_allclose(X[::20], g['X_traj_mpc'], rtol=0, atol=1e-7)
    np.testing.assert_allclose(out['f_hist'][0][::20], g['U0'], rtol=0, atol=1e-6)
    assert (out['status'] == 0).all()


def test_runner_batch_rows_are_independent(hm):
    """Robot b of a batched run == the same robot run alone (bitwise), and
    every robot tracks the oracle's closed loop from its own start state."""
    import hmpc_runner
    from oracle import hmpc_plant as pl
    B, n = 8, 10
    rng = np.random.default_rng(11)
    X0 = np.tile(hmpc_runner.X0_DEFAULT, (B, 1))
    X0[:, 0:3] += rng.uniform(-0.01, 0.01, (B, 3))
    X0[:, 7:10] += rng.uniform(-0.05, 0.05, (B, 3))
    r = hmpc_runner.Runner(dyn='3f', curve=True, N_run=400, N=10, batch=B, X0=X0)
    out = r.run(n_periods=n)
    r.close()
    r1 = hmpc_runner.Runner(dyn='3f', curve=True, N_run=400, N=10, batch=1, X0=X0[5])
    out1 = r1.run(n_periods=n)
    r1.close()
    np.testing.assert_array_equal(out['X_traj'][5], out1['X_traj'][0])
    ref = pl.run_closed_loop(N=10, N_run=400, curve=True, n_periods=n, X0=X0[2])
    np.testing.assert_allclose(out['X_traj'][2], ref['X_traj'], rtol=0, atol=1e-7)


def test_run_cli_mirror(hm, tmp_path):
    """hmpc_run.py, the reference run.py's CLI on the device Runner."""
    import hmpc_run
    out = tmp_path / 'run.npz'
    res = hmpc_run.main(['3f', '--N_run', '200', '--N', '10', '--batch', '2', '--out', str(out)])
    d = np.load(out)
    assert d['X_traj'].shape == (2, 201, 13) and (res['status'] == 0).all()
    np.testing.assert_array_equal(d['X_traj'][0], d['X_traj'][1])   # same start state


def test_runner_graph_replay_equals_eager(hm):
    """run(graph=True): the first call runs eagerly and captures the periods
    into a HIP graph, later calls replay it (re-planning on the device after
    set_start).  Every replay equals the eager run bit for bit."""
    import hmpc_runner
    B, n = 4, 12
    rng = np.random.default_rng(5)
    X0 = np.tile(hmpc_runner.X0_DEFAULT, (B, 1))
    X0[:, 0:3] += rng.uniform(-0.01, 0.01, (B, 3))
    X0b = X0.copy()
    X0b[:, 7:10] += rng.uniform(-0.05, 0.05, (B, 3))
    r = hmpc_runner.Runner(dyn='3f', curve=True, N_run=400, N=10, batch=B, X0=X0)
    e = r.run(n_periods=n)
    g1 = r.run(n_periods=n, graph=True)
    g2 = r.run(n_periods=n, graph=True)
    r.set_start(X0b)
    g3 = r.run(n_periods=n, graph=True)
    r.close()
    rb = hmpc_runner.Runner(dyn='3f', curve=True, N_run=400, N=10, batch=B, X0=X0b)
    eb = rb.run(n_periods=n)
    rb.close()
    for got, want in ((g1, e), (g2, e), (g3, eb)):
        for k in ('X_traj', 'f_hist', 'status', 'x_ref', 'pf_ref'):
            np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    assert not np.array_equal(e['X_traj'], eb['X_traj'])


def test_runner_eager_after_capture(hm):
    """An eager run on the default stream right after a graph capture on the
    Runner's stream, then a replay: the context's stream ordering
    skips the capture (no wait on, or record of, a captured event), and all
    three runs agree bit for bit."""
    import hmpc_runner
    B, n = 3, 8
    r = hmpc_runner.Runner(dyn='3f', curve=False, N_run=300, N=10, batch=B)
    g1 = r.run(n_periods=n, graph=True)    # eager on the Runner's stream, then the capture
    e = r.run(n_periods=n)                 # eager on the default stream
    g2 = r.run(n_periods=n, graph=True)    # replay
    e2 = r.run(n_periods=n)
    r.close()
    for got in (g1, g2, e2):
        for k in ('X_traj', 'f_hist', 'status'):
            np.testing.assert_array_equal(got[k], e[k], err_msg=k)
