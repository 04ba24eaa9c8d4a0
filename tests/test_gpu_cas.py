"""The CasADi variant on the GPU (hmpc::cas_kernel, HMPC_VARIANT_CAS;
src/mpc_cas_euler_3f.py) against the CPU restatement.

* the recorded instances of tests/golden/cas_N10.npz (the reference's own
  QP data): u* within 1e-6 of the recorded exact solution;
* 64 sampled instances of the bench workload (curve plan): every GPU solution
  is feasible for the reference-built rows and bounds and carries its own
  KKT certificate (non-negative multipliers by NNLS, stationarity <= 1e-8);
  u* within 1e-6 of oracle/cas_oracle's exact solve, which certifies every
  instance (a primal active-set method, oracle/qp_primal.py: the IPM it
  replaced stalled on about one in six of these degenerate problems);
* the drop-in module mpc_cas_euler_3f.Mpc with the reference's call surface.

Solve parity against qpOASES itself is unpinned (casadi/qpOASES absent)."""
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
U_TOL = 1e-6


@pytest.fixture(scope='module')
def ctx():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    import hmpc_plan
    c = hmpc_plan.runner_constants()
    cx = hmpc.Context('cas', 10, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    assert cx.kernel_name == 'hmpc::cas_kernel'
    yield cx
    cx.close()


def solve(cx, x_in, x_ref, C, N=10):
    B = len(x_in)
    return cx.solve_host(x_in, np.zeros((B, N + 1, 12)), x_ref, np.zeros((B, N, 3)), C)


def feasible(qp, z, N, tol=1e-7):
    from oracle import cas_oracle as co
    nX = 12 * (N + 1)
    g = qp['A'] @ z + qp['g0']
    keep = ~np.any(qp['A'][:, 12 * N:nX] != 0.0, axis=1)   # x_N's rows: x_N sits on them
    ok_g = np.all(g[keep] <= qp['ubg'][keep] + tol) and np.all(g[keep] >= np.where(
        qp['lbg'][keep] <= -co.BIG, -np.inf, qp['lbg'][keep]) - tol)
    zb = z.copy()
    ok_x = np.all(zb <= qp['ubx'] + tol) and np.all(zb >= qp['lbx'] - tol)
    return ok_g and ok_x


def test_recorded_instances(ctx):
    g = np.load(os.path.join(GOLDEN, 'cas_N10.npz'))
    r = solve(ctx, g['x_in'], g['x_ref'], g['C'])
    assert (r['status'] == 0).all()
    assert np.abs(r['u'] - g['u']).max() <= U_TOL


def test_sampled_instances(ctx):
    import hmpc_plan
    from oracle import cas_oracle as co
    N, B = 10, 64
    inst = hmpc_plan.sample_instances(B, N, curve=True, seed=5)
    c = hmpc_plan.runner_constants()
    r = solve(ctx, inst['x_in'], inst['x_ref'], inst['C'])
    assert (r['status'] == 0).all()
    n_cert = 0
    for b in range(B):
        qp = co.build_qp(0.02, N, c['m'], c['g'], 1.0, c['Jinv'], c['rh'], inst['x_in'][b], inst['x_ref'][b],
                         inst['C'][b])
        z = np.concatenate([r['x'][b].ravel(), r['u'][b].ravel()])
        assert feasible(qp, z, N), b
        obj = 0.5 * z @ qp['P'] @ z + qp['q'] @ z + qp['r']
        assert abs(obj - r['obj'][b]) <= 1e-9 * abs(obj)
        # optimal: a KKT certificate of the GPU point itself (independent of
        # any solver) ...
        assert co.kkt_residual(qp, z, N) <= 1e-8, b
        # ... and the oracle's exact, certified solve of every instance
        ref = co.solve(qp, N)
        assert ref['status'] == 'solved', (b, ref['status'])
        n_cert += 1
        assert np.abs(r['u'][b] - ref['u']).max() <= U_TOL, b
        assert abs(obj - ref['obj']) <= 1e-9 * abs(ref['obj'])
    assert n_cert == B


def test_dropin_module(ctx):
    import hmpc_plan
    import mpc_cas_euler_3f
    g = np.load(os.path.join(GOLDEN, 'cas_N10.npz'))
    c = hmpc_plan.runner_constants()
    mpc = mpc_cas_euler_3f.Mpc(t=c['t'], N=10, Jinv=c['Jinv'], rh=c['rh'], m=c['m'], g=c['g'], mu=1)
    u = mpc.mpcontrol(x_in=g['x_in'][0], x_ref_in=g['x_ref'][0], rf=None, C=g['C'][0])
    assert u.shape == (10, 6) and mpc.status == 0
    assert np.abs(u - g['u'][0]).max() <= U_TOL
