"""The CasADi variant (src/mpc_cas_euler_3f.py) pinned on
the CPU: the QP data the reference's own Mpc hands qpOASES -- recorded by
tests/golden/make_golden.py through a casadi stub (tests/golden/_stubs/casadi)
-- is reproduced by the numpy restatement oracle/cas_oracle.build_qp, and the
restatement's exact solve reproduces the recorded solution.

Solve parity against qpOASES itself is unpinned: casadi/qpOASES are absent,
and the recorded solution is the exact optimum of the recorded data
(oracle/cas_oracle.solve), not qpOASES's output."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def fx():
    return np.load(os.path.join(GOLDEN, 'cas_N10.npz'))


def recorded_A(g, b):
    off = np.concatenate([[0], np.cumsum(g['A_nnz'])])
    A = np.zeros(tuple(g['A_shape']))
    sl = slice(off[b], off[b + 1])
    A[g['A_row'][sl], g['A_col'][sl]] = g['A_val'][sl]
    return A


def test_problem_data_matches_the_reference(fx):
    from oracle import cas_oracle as co
    g = fx
    N = int(g['N'])
    for b in range(len(g['x_in'])):
        qp = co.build_qp(0.02, N, 7.5, 9.807, 1.0, g['Jinv'], g['rh'], g['x_in'][b], g['x_ref'][b], g['C'][b])
        np.testing.assert_array_equal(np.diag(qp['P']), g['Pdiag'][b])
        np.testing.assert_array_equal(qp['q'], g['q'][b])
        np.testing.assert_allclose(qp['A'], recorded_A(g, b), rtol=0, atol=1e-15)
        np.testing.assert_allclose(qp['g0'], g['g0'][b], rtol=0, atol=1e-15)
        for k in ('lbg', 'ubg', 'lbx', 'ubx'):
            np.testing.assert_array_equal(qp[k], g[k][b])
        assert abs(qp['r'] - g['r'][b]) <= 1e-12 * abs(g['r'][b])


def test_exact_solution_reproduced(fx):
    from oracle import cas_oracle as co
    g = fx
    N = int(g['N'])
    for b in range(len(g['x_in'])):
        qp = co.build_qp(0.02, N, 7.5, 9.807, 1.0, g['Jinv'], g['rh'], g['x_in'][b], g['x_ref'][b], g['C'][b])
        r = co.solve(qp, N)
        assert r['status'] == 'solved'
        assert np.abs(r['u'] - g['u'][b]).max() <= 1e-6


def test_reference_quirks_are_in_the_data(fx):
    """What the reference builds, not what it meant: the fy rows repeat the
    fx rows plus one last-stage row each (:75-76); only the first N + 1 rows
    are equalities (:98); the same yaw for every stage (:139)."""
    g = fx
    N = int(g['N'])
    A = recorded_A(g, 0)
    nd = 12 + 12 * N
    fx1 = A[nd:nd + N]
    fy1 = A[nd + 2 * N:nd + 3 * N + 1]
    np.testing.assert_array_equal(fy1[:N], fx1)
    assert (g['lbg'][0][:N + 1] == 0).all() and (g['lbg'][0][N + 1:] == -1e10).all()


def test_primal_active_set_certifies_sampled_instances():
    """oracle/qp_primal.py (exact primal active set from the simulated
    zero-input trajectory) certifies every sampled CasADi QP -- the IPM of
    qp_exact stalls on about one in six of these degenerate problems -- and
    agrees with the IPM + polish wherever that one certifies."""
    import warnings

    import hmpc_plan
    from oracle import cas_oracle as co
    from oracle import qp_exact
    N, B = 10, 16
    inst = hmpc_plan.sample_instances(B, N, curve=True, seed=5)
    c = hmpc_plan.runner_constants()
    both = 0
    for b in range(B):
        qp = co.build_qp(0.02, N, c['m'], c['g'], 1.0, c['Jinv'], c['rh'], inst['x_in'][b], inst['x_ref'][b],
                         inst['C'][b])
        r = co.solve(qp, N)
        assert r['status'] == 'solved', (b, r['status'])
        z = r['z']
        assert co.kkt_residual(qp, z, N) <= 1e-8
        # the same reduced problem through the IPM route
        keep = np.ones(len(z), bool)
        keep[12 * N:12 * (N + 1)] = False
        rows = ~np.any(qp['A'][:, ~keep] != 0.0, axis=1)
        inf = lambda v: np.where(v >= co.BIG, np.inf, np.where(v <= -co.BIG, -np.inf, v))   # noqa: E731
        Ar = np.vstack([qp['A'][rows][:, keep], np.eye(int(keep.sum()))])
        lo = np.concatenate([inf(qp['lbg'][rows]) - qp['g0'][rows], inf(qp['lbx'][keep])])
        hi = np.concatenate([inf(qp['ubg'][rows]) - qp['g0'][rows], inf(qp['ubx'][keep])])
        fr = np.isinf(lo) & np.isinf(hi)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            ipm = qp_exact.solve(qp['P'][np.ix_(keep, keep)], qp['q'][keep], Ar[~fr], lo[~fr], hi[~fr])
        if ipm['status'] == 'solved':
            both += 1
            assert np.abs(ipm['x'] - z[keep]).max() <= 1e-7
    assert both >= B // 2
