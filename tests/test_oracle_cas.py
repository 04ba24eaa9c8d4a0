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
