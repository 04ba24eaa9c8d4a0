"""The oracle (oracle/hmpc_oracle.py) against the reference's own recorded QPs.

Fixtures come from tests/golden/make_golden.py, which ran the REFERENCE's
``Mpc.gen_dt_dynamics`` / ``Mpc.build_qp`` (src/mpc_cvx_euler_{3f,2f}.py)
through a recording cvxpy stub.  The oracle must reproduce that problem data
exactly (Ad, Bd, P, q, r, A, l, u), for both u_ref semantics, and its exact
solver must return KKT-certified optima of it.
"""
import glob
import os

import numpy as np
import pytest

from oracle import hmpc_oracle as ho
from oracle import qp_exact

FIXTURES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), 'golden', 'qp_*.npz')))


def params_of(d, i):
    return ho.MpcParams(variant=str(d['variant']), N=int(d['N']), t=0.02, m=7.5, g=9.807,
                        mu=float(d['mu'][i]), Jinv=d['Jinv'], rh=d['rh'])


@pytest.mark.parametrize('path', FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
def test_problem_data_bit_exact(path):
    d = np.load(path)
    for i in range(int(d['n_full'])):
        p = params_of(d, i)
        Ad, Bd = ho.gen_dt_dynamics(p, d['x_lin'][i], d['pf'][i])
        assert np.array_equal(Ad, d['Ad'][i])
        assert np.array_equal(Bd, d['Bd'][i])
        _, _, Gd = ho.constant_matrices(p)
        for tag, mode in (('alias', 'aliased'), ('stage', 'per_stage')):
            qp = ho.build_qp(p, d['x_in'][i], d['x_ref'][i], Ad, Bd, Gd, d['C'][i], mode)
            assert np.array_equal(np.diag(qp['P']), d[f'i{i}_{tag}_Pdiag'])
            assert np.count_nonzero(qp['P'] - np.diag(np.diag(qp['P']))) == 0
            assert np.array_equal(qp['q'], d[f'i{i}_{tag}_q'])
            assert qp['r'] == float(d[f'i{i}_{tag}_r'])
        shape = tuple(d[f'i{i}_A_shape'])
        A = np.zeros(shape)
        A[d[f'i{i}_A_row'], d[f'i{i}_A_col']] = d[f'i{i}_A_val']
        assert np.array_equal(qp['A'], A)
        assert np.array_equal(qp['l'], d[f'i{i}_l'])
        assert np.array_equal(qp['u'], d[f'i{i}_u'])


@pytest.mark.parametrize('path', FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
def test_exact_solutions_certified(path):
    d = np.load(path)
    cert = d['cert_alias']
    ok = d['status_alias'] == 0
    assert ok.mean() > 0.8
    assert np.nanmax(cert[ok]) < 1e-9
    # re-solve a few with the oracle: identical optimum
    for i in np.where(ok)[0][:3]:
        s = ho.solve_instance(params_of(d, i), d['x_in'][i], d['x_lin'][i], d['x_ref'][i],
                              d['pf'][i], d['C'][i], 'aliased')
        assert s['status'] == 'solved'
        assert np.abs(s['u'] - d['u_alias'][i]).max() < 1e-9
        assert abs(s['obj'] - d['obj_alias'][i]) <= 1e-9 * abs(d['obj_alias'][i])
        # the optimum satisfies the reference's constraints directly
        x, u = s['x'], s['u']
        assert np.all(np.abs(u[:, 3:5]) <= 7.78 + 1e-9) and np.all(np.abs(u[:, 5]) <= 4 + 1e-9)
        assert np.all(x[:-1, 2] >= 0.1 - 1e-9)
        assert np.allclose(x[0], d['x_in'][i], atol=1e-12)


def test_aliasing_changes_the_problem():
    """The u_ref aliasing is visible in the data."""
    d = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'qp_3f_N10_straight.npz'))
    C = d['C']
    mixed = np.where((C.min(axis=1) == 0) & (C.max(axis=1) == 1))[0]
    assert len(mixed) > 0
    diff = [np.abs(d['u_alias'][i] - d['u_stage'][i]).max() for i in mixed
            if d['status_alias'][i] == 0 and d['status_stage'][i] == 0]
    assert max(diff) > 1.0


def test_qp_exact_small_known_answer():
    """min 1/2|z|^2 - [1,1]'z  s.t. z1 + z2 <= 1, -5 <= z <= 5  ->  z = (0.5, 0.5)."""
    P = np.eye(2)
    q = -np.ones(2)
    A = np.array([[1.0, 1.0], [1.0, 0.0], [0.0, 1.0]])
    l = np.array([-np.inf, -5, -5])
    u = np.array([1.0, 5, 5])
    s = qp_exact.solve(P, q, A, l, u)
    assert s['status'] == 'solved'
    assert np.allclose(s['x'], [0.5, 0.5], atol=1e-12)


def test_qp_exact_detects_infeasible():
    P = np.eye(1)
    q = np.zeros(1)
    A = np.array([[1.0], [1.0]])
    l = np.array([1.0, -np.inf])
    u = np.array([np.inf, 0.0])
    s = qp_exact.solve(P, q, A, l, u)
    assert s['status'] == 'primal_infeasible'
