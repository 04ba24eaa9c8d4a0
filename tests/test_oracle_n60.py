"""The reference Runner's own configuration (run.py 3f --N_run=2000: N = 60,
src/robotrunner.py:46) pinned end to end on the CPU.

tests/golden/loop_3f_N60_config1.npz is the reference's Runner.run loop
(src/robotrunner.py:81-113) recorded by make_golden.py through the reference's
own Mpc.mpcontrol / build_qp (recording cvxpy stub, exact solve by
oracle/qp_exact).  Every one of its 100 calls (101 QP solves) is replayed here
through the C port (the second checker) with the reference's time-shift
semantics (src/mpc_cvx_euler_3f.py:49-62), and the previously misreported
last call through qp_exact itself.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
U_TOL = 1e-6


@pytest.fixture(scope='module')
def loop():
    return np.load(os.path.join(GOLDEN, 'loop_3f_N60_config1.npz'))


def call_inputs(g, c):
    """(x_in, x_lin, x_ref, pf, C) of call c's (last) solve; call 0 is the
    init double solve, whose first linearisation is [x_in; x_ref]."""
    N = int(g['N'])
    x_in = g['x_in'][c]
    x_ref = g[f'c{c}_x_ref']
    pf = g[f'c{c}_pf']
    C = g['C'][c]
    if c == 0:
        x_lin = np.vstack([x_in, x_ref])
    else:
        prev = g[f'c{c - 1}_xstar']
        x_lin = np.vstack([x_in, prev[2:], prev[-1:]])
        assert x_lin.shape == (N + 1, 12)
    return x_in, x_lin, x_ref, pf, C


def test_fixture_is_the_full_reference_run(loop):
    g = loop
    assert int(g['N']) == 60 and int(g['N_run']) == 2000
    assert len(g['k']) == 100 and int(g['n_detail']) == 100
    assert g['init'][0] and not g['init'][1:].any()
    np.testing.assert_array_equal(g['k'], np.arange(0, 2000, 20))


def test_port_replays_every_reference_call(loop):
    from oracle import port
    g = loop
    N = int(g['N'])
    for c in range(len(g['k'])):
        x_in, x_lin, x_ref, pf, C = call_inputs(g, c)
        if c == 0:   # init pass 1 (3f :50-58)
            r = port.solve_batch('3f', N, x_in[None], x_lin[None], x_ref[None], pf[None], C[None])
            assert r['status'][0] == 0
            x_lin = r['x'][0]
        r = port.solve_batch('3f', N, x_in[None], x_lin[None], x_ref[None], pf[None], C[None])
        assert r['status'][0] == 0, c
        assert np.abs(r['u'][0] - g[f'c{c}_U']).max() <= U_TOL, c
        assert np.abs(r['x'][0] - g[f'c{c}_xstar']).max() <= U_TOL, c


def test_qp_exact_solves_the_last_call(loop):
    """Call 100 (the 101st solve): the round-1 oracle's cold-start IPM
    diverged there and reported it primal-infeasible; the reference's own
    x* satisfies every row of the reference-built problem."""
    from oracle import hmpc_oracle as ho
    g = loop
    N = int(g['N'])
    c = len(g['k']) - 1
    x_in, x_lin, x_ref, pf, C = call_inputs(g, c)
    p = ho.MpcParams.runner('3f', N)
    r = ho.solve_instance(p, x_in, x_lin, x_ref, pf, C)
    assert r['status'] == 'solved'
    assert np.abs(r['u'] - g[f'c{c}_U']).max() <= U_TOL
    qp = r['qp']
    z = np.concatenate([g[f'c{c}_xstar'].ravel(), g[f'c{c}_U'].ravel()])
    Az = qp['A'] @ z
    assert max(np.max(qp['l'] - Az), np.max(Az - qp['u'])) <= 1e-9


def test_min_violation_certificate():
    """qp_exact reports primal_infeasible only with an LP certificate: the
    least uniform violation t* of l <= A z <= u is > 0."""
    import hmpc_plan as hp
    from oracle import hmpc_oracle as ho
    from oracle import qp_exact
    N = 20
    inst = hp.sample_instances(2, N, curve=False, seed=3)
    p = ho.MpcParams.runner('3f', N)
    _, _, Gd = ho.constant_matrices(p)
    x_in = inst['x_in'].copy()
    x_in[1, 2] = 0.05                   # z_0 < 0.1: infeasible
    for i, feasible in ((0, True), (1, False)):
        Ad, Bd = ho.gen_dt_dynamics(p, inst['x_lin'][i], inst['pf'][i])
        qp = ho.build_qp(p, x_in[i], inst['x_ref'][i], Ad, Bd, Gd, inst['C'][i])
        t, z = qp_exact.min_violation(qp['A'], qp['l'], qp['u'])
        if feasible:
            assert t <= 1e-9 and z is not None
        else:
            assert t > 1e-3
