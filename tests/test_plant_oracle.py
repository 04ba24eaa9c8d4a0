"""The plant/closed-loop oracle (oracle/hmpc_plant.py) against the reference's
own outputs: tests/golden/plant.npz (dynamics_ct, rk4_normalized, convert of
src/robotrunner.py on 16 random states) and loop_3f_N10.npz (50 MPC periods
of Runner.run, src/robotrunner.py:81-113)."""
import os

import numpy as np

from oracle import hmpc_oracle as ho
from oracle import hmpc_plant as pl

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def test_plant_functions_match_reference():
    c = ho.runner_constants()
    d = np.load(os.path.join(GOLDEN, 'plant.npz'))
    for i in range(len(d['X'])):
        dX = pl.dynamics_ct(d['X'][i], d['U'][i], d['pf'][i], c['m'], c['g'], c['J'], c['rh'])
        np.testing.assert_allclose(dX, d['dX'][i], rtol=1e-13, atol=1e-12)
        Xn = pl.rk4_normalized(d['X'][i], d['U'][i], d['pf'][i], 1e-3, c['m'], c['g'], c['J'],
                               c['rh'])
        np.testing.assert_allclose(Xn, d['Xn'][i], rtol=0, atol=1e-14)
        np.testing.assert_allclose(pl.convert(d['X'][i]), d['x_conv'][i], rtol=0, atol=1e-14)


def test_closed_loop_matches_reference_runner():
    g = np.load(os.path.join(GOLDEN, 'loop_3f_N10.npz'))
    n = int(len(g['k']))
    r = pl.run_closed_loop(N=int(g['N']), N_run=int(g['N_run']), curve=bool(g['curve']),
                           n_periods=n)
    assert [c['k'] for c in r['calls']] == list(g['k'])
    np.testing.assert_array_equal(np.array([c['C'] for c in r['calls']]), g['C'])
    np.testing.assert_allclose(np.array([c['x_in'] for c in r['calls']]), g['x_in'], rtol=0,
                               atol=1e-12)
    np.testing.assert_allclose(np.array([c['U'][0] for c in r['calls']]), g['U0'], rtol=0,
                               atol=1e-9)
    np.testing.assert_allclose(r['X_traj'][::20], g['X_traj_mpc'], rtol=0, atol=1e-12)
