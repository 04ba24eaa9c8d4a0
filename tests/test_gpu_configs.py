"""Full-configuration parity as a test, not only as the bench's parity_sample:
BASELINE configs[2] (3f, --curve, N = 10) and configs[1] (2f, straight,
N = 10) at B = 4096 of the bench workload, every instance against the C port
(oracle/hmpc_port.c: an independent condensing and solver, pinned to the
reference-built problem data): equal statuses, |du| <= 1e-6, objective
1e-9 relative, x* 1e-6.  B = 4096 takes the longest-first class order
(hmpc_set_order auto); B = 16384 of configs[2] the index order, so both
dense-split launch forms (bucket lists and plain class lists) are covered, and
B = 32768 the swing-first launch (the all-swing class before the full class
on the caller's stream, HMPC_SWING_FIRST_B).  Reference: src/mpc_cvx_euler_3f.py:96-160,
src/mpc_cvx_euler_2f.py:96-158."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def hm():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    return hmpc


@pytest.mark.parametrize('variant,curve,B,order', [('3f', True, 4096, 'auto'), ('3f', True, 16384, 'auto'),
                                                   ('3f', True, 4096, 'index'), ('2f', False, 4096, 'auto'),
                                                   ('3f', True, 32768, 'auto')])
def test_config_vs_port(hm, variant, curve, B, order):
    import hmpc_plan
    from oracle import port
    N = 10
    inst = hmpc_plan.sample_instances(B, N, curve=curve, seed=2024)   # the bench's seed
    c = hmpc_plan.runner_constants()
    cx = hm.Context(variant, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    cx.set_order(order)
    g = cx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    cx.close()
    ref = port.solve_batch(variant, N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                           mu=inst['mu'], nthreads=16)
    assert np.array_equal(g['status'], ref['status'])
    ok = ref['status'] == 0
    assert ok.mean() > 0.99
    assert np.abs(g['u'][ok] - ref['u'][ok]).max() <= 1e-6
    rel = np.abs(g['obj'][ok] - ref['obj'][ok]) / np.abs(ref['obj'][ok])
    assert rel.max() <= 1e-9, rel.max()
    assert np.abs(g['x'][ok] - ref['x'][ok]).max() <= 1e-6
