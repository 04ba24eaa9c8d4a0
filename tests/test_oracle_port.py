"""The oracle's C port (oracle/hmpc_port.c: dense condensing + classic
Goldfarb-Idnani) against the golden fixtures recorded from the reference's own
build_qp, and against the numpy oracle on freshly drawn instances.  CPU only."""
import glob
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURES = sorted(glob.glob(os.path.join(ROOT, 'tests', 'golden', 'qp_*.npz')))


@pytest.fixture(scope='module')
def port():
    subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'oracle')])
    from oracle import port as pt
    pt.load()
    return pt


@pytest.mark.parametrize('path', FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
@pytest.mark.parametrize('uref', ['aliased', 'per_stage'])
def test_port_matches_golden_optimum(port, path, uref):
    d = np.load(path)
    tag = 'alias' if uref == 'aliased' else 'stage'
    N = int(d['N'])
    r = port.solve_batch(str(d['variant']), N, d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'],
                         mu=d['mu'], uref_mode=uref, nthreads=4)
    ok = d[f'status_{tag}'] == 0
    assert np.array_equal(r['status'] == 0, ok), (r['status'], d[f'status_{tag}'])
    assert np.abs(r['u'][ok] - d[f'u_{tag}'][ok]).max() < 1e-7
    ref = d[f'obj_{tag}'][ok]
    assert (np.abs(r['obj'][ok] - ref) / np.abs(ref)).max() < 1e-9


@pytest.mark.parametrize('variant,N,curve', [('3f', 10, True), ('2f', 10, False), ('3f', 20, True),
                                             ('3f', 5, False)])
def test_port_matches_numpy_oracle(port, variant, N, curve):
    import hmpc_plan
    from oracle import hmpc_oracle as ho
    inst = hmpc_plan.sample_instances(12, N, curve=curve, seed=77, mu_sweep=(0.3, 1.2))
    r = port.solve_batch(variant, N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'],
                         inst['C'], mu=inst['mu'])
    for i in range(12):
        p = ho.MpcParams.runner(variant, N, mu=float(inst['mu'][i]))
        s = ho.solve_instance(p, inst['x_in'][i], inst['x_lin'][i], inst['x_ref'][i], inst['pf'][i],
                              inst['C'][i])
        assert (s['status'] == 'solved') == (r['status'][i] == 0)
        if s['status'] == 'solved':
            assert np.abs(r['u'][i] - s['u']).max() < 1e-7
            assert abs(r['obj'][i] - s['obj']) <= 1e-9 * abs(s['obj'])
            assert np.allclose(r['x'][i], s['x'], atol=1e-9)


def test_port_flags_infeasible_and_is_thread_invariant(port):
    import hmpc_plan
    inst = hmpc_plan.sample_instances(64, 10, curve=True, seed=3)
    inst['x_in'][5, 2] = 0.05            # z0 < 0.1: infeasible
    args = [inst[k] for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C')]
    r1 = port.solve_batch('3f', 10, *args, nthreads=1)
    r8 = port.solve_batch('3f', 10, *args, nthreads=8)
    assert r1['status'][5] == 2 and (np.delete(r1['status'], 5) == 0).all()
    for k in ('u', 'x', 'obj', 'status'):
        assert np.array_equal(r1[k], r8[k])
