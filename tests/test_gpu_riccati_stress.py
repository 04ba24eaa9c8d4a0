"""Stress parity of the Riccati kernel (hmpc_ric.hip) against the C port at
batch sizes where the rare paths run: the cached-column z and its sweep
fallback, drops, the overflow hand-off, both occupancy builds.

Per case: equal statuses for every instance and, where solved, |du| <= 1e-6,
|dx*| <= 1e-6 (x* feeds the next mpcontrol call, src/mpc_cvx_euler_3f.py:58,68)
and a relative objective error <= 1e-8.  x* is checked on its own: a sweep
defect once corrupted x* of overflowed instances while u* stayed right
(the DPP hazard).
Workloads: the bench sampler with the mu sweep and start-state noise scaled
up (x3 velocities, x2 rates) so that active sets are larger than the bench's."""
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


@pytest.mark.parametrize('variant,N,B,curve,kernel', [
    ('3f', 13, 2048, True, 'hmpc::ric_kernel<3, 2, 0, 0, 0>'),
    ('3f', 20, 4096, False, 'hmpc::ric_kernel<3, 2, 20, 38, 0>'),
    ('2f', 20, 2048, True, 'hmpc::ric_kernel<2, 2, 20, 38, 0>'),
    ('3f', 40, 1024, True, 'hmpc::ric_factor_kernel<3, 0, 0> + hmpc::ric_kernel<3, 1, 0, 0, 2>'),
    ('3f', 60, 1024, False, 'hmpc::ric_factor_kernel<3, 60, 47> + hmpc::ric_kernel<3, 1, 60, 47, 2>'),
    ('2f', 60, 1024, True, 'hmpc::ric_factor_kernel<2, 60, 47> + hmpc::ric_kernel<2, 1, 60, 47, 2>'),
])
def test_riccati_stress_vs_port(hm, variant, N, B, curve, kernel):
    import hmpc_plan
    from oracle import port
    inst = hmpc_plan.sample_instances(B, N, curve=curve, seed=100 + N, mu_sweep=(0.3, 1.2))
    rng = np.random.default_rng(N)
    inst['x_in'][:, 6:9] += rng.uniform(-0.4, 0.4, (B, 3))
    inst['x_in'][:, 9:12] += rng.uniform(-0.4, 0.4, (B, 3))
    inst['x_lin'][:, 0] = inst['x_in']
    c = hmpc_plan.runner_constants()
    cx = hm.Context(variant, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    assert cx.kernel_name == kernel
    gpu = cx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    cx.close()
    ref = port.solve_batch(variant, N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                           mu=inst['mu'], nthreads=16)
    assert np.array_equal(gpu['status'], ref['status']), np.argwhere(gpu['status'] != ref['status'])[:5]
    ok = ref['status'] == 0
    assert ok.mean() > 0.9
    assert np.abs(gpu['u'][ok] - ref['u'][ok]).max() <= 1e-6
    assert np.abs(gpu['x'][ok] - ref['x'][ok]).max() <= 1e-6
    rel = np.abs(gpu['obj'][ok] - ref['obj'][ok]) / np.maximum(np.abs(ref['obj'][ok]), 1.0)
    assert rel.max() <= 1e-8, rel.max()


def test_n60_small_batch_capacity(hm):
    """The Runner's horizon at small batches (B <= 3 workgroups per CU) runs the
    solve kernel with R's capacity 64 (round 6): the reference's own run has
    calls with up to 59 active rows, which capacity 47 sent to the slow
    generic overflow pass.  Checked against the port at B = 256, and the
    context reports the capacity and kernel of that solve."""
    import hmpc_plan
    from oracle import port
    N, B = 60, 256
    inst = hmpc_plan.sample_instances(B, N, curve=False, seed=160, mu_sweep=(0.3, 1.2))
    rng = np.random.default_rng(160)
    inst['x_in'][:, 6:9] += rng.uniform(-0.4, 0.4, (B, 3))
    inst['x_lin'][:, 0] = inst['x_in']
    c = hmpc_plan.runner_constants()
    cx = hm.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    gpu = cx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    assert cx.kernel_name == 'hmpc::ric_factor_kernel<3, 60, 47> + hmpc::ric_kernel<3, 1, 60, 64, 2>'
    assert cx.active_capacity == 64
    cx.close()
    ref = port.solve_batch('3f', N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                           mu=inst['mu'], nthreads=16)
    assert np.array_equal(gpu['status'], ref['status'])
    ok = ref['status'] == 0
    assert ok.mean() > 0.9
    assert np.abs(gpu['u'][ok] - ref['u'][ok]).max() <= 1e-6
    assert np.abs(gpu['x'][ok] - ref['x'][ok]).max() <= 1e-6
    rel = np.abs(gpu['obj'][ok] - ref['obj'][ok]) / np.maximum(np.abs(ref['obj'][ok]), 1.0)
    assert rel.max() <= 1e-8, rel.max()
