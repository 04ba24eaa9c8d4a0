"""The dense split's all-swing class (csrc/hmpc_swing.hip): windows whose
every stage swings fix every force (src/mpc_cvx_euler_3f.py:134-136), leave
the 3N torques under box rows (:123-128), and are solved two per wavefront,
one per 32-lane half.

Pinned here, each against the C port (oracle/hmpc_port.c):
  * distinct and duplicated pairings, odd list lengths (the last block's
    upper half then repeats the lower half's instance and stores nothing);
  * a half's result does not depend on its partner: the same instances in
    shuffled batches (other partners, other halves) are bit-identical;
  * 2f windows (the same torque QP), the mpcontrol linearisations (init pass
    x_lin = [x_in; x_ref], time shift of x_prev), infeasible z rows.
"""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

KEYS = ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')


@pytest.fixture(scope='module')
def hm():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    return hmpc


def swing_pool(variant, curve, seed, n, mu_sweep=(0.3, 1.2)):
    import hmpc_plan
    a = hmpc_plan.sample_instances(8 * n + 4096, 10, curve=curve, seed=seed, mu_sweep=mu_sweep)
    sw = np.where((a['C'] != 0).sum(1) == 0)[0][:n]
    assert len(sw) == n
    return {k: np.ascontiguousarray(a[k][sw]) for k in KEYS}


def take(inst, idx):
    return {k: np.ascontiguousarray(inst[k][idx]) for k in KEYS}


def solve(hm, variant, inst, order='index'):
    import hmpc_plan
    c = hmpc_plan.runner_constants()
    cx = hm.Context(variant, 10, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    cx.set_order(order)
    r = cx.solve_host(*(inst[k] for k in KEYS[:5]), mu=inst['mu'])
    # (index order: the all-swing class ran; longest-first: the compacted one)
    assert ('swing_kernel' in cx.kernel_name) == (order == 'index'), (order, cx.kernel_name)
    cx.close()
    return r


def port(variant, inst):
    from oracle import port as p
    return p.solve_batch(variant, 10, *(inst[k] for k in KEYS[:5]), mu=inst['mu'], nthreads=16)


def check(g, ref, tol=1e-6, swing=True):
    assert np.array_equal(g['status'], ref['status'])
    ok = ref['status'] == 0
    assert np.abs(g['u'][ok] - ref['u'][ok]).max() <= tol
    rel = np.abs(g['obj'][ok] - ref['obj'][ok]) / np.abs(ref['obj'][ok])
    assert rel.max() <= 1e-9, rel.max()
    assert np.abs(g['x'][ok] - ref['x'][ok]).max() <= tol
    if swing:
        assert (g['u'][ok][..., :3] == 0).all()   # every force fixed


@pytest.mark.parametrize('variant,curve', [('3f', True), ('3f', False), ('2f', False)])
def test_swing_vs_port(hm, variant, curve):
    inst = swing_pool(variant, curve, 31, 1024)
    ref = port(variant, inst)
    # the pool has windows whose box rows bind (active-set iterations)
    assert (ref['iters'] > 0).any() or not curve   # (straight windows: box rows never bind)
    for order in ('index', 'auto'):   # (auto at B = 1024: longest-first, no swing class)
        check(solve(hm, variant, inst, order), ref)


@pytest.mark.parametrize('B', [1, 2, 3, 63, 65, 511])
def test_swing_odd_lists(hm, B):
    inst = take(swing_pool('3f', True, 32, 512), slice(0, B))
    check(solve(hm, '3f', inst), port('3f', inst))


def test_swing_partner_invariance(hm):
    """The same instances with other partners and in the other half: results
    bit for bit equal (one classify block keeps the list in index order, so
    the pairing is (0, 1), (2, 3), ...)."""
    inst = swing_pool('3f', True, 33, 512)
    ref = port('3f', inst)
    base = solve(hm, '3f', inst)
    check(base, ref)
    rng = np.random.default_rng(5)
    for rep in range(3):
        perm = rng.permutation(512)
        g = solve(hm, '3f', take(inst, perm))
        for k in ('u', 'x', 'obj', 'status', 'iters'):
            assert np.array_equal(g[k], base[k][perm]), (rep, k)
    # each instance paired with itself
    dup = np.repeat(np.arange(256), 2)
    g = solve(hm, '3f', take(inst, dup))
    for k in ('u', 'x', 'obj', 'status', 'iters'):
        assert np.array_equal(g[k], base[k][dup]), k


def test_swing_mixed_batch_invariance(hm):
    """In a mixed batch (all three classes) the all-swing instances solve as
    they do alone, and a shuffle of the whole batch permutes the results."""
    import hmpc_plan
    a = hmpc_plan.sample_instances(4096, 10, curve=True, seed=34, mu_sweep=(0.3, 1.2))
    inst = {k: np.ascontiguousarray(a[k]) for k in KEYS}
    base = solve(hm, '3f', inst)
    check(base, port('3f', inst), swing=False)
    perm = np.random.default_rng(6).permutation(4096)
    g = solve(hm, '3f', take(inst, perm))
    for k in ('u', 'x', 'obj', 'status', 'iters'):
        assert np.array_equal(g[k], base[k][perm]), k


def test_swing_mpcontrol_modes(hm):
    """mpcontrol's linearisations (3f :52-53 init, :59-62 shift) on all-swing
    windows: the device passes equal the same solves with the host building
    x_lin."""
    import hmpc_plan
    inst = swing_pool('3f', True, 35, 256)
    B = 256
    c = hmpc_plan.runner_constants()
    cx = hm.Context('3f', 10, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    cx.set_order('index')   # (the all-swing class)
    d = {k: torch.from_numpy(inst[k]).cuda() for k in ('x_in', 'x_ref', 'pf', 'C', 'mu')}
    xp = torch.zeros((B, 11, 12), dtype=torch.float64, device='cuda')
    o1 = cx.mpcontrol_device(True, d['x_in'], d['x_ref'], d['pf'], d['C'], xp, mu=d['mu'])
    x1 = xp.clone()
    o2 = cx.mpcontrol_device(False, d['x_in'], d['x_ref'], d['pf'], d['C'], xp, mu=d['mu'])
    torch.cuda.synchronize()
    x_lin = torch.cat([d['x_in'][:, None], x1[:, 2:], x1[:, -1:]], dim=1).cpu().numpy()
    r = cx.solve_host(inst['x_in'], x_lin, inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    cx.close()
    assert (o1['status'] == 0).all()
    assert np.array_equal(r['status'], o2['status'].cpu().numpy())
    np.testing.assert_array_equal(r['u'], o2['u'].cpu().numpy())
    sh = dict(inst, x_lin=x_lin)
    check(r, port('3f', sh))


def test_swing_infeasible_heights(hm):
    """z >= 0.1 (:129) has zero normals in an all-swing window: a start below
    it, or a free fall through it, is infeasible like the port says."""
    inst = swing_pool('3f', True, 36, 64)
    inst['x_in'][:16, 2] = 0.05          # z_0 below the bound
    inst['x_in'][16:32, 8] = -6.0        # falling fast: a later z_k below it
    inst['x_lin'][:, 0] = inst['x_in']
    ref = port('3f', inst)
    assert (ref['status'][:32] == 2).all()
    check(solve(hm, '3f', inst), ref)
