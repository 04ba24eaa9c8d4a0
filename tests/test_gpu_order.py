"""Instance order (hmpc_set_order): the dense split's class lists and the
Riccati kernel's work queue served longest-first (stance-stage buckets, most
stance stages first) or in batch index order.  Each instance is solved by the
same kernel either way -- except the dense N = 10 all-swing windows, which the
swing class (hmpc_swing.hip) solves in index order and the compacted class in
the longest-first queue -- so the results must be bit-identical between the
orders (those windows: within 1e-9), and equal to the C port's; the overflow pass and the self-resetting
bucket counters must survive alternating orders on one context."""
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


def context(hm, variant, N):
    import hmpc_plan
    c = hmpc_plan.runner_constants()
    return hm.Context(variant, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])


def same_across_orders(a, b, C, N):
    """a (longest-first) and b (index order) bit-identical, except the dense
    N = 10 all-swing windows (another kernel under 'index': the swing class),
    which agree within 1e-9 with equal statuses."""
    B = len(a['status'])
    sw = np.zeros(B, bool)
    if N == 10:
        sw = ~(np.asarray(C).reshape(B, -1)[:, :N] != 0).any(axis=1)
    for k in a:
        assert np.array_equal(a[k][~sw], b[k][~sw]), k
    assert np.array_equal(a['status'][sw], b['status'][sw])
    ok = sw & (b['status'] == 0)
    for k in ('u', 'x'):
        assert np.abs(a[k][ok] - b[k][ok]).max(initial=0.0) <= 1e-9, k
    assert (np.abs(a['obj'][ok] - b['obj'][ok]) <= 1e-12 * np.abs(b['obj'][ok])).all()


@pytest.mark.parametrize('variant,N,B,curve,musweep', [
    ('3f', 10, 3000, True, False),     # dense split, 3f
    ('2f', 10, 2048, False, False),    # dense split, 2f (5N-wide full class)
    ('3f', 20, 1500, False, True),     # Riccati, 2 waves / SIMD
    ('3f', 60, 300, False, False),     # Riccati, the Runner's horizon
])
def test_orders_agree_bit_for_bit(hm, variant, N, B, curve, musweep):
    import hmpc_plan
    from oracle import port
    inst = hmpc_plan.sample_instances(B, N, curve=curve, seed=77 + N,
                                      mu_sweep=(0.3, 1.2) if musweep else None)
    cx = context(hm, variant, N)
    args = (inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'])
    res = {}
    # alternate on one context: the bucket / class counters reset themselves
    for order in ('longest_first', 'index', 'longest_first', 'auto'):
        cx.set_order(order)
        r = cx.solve_host(*args, mu=inst['mu'])
        if order in res:
            for k in r:
                assert np.array_equal(r[k], res[order][k]), (order, k)
        res.setdefault(order, r)
    cx.close()
    a, b = res['longest_first'], res['index']
    same_across_orders(a, b, inst['C'], N)
    n = min(B, 256)
    ref = port.solve_batch(variant, N, *(v[:n] for v in args), mu=inst['mu'][:n], nthreads=16)
    assert np.array_equal(a['status'][:n], ref['status'])
    ok = ref['status'] == 0
    assert np.abs(a['u'][:n][ok] - ref['u'][ok]).max() <= 1e-6


def test_longest_first_with_overflow(hm):
    """Instances whose active set outgrows the kernel (forced by large initial
    velocities) go to the overflow pass under either order."""
    import hmpc_plan
    from oracle import port
    N, B = 10, 512
    inst = hmpc_plan.sample_instances(B, N, curve=True, seed=5, mu_sweep=(0.2, 0.2))
    rng = np.random.default_rng(5)
    inst['x_in'][:, 9:12] += rng.choice([-1, 1], (B, 3)) * rng.uniform(0.7, 1.0, (B, 3)) * 50.0
    inst['x_in'][:, 6:8] += rng.choice([-1, 1], (B, 2)) * rng.uniform(0.7, 1.0, (B, 2)) * 8.0
    inst['x_lin'][:, 0] = inst['x_in']
    args = (inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'])
    cx = context(hm, '3f', N)
    cx.set_order('longest_first')
    a = cx.solve_host(*args, mu=inst['mu'])
    cx.set_order('index')
    b = cx.solve_host(*args, mu=inst['mu'])
    cx.close()
    same_across_orders(a, b, inst['C'], N)
    ref = port.solve_batch('3f', N, *args, mu=inst['mu'], nthreads=16)
    assert np.array_equal(a['status'], ref['status'])
    ok = ref['status'] == 0
    assert np.abs(a['u'][ok] - ref['u'][ok]).max() <= 1e-6


def test_set_order_rejects_unknown(hm):
    cx = context(hm, '3f', 10)
    with pytest.raises(hm.HmpcError):
        cx._check(cx._lib.hmpc_set_order(cx._h, 7), 'hmpc_set_order')
    cx.close()


@pytest.mark.parametrize('N', [10, 20, 40])
def test_ragged_small_batches(hm, N):
    """Batches of 1, 2, 3, 63, 65 and 1025 instances through every kernel
    path small batches take: the dense split with longest-first buckets
    (N = 10; a class may be empty), the two-wave Riccati queue (N = 20), the
    factorisation kernel + one-wave Riccati queue (N = 40).  Each instance
    must come out as in one large batch, bit for bit, and match the port."""
    import hmpc_plan
    from oracle import port
    inst = hmpc_plan.sample_instances(1025, N, curve=True, seed=300 + N)
    keys = ('x_in', 'x_lin', 'x_ref', 'pf', 'C')
    cx = context(hm, '3f', N)
    whole = cx.solve_host(*(inst[k] for k in keys), mu=inst['mu'])
    for b in (1, 2, 3, 63, 65):
        part = cx.solve_host(*(inst[k][:b] for k in keys), mu=inst['mu'][:b])
        for k in part:
            assert np.array_equal(part[k], whole[k][:b]), (b, k)
    cx.close()
    n = 65
    ref = port.solve_batch('3f', N, *(inst[k][:n] for k in keys), mu=inst['mu'][:n], nthreads=16)
    assert np.array_equal(whole['status'][:n], ref['status'])
    ok = ref['status'] == 0
    assert np.abs(whole['u'][:n][ok] - ref['u'][ok]).max() <= 1e-6
