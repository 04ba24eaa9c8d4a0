"""The active-set capacity cliff is gone: instances whose optimal active set
is larger than the main kernel's capacity (hmpc_active_capacity: dense N = 10
kernel 20 in registers; Riccati kernel ric_qcap(N) in LDS -- 50 at N = 10,
47 at N = 60)
are handed to the overflow pass (capacity 6N, R in global memory) and come
back solved, equal to the C port, instead of HMPC_NUMERICAL.

Adversarial instances: mu = 0.2..0.3 and large start-state errors (angular
rates +-8..50 rad/s, horizontal velocity +-1.4..8 m/s) saturate the torque box and
the friction pyramid over most stages.  The active-set size at the optimum is
counted on the CPU from the port's solution against the reference-form
constraint rows (oracle/hmpc_oracle.build_qp), so the test proves the cases
really exceed the capacities it claims to cover.
"""
import os

import numpy as np
import pytest
from conftest import DENSE10_3F_LPT

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

U_TOL = 1e-6


@pytest.fixture(scope='module')
def hm():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    return hmpc


def adversarial(B, N, seed, wscale, vscale, mu=0.3):
    import hmpc_plan as hp
    inst = hp.sample_instances(B, N, curve=True, seed=seed, mu_sweep=(mu, mu))
    rng = np.random.default_rng(seed)
    inst['x_in'][:, 9:12] += rng.choice([-1, 1], (B, 3)) * rng.uniform(0.7, 1.0, (B, 3)) * wscale
    inst['x_in'][:, 6:8] += rng.choice([-1, 1], (B, 2)) * rng.uniform(0.7, 1.0, (B, 2)) * vscale
    inst['x_in'][:, 3:5] += rng.uniform(-0.4, 0.4, (B, 2))
    inst['x_lin'][:, 0] = inst['x_in']
    return inst


def active_rows(N, inst, ref, i):
    """Inequality rows of the reference-built QP active at the port's optimum."""
    from oracle import hmpc_oracle as ho
    p = ho.MpcParams.runner('3f', N, mu=float(inst['mu'][i]))
    _, _, Gd = ho.constant_matrices(p)
    Ad, Bd = ho.gen_dt_dynamics(p, inst['x_lin'][i], inst['pf'][i])
    qp = ho.build_qp(p, inst['x_in'][i], inst['x_ref'][i], Ad, Bd, Gd, inst['C'][i])
    z = np.concatenate([ref['x'][i].ravel(), ref['u'][i].ravel()])
    Az = qp['A'] @ z
    ineq = qp['l'] != qp['u']
    act = ineq & ((np.abs(Az - qp['l']) < 1e-7) | (np.abs(Az - qp['u']) < 1e-7))
    return int(act.sum())


def check_x_obj(gpu, ref):
    """x* (the next call's linearisation, src/mpc_cvx_euler_3f.py:58,68) and
    the objective of an overflowed instance come from the overflow pass."""
    assert np.abs(gpu['x'] - ref['x']).max() <= U_TOL
    rel = np.abs(gpu['obj'] - ref['obj']) / np.maximum(np.abs(ref['obj']), 1.0)
    assert rel.max() <= 1e-8, rel.max()


def solve_both(hm, N, inst, precision):
    import hmpc_plan
    from oracle import port
    c = hmpc_plan.runner_constants()
    cx = hm.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                    precision=precision)
    gpu = cx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    kernel = cx.kernel_name
    cap = cx.active_capacity
    cx.close()
    ref = port.solve_batch('3f', N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                           mu=inst['mu'], nthreads=16)
    return gpu, ref, kernel, cap


@pytest.mark.parametrize('precision,kernel', [('f64', DENSE10_3F_LPT),   # (B = 48: longest-first)
                                             ('f64_riccati', 'hmpc::ric_kernel<3, 2, 0, 0, 0>')])
def test_overflow_n10(hm, precision, kernel):
    N, B = 10, 48
    inst = adversarial(B, N, 2, 50.0, 8.0, mu=0.2)   # optimal active sets up to 55 of 60
    gpu, ref, k, cap = solve_both(hm, N, inst, precision)
    if 'HMPC_LIB' not in os.environ:   # (an A/B build may dispatch other classes)
        assert k == kernel
    assert (ref['status'] == 0).all()
    assert np.array_equal(gpu['status'], ref['status'])
    assert np.abs(gpu['u'] - ref['u']).max() <= U_TOL
    check_x_obj(gpu, ref)
    nact = [active_rows(N, inst, ref, i) for i in range(B)]
    assert max(nact) > cap, nact


def test_overflow_n60(hm):
    N, B = 60, 24
    inst = adversarial(B, N, 2, 12.0, 2.0)
    gpu, ref, k, cap = solve_both(hm, N, inst, 'f64')
    # (a small batch: the capacity-64 solve kernel, round 6)
    assert k == 'hmpc::ric_factor_kernel<3, 60, 47> + hmpc::ric_kernel<3, 1, 60, 64, 2>'
    assert cap == 64
    assert (ref['status'] == 0).all()
    assert np.array_equal(gpu['status'], ref['status'])
    assert np.abs(gpu['u'] - ref['u']).max() <= U_TOL
    check_x_obj(gpu, ref)
    nact = np.array([active_rows(N, inst, ref, i) for i in range(B)])
    assert (nact > cap).sum() >= 8, (cap, nact)    # the overflow pass
    assert ((nact > 47) & (nact <= cap)).any(), nact   # beyond the large-batch capacity, in the main pass


def test_overflow_mpcontrol_shift_in_place(hm):
    """mpcontrol's time-shift pass reads x_prev and writes x* into the same
    buffer: an overflowed instance's main pass must leave x_prev intact for
    the overflow pass.  Two calls (init, then shift) against the drop-in
    replay with host-side linearisation."""
    import hmpc_plan
    N, B = 10, 16
    inst = adversarial(B, N, 3, 30.0, 5.0)
    c = hmpc_plan.runner_constants()
    cx = hm.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda()
         for k in ('x_in', 'x_ref', 'pf', 'C', 'mu')}
    xp = torch.zeros((B, N + 1, 12), dtype=torch.float64, device='cuda')
    o1 = cx.mpcontrol_device(True, d['x_in'], d['x_ref'], d['pf'], d['C'], xp, mu=d['mu'])
    x1 = xp.clone()
    o2 = cx.mpcontrol_device(False, d['x_in'], d['x_ref'], d['pf'], d['C'], xp, mu=d['mu'])
    torch.cuda.synchronize()
    assert (o1['status'] == 0).all() and (o2['status'] == 0).all()
    # the same second solve from the host: linearisation = time shift of x1
    x_lin = torch.cat([d['x_in'][:, None], x1[:, 2:], x1[:, -1:]], dim=1).cpu().numpy()
    r = cx.solve_host(inst['x_in'], x_lin, inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    cx.close()
    assert np.array_equal(r['status'], o2['status'].cpu().numpy())
    np.testing.assert_array_equal(r['u'], o2['u'].cpu().numpy())


@pytest.mark.parametrize('N', [10, 20])
def test_counters_reset_between_solves(hm, N):
    """The overflow pass zeroes [overflow count | Riccati instance counter] at
    its end instead of a memset before every solve (hmpc_ric.hip,
    ric_overflow_kernel).  Back-to-back solves on ONE context -- an
    overflowing batch, a normal one, the overflowing one again, on the device
    entry point and the host one -- must equal fresh-context solves bit for
    bit; a stale counter would skip instances or re-solve stale list ids."""
    import hmpc_plan
    c = hmpc_plan.runner_constants()
    adv = adversarial(48, N, 2, 50.0, 8.0, mu=0.2)   # overflows (test_overflow_n10)
    nor = hmpc_plan.sample_instances(300, N, curve=True, seed=9)
    keys = ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')

    def ctx():
        return hm.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])

    def dev_solve(cx, inst):
        d = {k: torch.from_numpy(np.ascontiguousarray(inst[k])).cuda() for k in keys}
        o = cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
        torch.cuda.synchronize()
        return {k: o[k].cpu().numpy() for k in ('u', 'obj', 'status')}

    def host_solve(cx, inst):
        r = cx.solve_host(*(inst[k] for k in keys[:5]), mu=inst['mu'])
        return {k: r[k] for k in ('u', 'obj', 'status')}

    fresh = {}
    for name, inst in (('adv', adv), ('nor', nor)):
        cx = ctx()
        fresh[name] = dev_solve(cx, inst)
        cx.close()
    assert (fresh['nor']['status'] == 0).all()
    cx = ctx()
    seq = [('adv', dev_solve), ('nor', dev_solve), ('adv', host_solve), ('nor', host_solve),
           ('adv', dev_solve), ('adv', dev_solve), ('nor', dev_solve)]
    for name, fn in seq:
        r = fn(cx, adv if name == 'adv' else nor)
        for k in ('u', 'obj', 'status'):
            assert np.array_equal(r[k], fresh[name][k]), (name, fn.__name__, k)
    cx.close()


def test_overflow_n60_second_tier(hm):
    """A large N = 60 batch (B = 1024: the capacity-47 solve kernel, 4 groups
    per CU) whose main pass overflows: the capacity-64 kernel re-solves the
    overflow list first (round 6), the generic capacity-6N pass only what
    outgrows 64.  Every instance equals the port; the adversarial ones span
    both tiers (active sets 61-94 of the reference-form rows)."""
    import hmpc_plan
    from oracle import port
    N, B, A = 60, 1024, 24
    inst = hmpc_plan.sample_instances(B - A, N, curve=False, seed=61)
    adv = adversarial(A, N, 2, 12.0, 2.0)
    inst = {k: np.concatenate([inst[k], adv[k]]) for k in inst}
    c = hmpc_plan.runner_constants()
    cx = hm.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    t0 = cx.overflow_total
    gpu = cx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    handed = cx.overflow_total - t0
    assert cx.kernel_name == 'hmpc::ric_factor_kernel<3, 60, 47> + hmpc::ric_kernel<3, 1, 60, 47, 2>'
    assert cx.active_capacity == 47
    cx.close()
    ref = port.solve_batch('3f', N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                           mu=inst['mu'], nthreads=16)
    assert np.array_equal(gpu['status'], ref['status'])
    ok = ref['status'] == 0
    assert ok[B - A:].all()
    assert np.abs(gpu['u'][ok] - ref['u'][ok]).max() <= U_TOL
    assert np.abs(gpu['x'][ok] - ref['x'][ok]).max() <= U_TOL
    rel = np.abs(gpu['obj'][ok] - ref['obj'][ok]) / np.maximum(np.abs(ref['obj'][ok]), 1.0)
    assert rel.max() <= 1e-8
    assert handed >= A, handed   # every adversarial instance left the main pass
