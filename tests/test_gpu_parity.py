"""GPU parity: libhmpc.so (HIP, gfx950) against the oracle, through the C ABI.

Tolerances (north star: "u* within 1e-6 of cvxpy/OSQP"): max |u* - u*_oracle|
<= 1e-6 (N or N.m) and |obj - obj_oracle| <= 1e-9 |obj_oracle| on every
feasible instance; statuses must agree (infeasible instances are flagged,
not compared).  The oracle's u* is the exact optimum of the reference-built QP
(oracle/qp_exact.py, KKT-certified); see oracle/__init__.py for the pinning.
"""
import glob
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

U_TOL = 1e-6
OBJ_RTOL = 1e-9

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, 'qp_*.npz')))


@pytest.fixture(scope='module')
def hm():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    return hmpc


def ctx_for(hm, variant, N, uref='aliased', mu=1.0):
    from oracle import hmpc_oracle as ho
    c = ho.runner_constants()
    return hm.Context(variant, N, t=c['t'], m=c['m'], g=c['g'], mu=mu, Jinv=c['Jinv'], rh=c['rh'],
                      uref_mode=uref)


def oracle_solve(variant, N, inst, i, uref='aliased'):
    from oracle import hmpc_oracle as ho
    p = ho.MpcParams.runner(variant, N, mu=float(inst['mu'][i]))
    return ho.solve_instance(p, inst['x_in'][i], inst['x_lin'][i], inst['x_ref'][i],
                             inst['pf'][i], inst['C'][i], uref)


def compare(gpu, ref_u, ref_obj, ref_ok):
    st = gpu['status']
    assert np.array_equal(st == 0, ref_ok), (st, ref_ok)
    ok = ref_ok
    du = np.abs(gpu['u'][ok] - ref_u[ok]).max(initial=0.0)
    dob = (np.abs(gpu['obj'][ok] - ref_obj[ok]) / np.abs(ref_obj[ok])).max(initial=0.0)
    assert du <= U_TOL, du
    assert dob <= OBJ_RTOL, dob
    return du, dob


@pytest.mark.parametrize('path', FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
@pytest.mark.parametrize('uref', ['aliased', 'per_stage'])
def test_golden_fixtures(hm, path, uref):
    d = np.load(path)
    variant, N = str(d['variant']), int(d['N'])
    ctx = ctx_for(hm, variant, N, uref)
    tag = 'alias' if uref == 'aliased' else 'stage'
    r = ctx.solve_host(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    compare(r, d[f'u_{tag}'], d[f'obj_{tag}'], d[f'status_{tag}'] == 0)
    # x* satisfies the dynamics the reference's Ad/Bd define
    ok = d[f'status_{tag}'] == 0
    Gd = np.zeros(12)
    Gd[8] = -9.807 * 0.02
    for i in np.where(ok)[0][:4]:
        x, u = r['x'][i], r['u'][i]
        for k in range(N):
            assert np.allclose(x[k + 1], d['Ad'][i][k] @ x[k] + d['Bd'][i][k] @ u[k] + Gd,
                               atol=1e-10)


@pytest.mark.parametrize('variant,N,curve,mu_sweep,B', [
    ('3f', 10, True, None, 48),
    ('3f', 10, False, (0.3, 1.2), 32),
    ('2f', 10, False, None, 32),
    ('2f', 10, True, (0.3, 1.2), 16),
    ('3f', 20, False, (0.3, 1.2), 16),
    ('3f', 5, True, None, 16),
])
def test_random_instances_vs_oracle(hm, variant, N, curve, mu_sweep, B):
    import hmpc_plan
    inst = hmpc_plan.sample_instances(B, N, curve=curve, seed=1000 + N, mu_sweep=mu_sweep)
    ctx = ctx_for(hm, variant, N)
    r = ctx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                       mu=inst['mu'])
    ref_u = np.zeros((B, N, 6))
    ref_obj = np.ones(B)
    ok = np.zeros(B, bool)
    for i in range(B):
        s = oracle_solve(variant, N, inst, i)
        if s['status'] == 'solved':
            ok[i] = True
            ref_u[i] = s['u']
            ref_obj[i] = s['obj']
    assert ok.mean() > 0.9
    compare(r, ref_u, ref_obj, ok)


def test_device_path_bitwise_equals_host_path_and_is_batch_invariant(hm):
    """Per-instance results do not depend on batch size, position or path
    (the multi-GPU correctness argument of SURVEY.md 8e)."""
    import hmpc_plan
    N = 10
    inst = hmpc_plan.sample_instances(1000, N, curve=True, seed=5)
    ctx = ctx_for(hm, '3f', N)
    host = ctx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'])
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
           for k, v in inst.items() if k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C')}
    perm = np.random.default_rng(0).permutation(1000)[:333]
    sub = {k: v[torch.from_numpy(perm).cuda()].contiguous() for k, v in dev.items()}
    out = ctx.solve_device(sub['x_in'], sub['x_lin'], sub['x_ref'], sub['pf'], sub['C'])
    torch.cuda.synchronize()
    assert np.array_equal(out['u'].cpu().numpy(), host['u'][perm])
    assert np.array_equal(out['obj'].cpu().numpy(), host['obj'][perm])
    assert np.array_equal(out['status'].cpu().numpy(), host['status'][perm])


def test_large_batch_feasibility_properties(hm):
    """B = 65536 (config 3): every instance solved, and x*/u* satisfy every
    constraint of the reference's build_qp (size-independent checks)."""
    import hmpc_plan
    N = 10
    inst = hmpc_plan.sample_instances(65536, N, curve=True, seed=9)
    ctx = ctx_for(hm, '3f', N)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
           for k, v in inst.items() if k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C')}
    out = ctx.solve_device(dev['x_in'], dev['x_lin'], dev['x_ref'], dev['pf'], dev['C'])
    torch.cuda.synchronize()
    st = out['status'].cpu().numpy()
    u = out['u'].cpu().numpy()
    x = out['x'].cpu().numpy()
    C = inst['C']
    solved = st == 0
    assert solved.mean() > 0.999, np.bincount(st)
    tol = 1e-7
    us, xs, Cs = u[solved], x[solved], C[solved]
    assert np.all(np.abs(us[..., 3:5]) <= 7.78 + tol) and np.all(np.abs(us[..., 5]) <= 4 + tol)
    stance = Cs != 0
    fx, fy, fz = us[..., 0], us[..., 1], us[..., 2]
    assert np.all(fz[stance] >= -tol) and np.all(fz[stance] <= 206 + tol)
    assert np.all(np.abs(fx[stance]) <= fz[stance] + tol)
    assert np.all(np.abs(fy[stance]) <= fz[stance] + tol)
    assert np.all(np.abs(us[..., 0:3][~stance]) <= 1e-12)
    assert np.all(xs[:, :-1, 2] >= 0.1 - tol)
    assert np.allclose(xs[:, 0], inst['x_in'][solved], atol=0)


def test_infeasible_and_empty_batches(hm):
    import hmpc_plan
    N = 10
    inst = hmpc_plan.sample_instances(4, N, seed=2)
    inst['x_in'][1, 2] = 0.05            # z0 < 0.1: x[0,2] >= 0.1 cannot hold
    inst['x_lin'][1, 0, 2] = 0.05
    ctx = ctx_for(hm, '3f', N)
    r = ctx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'])
    assert r['status'][1] == 2
    assert np.all(r['status'][[0, 2, 3]] == 0)
    e = ctx.solve_host(inst['x_in'][:0], inst['x_lin'][:0], inst['x_ref'][:0], inst['pf'][:0],
                       inst['C'][:0])
    assert e['u'].shape == (0, N, 6)


def test_dropin_mpc_replays_reference_closed_loop(hm):
    """The drop-in Mpc (mpc_cvx_euler_3f.Mpc) fed the inputs the REFERENCE
    Runner produced (loop_3f_N10.npz, 50 mpcontrol calls incl. the init
    double solve and the time-shifted warm linearisation) returns the same u."""
    import mpc_cvx_euler_3f
    from oracle import hmpc_oracle as ho
    d = np.load(os.path.join(GOLDEN, 'loop_3f_N10.npz'))
    c = ho.runner_constants()
    mpc = mpc_cvx_euler_3f.Mpc(t=0.02, N=10, m=c['m'], g=c['g'], mu=1, Jinv=c['Jinv'], rh=c['rh'])
    n = int(d['n_detail'])
    worst = 0.0
    for j in range(n):
        U = mpc.mpcontrol(x_in=d['x_in'][j], x_ref_in=d[f'c{j}_x_ref'], pf=d[f'c{j}_pf'],
                          C=d['C'][j], init=bool(d['init'][j]))
        worst = max(worst, np.abs(U - d[f'c{j}_U']).max())
        assert np.abs(mpc.x.value - d[f'c{j}_xstar']).max() < 1e-6
    assert worst <= U_TOL, worst
    assert mpc.solves == n + 1


def test_dropin_raises_like_the_reference_on_failure(hm):
    import mpc_cvx_euler_3f
    import hmpc_plan
    from oracle import hmpc_oracle as ho
    c = ho.runner_constants()
    inst = hmpc_plan.sample_instances(1, 10, seed=4)
    mpc = mpc_cvx_euler_3f.Mpc(t=0.02, N=10, m=c['m'], g=c['g'], mu=1, Jinv=c['Jinv'], rh=c['rh'])
    x_in = inst['x_in'][0].copy()
    x_in[2] = 0.0
    with pytest.raises(Exception, match='QP FAILED'):
        mpc.mpcontrol(x_in=x_in, x_ref_in=inst['x_ref'][0], pf=inst['pf'][0], C=inst['C'][0],
                      init=True)


def test_device_mpcontrol_matches_dropin(hm):
    """hmpc_mpcontrol_batch (on-device linearisation + time shift) equals
    the drop-in's host-side mpcontrol, call for call."""
    import mpc_cvx_euler_3f
    from oracle import hmpc_oracle as ho
    d = np.load(os.path.join(GOLDEN, 'loop_3f_N10.npz'))
    c = ho.runner_constants()
    mpc = mpc_cvx_euler_3f.Mpc(t=0.02, N=10, m=c['m'], g=c['g'], mu=1, Jinv=c['Jinv'], rh=c['rh'])
    ctx = ctx_for(hm, '3f', 10)
    xprev = torch.zeros((1, 11, 12), dtype=torch.float64, device='cuda')
    for j in range(12):
        args = dict(x_in=d['x_in'][j], x_ref_in=d[f'c{j}_x_ref'], pf=d[f'c{j}_pf'], C=d['C'][j])
        U = mpc.mpcontrol(init=bool(d['init'][j]), **args)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)[None]).cuda()  # noqa: E731
        out = ctx.mpcontrol_device(bool(d['init'][j]), t(args['x_in']), t(args['x_ref_in']),
                                   t(args['pf']), t(args['C']), xprev)
        torch.cuda.synchronize()
        assert out['status'].item() == 0
        assert np.array_equal(out['u'][0].cpu().numpy(), U)
        assert np.array_equal(xprev[0].cpu().numpy(), mpc.x.value)


@pytest.mark.parametrize('variant,curve', [('3f', False), ('2f', False), ('3f', True)])
def test_dense_n20_forced(hm, variant, curve):
    """The two-wave dense kernel at N = 20 (HMPC_PREC_F64_DENSE, an A/B-only
    precision; the default N = 20 path is the Riccati kernel): statuses, u*,
    x* and the objective against the C port.  tools/exec_lint.py reports
    exec-masked spill copies in this kernel (tests/test_exec_lint.py): this
    checks their values are not read by lanes outside their regions."""
    import hmpc_plan
    from oracle import hmpc_oracle as ho
    from oracle import port
    N, B = 20, 256
    inst = hmpc_plan.sample_instances(B, N, curve=curve, seed=77, mu_sweep=(0.3, 1.2))
    c = ho.runner_constants()
    cx = hm.Context(variant, N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'],
                    precision='f64_dense')
    assert cx.kernel_name == f'hmpc::solve_kernel<{variant[0]}, 20, double, 0, 0>'
    g = cx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    cx.close()
    ref = port.solve_batch(variant, N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                           mu=inst['mu'], nthreads=16)
    assert np.array_equal(g['status'], ref['status'])
    ok = ref['status'] == 0
    assert ok.mean() > 0.9
    assert np.abs(g['u'][ok] - ref['u'][ok]).max() <= U_TOL
    assert np.abs(g['x'][ok] - ref['x'][ok]).max() <= U_TOL
    assert (np.abs(g['obj'][ok] - ref['obj'][ok]) / np.abs(ref['obj'][ok])).max() <= OBJ_RTOL
