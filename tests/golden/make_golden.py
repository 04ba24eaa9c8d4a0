#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own code.

Run here only (it reads /root/reference, which does not exist on the GPU box):

    python tests/golden/make_golden.py

What it does:
* imports /root/reference/src with bytecode writing disabled, a recording
  cvxpy stub and a transforms3d restatement on sys.path (tests/golden/_stubs);
* problem data: calls the reference's ``Mpc.gen_dt_dynamics`` and
  ``Mpc.build_qp``; the stub canonicalises the returned cost/constraint list
  into OSQP form (P, q, r, A, l, u), once with constants captured by
  reference (cvxpy semantics => the u_ref aliasing) and once with copies
  (the intended per-stage u_ref);
* solutions: the stub's ``Problem.solve`` delegates to the oracle's exact
  solver (oracle/qp_exact.py) -- cvxpy/OSQP are not installed; every
  solution carries its KKT certificate;
* planner: ``Runner.path_plan_init`` (straight and --curve), ``gait_map``;
* closed loop: the reference Runner loop (gait, plan grab, convert,
  ``Mpc.mpcontrol``, ``rk4_normalized``) at N=10 and, for config 1, N=60;
* the CasADi variant (src/mpc_cas_euler_3f.py): its own Mpc builds its QP
  through a recording casadi stub (tests/golden/_stubs/casadi, sympy
  algebra); the QP data handed to qpOASES is recorded and solved exactly by
  oracle/cas_oracle.py (qpOASES is absent: solve parity unpinned).

Only inputs and outputs are written (npz); no reference source is copied.
"""
import os
import sys

sys.dont_write_bytecode = True
os.environ['PYTHONDONTWRITEBYTECODE'] = '1'

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = '/root/reference/src'
sys.path.insert(0, os.path.join(HERE, '_stubs'))
sys.path.insert(1, REF_SRC)
sys.path.insert(2, REPO)

import numpy as np  # noqa: E402

import cvxpy  # noqa: E402  (the recording stub)
from oracle import qp_exact  # noqa: E402

cvxpy.SOLVER = qp_exact.solve

import mpc_cvx_euler_2f as ref2f  # noqa: E402
import mpc_cvx_euler_3f as ref3f  # noqa: E402
import robotrunner  # noqa: E402

REFMOD = {'3f': ref3f, '2f': ref2f}


def coo(A):
    r, c = np.nonzero(A)
    return r.astype(np.int32), c.astype(np.int32), A[r, c]


def reference_plan(curve, N_run=2000, N=60):
    rr = robotrunner.Runner(dt=1e-3, dyn='3f', curve=curve, N_run=N_run)
    rr.N = N
    rr.N_k = int(rr.N * rr.mpc_factor)
    x0 = robotrunner.convert(np.tile(rr.X_0, (N_run + 1, 1))[0, :])
    xf = robotrunner.convert(rr.X_f)
    x_ref, pf_ref = rr.path_plan_init(x_in=x0, xf=xf)
    return rr, x_ref, pf_ref


def sample(rr, plan, pf_plan, B, N, rng, mu_sweep=None, N_run=2000):
    """SURVEY.md 8d sampler on the reference's own plan and gait_map."""
    f = rr.mpc_factor
    out = []
    for _ in range(B):
        k0 = f * int(rng.integers(0, N_run // f))
        noise = np.concatenate([rng.uniform(-0.02, 0.02, 3), rng.uniform(-0.05, 0.05, 3),
                                rng.uniform(-0.2, 0.2, 6)])
        mu = float(rng.uniform(*mu_sweep)) if mu_sweep else 1.0
        C = rr.gait_map(N, 0.02, rr.t_start + (k0 + 1) * 1e-3, 0)
        x_ref = plan[k0:k0 + f * N:f].copy()
        pf = pf_plan[k0:k0 + f * N:f].copy()
        x_in = plan[k0] + noise
        x_lin = np.vstack([x_in, x_ref])
        out.append(dict(k0=k0, x_in=x_in, x_lin=x_lin, x_ref=x_ref, pf=pf, C=C, mu=mu))
    return out


def run_reference_qp(variant, N, inst, rr, copy_constants):
    cvxpy.COPY_CONSTANTS = copy_constants
    mod = REFMOD[variant]
    mpc = mod.Mpc(t=rr.mpc_dt, N=N, m=rr.m, g=rr.g, mu=inst['mu'], Jinv=rr.Jinv, rh=rr.rh)
    mpc.gen_dt_dynamics(inst['x_lin'], inst['pf'])
    cost, constr = mpc.build_qp(inst['x_in'], inst['x_ref'], mpc.Ad, mpc.Bd, mpc.Gd, inst['C'])
    n0 = len(cvxpy.RECORD)
    try:
        mpc.solve_qp(cost, constr)
    except Exception as exc:  # the reference's "*** QP FAILED ***"
        assert 'QP FAILED' in str(exc)
    cvxpy.COPY_CONSTANTS = False
    rec = cvxpy.RECORD[n0]
    return mpc, rec


STATUS_CODE = {'solved': 0, 'solved_inaccurate': 1, 'primal_infeasible': 2, 'failed': 3}


def make_qp_fixture(variant, N, curve, B, n_full, seed, mu_sweep=None):
    rr, plan, pf_plan = reference_plan(curve)
    rng = np.random.default_rng(seed)
    insts = sample(rr, plan, pf_plan, B, N, rng, mu_sweep)
    d = {k: [] for k in ['x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu', 'k0', 'Ad', 'Bd',
                         'u_alias', 'x_alias', 'obj_alias', 'status_alias',
                         'u_stage', 'x_stage', 'obj_stage', 'status_stage', 'cert_alias']}
    full = {}
    for i, inst in enumerate(insts):
        for k in ['x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu', 'k0']:
            d[k].append(inst[k])
        mpc, rec_a = run_reference_qp(variant, N, inst, rr, False)
        _, rec_s = run_reference_qp(variant, N, inst, rr, True)
        d['Ad'].append(mpc.Ad.copy())
        d['Bd'].append(mpc.Bd.copy())
        for tag, rec in (('alias', rec_a), ('stage', rec_s)):
            sol, qp = rec['sol'], rec['qp']
            st = STATUS_CODE[sol['status']]
            d['status_' + tag].append(st)
            if sol['x'] is None:
                d['u_' + tag].append(np.full((N, 6), np.nan))
                d['x_' + tag].append(np.full((N + 1, 12), np.nan))
                d['obj_' + tag].append(np.nan)
            else:
                z = sol['x']
                d['x_' + tag].append(z[:(N + 1) * 12].reshape(N + 1, 12))
                d['u_' + tag].append(z[(N + 1) * 12:].reshape(N, 6))
                d['obj_' + tag].append(0.5 * z @ qp['P'] @ z + qp['q'] @ z + qp['r'])
            if tag == 'alias':
                c = sol['cert'] or {}
                d['cert_alias'].append([c.get(k, np.nan) for k in
                                        ('primal_eq', 'primal_ineq', 'dual_neg', 'stationarity')])
        if i < n_full:
            for tag, rec in (('alias', rec_a), ('stage', rec_s)):
                qp = rec['qp']
                assert np.count_nonzero(qp['P'] - np.diag(np.diag(qp['P']))) == 0
                full[f'i{i}_{tag}_Pdiag'] = np.diag(qp['P']).copy()
                full[f'i{i}_{tag}_q'] = qp['q']
                full[f'i{i}_{tag}_r'] = np.array(qp['r'])
            r, c, v = coo(rec_a['qp']['A'])
            full[f'i{i}_A_row'], full[f'i{i}_A_col'], full[f'i{i}_A_val'] = r, c, v
            full[f'i{i}_A_shape'] = np.array(rec_a['qp']['A'].shape, dtype=np.int32)
            full[f'i{i}_l'] = rec_a['qp']['l']
            full[f'i{i}_u'] = rec_a['qp']['u']
            assert np.array_equal(rec_a['qp']['A'], rec_s['qp']['A'])
    arrs = {k: np.array(v) for k, v in d.items()}
    arrs.update(full)
    arrs['n_full'] = np.array(n_full)
    arrs['Jinv'] = rr.Jinv
    arrs['rh'] = rr.rh
    arrs['variant'] = np.array(variant)
    arrs['N'] = np.array(N)
    arrs['curve'] = np.array(curve)
    name = f'qp_{variant}_N{N}_{"curve" if curve else "straight"}{"_musweep" if mu_sweep else ""}.npz'
    np.savez_compressed(os.path.join(HERE, name), **arrs)
    sts = arrs['status_alias']
    print(f'{name}: {B} instances, status counts {np.bincount(sts, minlength=4)}, '
          f'max cert {np.nanmax(arrs["cert_alias"]):.2e}')


def make_plan_fixture():
    arrs = {}
    for curve in (False, True):
        rr, x_ref, pf_ref = reference_plan(curve)
        tag = 'curve' if curve else 'straight'
        arrs[f'{tag}_x_ref'] = x_ref
        arrs[f'{tag}_pf_ref'] = pf_ref
    rr, _, _ = reference_plan(False)
    ts = rr.t_start + (np.arange(0, 2000, 20) + 1) * 1e-3
    arrs['gait_ts'] = ts
    arrs['gait_C10'] = np.array([rr.gait_map(10, 0.02, t, 0) for t in ts])
    np.savez_compressed(os.path.join(HERE, 'plan.npz'), **arrs)
    print('plan.npz written')


def make_closed_loop_fixture(N, N_run, curve, name, n_detail):
    """The reference Runner.run loop (src/robotrunner.py:81-113) without plots."""
    rr = robotrunner.Runner(dt=1e-3, dyn='3f', curve=curve, N_run=N_run)
    rr.N = N
    rr.N_k = int(rr.N * rr.mpc_factor)
    rr.mpc = ref3f.Mpc(t=rr.mpc_dt, N=N, m=rr.m, g=rr.g, mu=1, Jinv=rr.Jinv, rh=rr.rh)
    Nr = rr.N_run + 1
    t = rr.t_start
    t0 = 0
    mpc_factor = rr.mpc_factor
    mpc_counter = mpc_factor
    X_traj = np.tile(rr.X_0, (Nr, 1))
    f_hist = np.zeros((Nr, rr.n_U))
    U = np.zeros(rr.n_U)
    x_ref, pf_ref = rr.path_plan_init(x_in=robotrunner.convert(X_traj[0, :]), xf=robotrunner.convert(rr.X_f))
    init = True
    calls = {k: [] for k in ['k', 'x_in', 'C', 'init', 'U0', 'X']}
    detail = {}
    ncall = 0
    for k in range(0, rr.N_run):
        t = t + rr.dt
        if mpc_counter == mpc_factor:
            mpc_counter = 0
            C = rr.gait_map(rr.N, rr.mpc_dt, t, t0)
            x_refk = rr.path_plan_grab(x_ref=x_ref, k=k)
            pf_refk = rr.path_plan_grab(x_ref=pf_ref, k=k)
            x_in = robotrunner.convert(X_traj[k, :])
            U = rr.mpc.mpcontrol(x_in=x_in, x_ref_in=x_refk, pf=pf_refk, C=C, init=init)
            calls['k'].append(k); calls['x_in'].append(x_in); calls['C'].append(C)
            calls['init'].append(init); calls['U0'].append(U[0].copy()); calls['X'].append(X_traj[k].copy())
            if ncall < n_detail:
                detail[f'c{ncall}_x_ref'] = np.array(x_refk)
                detail[f'c{ncall}_pf'] = np.array(pf_refk)
                detail[f'c{ncall}_U'] = np.array(U)
                detail[f'c{ncall}_xstar'] = np.array(rr.mpc.x.value)
            ncall += 1
            init = False
        mpc_counter += 1
        f_hist[k, :] = U[0, :]
        X_traj[k + 1, :] = rr.rk4_normalized(xk=X_traj[k, :], uk=f_hist[k, :], pfk=pf_ref[k, :])
    arrs = {k: np.array(v) for k, v in calls.items()}
    arrs.update(detail)
    arrs['X_traj_final'] = X_traj[-1]
    arrs['X_traj_mpc'] = X_traj[::mpc_factor]
    arrs['n_detail'] = np.array(n_detail)
    arrs['N'] = np.array(N)
    arrs['N_run'] = np.array(N_run)
    arrs['curve'] = np.array(curve)
    np.savez_compressed(os.path.join(HERE, name), **arrs)
    print(f'{name}: {ncall} mpcontrol calls')


def make_cas_fixture(N, B, seed, curve=True):
    """The CasADi variant's QP data (src/mpc_cas_euler_3f.py:14-152) for B
    sampled instances, as the reference's own Mpc builds it."""
    import casadi  # noqa: F401  (the recording stub)
    import mpc_cas_euler_3f as refcas
    from oracle import cas_oracle
    casadi.SOLVER = lambda rec: cas_oracle.solve(rec, N)['z']
    rr, plan, pf_plan = reference_plan(curve)
    rng = np.random.default_rng(seed)
    insts = sample(rr, plan, pf_plan, B, N, rng)
    mpc = refcas.Mpc(t=rr.mpc_dt, N=N, Jinv=rr.Jinv, rh=rr.rh, m=rr.m, g=rr.g, mu=1)
    keys = ('x_in', 'x_ref', 'C', 'Pdiag', 'q', 'r', 'g0', 'lbg', 'ubg', 'lbx', 'ubx', 'u', 'z')
    arrs = {k: [] for k in keys}
    A_r, A_c, A_v, A_n = [], [], [], []
    for inst in insts:
        n0 = len(casadi.RECORD)
        u = mpc.mpcontrol(x_in=inst['x_in'], x_ref_in=inst['x_ref'], rf=inst['pf'], C=inst['C'])
        rec = casadi.RECORD[n0]
        P = rec['P']
        assert np.count_nonzero(P - np.diag(np.diag(P))) == 0
        vals = dict(x_in=inst['x_in'], x_ref=inst['x_ref'], C=inst['C'], Pdiag=np.diag(P), q=rec['q'],
                    r=rec['r'], g0=rec['g0'], lbg=rec['lbg'], ubg=rec['ubg'], lbx=rec['lbx'],
                    ubx=rec['ubx'], u=u, z=rec['z'])
        for k in keys:
            arrs[k].append(vals[k])
        r, c, v = coo(rec['A'])
        A_r.append(r); A_c.append(c); A_v.append(v); A_n.append(len(v))
    out = {k: np.array(v) for k, v in arrs.items()}
    out['A_row'] = np.concatenate(A_r)
    out['A_col'] = np.concatenate(A_c)
    out['A_val'] = np.concatenate(A_v)
    out['A_nnz'] = np.array(A_n)
    out['A_shape'] = np.array(rec['A'].shape)
    out['N'] = np.array(N)
    out['curve'] = np.array(curve)
    out['Jinv'] = rr.Jinv
    out['rh'] = rr.rh
    name = f'cas_N{N}.npz'
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(f'{name}: {B} instances, A {rec["A"].shape}')


def make_plant_fixture():
    """dynamics_ct / rk4_normalized / convert samples."""
    rr = robotrunner.Runner(dt=1e-3, dyn='3f', curve=False, N_run=2000)
    rng = np.random.default_rng(7)
    X = np.zeros((16, 13)); U = rng.uniform(-50, 150, (16, 6)); pf = rng.uniform(-0.5, 0.5, (16, 3))
    X[:, 0:3] = rng.uniform(-1, 1, (16, 3))
    q = rng.normal(size=(16, 4)); X[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    X[:, 7:13] = rng.uniform(-1, 1, (16, 6))
    dX = np.array([rr.dynamics_ct(X[i], U[i], pf[i]) for i in range(16)])
    Xn = np.array([rr.rk4_normalized(X[i], U[i], pf[i]) for i in range(16)])
    xc = np.array([robotrunner.convert(X[i]) for i in range(16)])
    np.savez_compressed(os.path.join(HERE, 'plant.npz'), X=X, U=U, pf=pf, dX=dX, Xn=Xn, x_conv=xc)
    print('plant.npz written')


if __name__ == '__main__':
    which = sys.argv[1:] or ['plan', 'qp', 'loop', 'plant', 'cas']
    if 'plan' in which:
        make_plan_fixture()
    if 'plant' in which:
        make_plant_fixture()
    if 'qp' in which:
        make_qp_fixture('3f', 10, True, 32, 6, seed=1)
        make_qp_fixture('3f', 10, False, 32, 6, seed=2)
        make_qp_fixture('2f', 10, False, 32, 6, seed=3)
        make_qp_fixture('2f', 10, True, 16, 4, seed=4)
        make_qp_fixture('3f', 20, False, 12, 3, seed=5, mu_sweep=(0.3, 1.2))
        make_qp_fixture('3f', 10, True, 16, 2, seed=6, mu_sweep=(0.3, 1.2))
    if 'cas' in which:
        make_cas_fixture(10, 8, seed=21)
    if 'loop' in which:
        make_closed_loop_fixture(10, 1000, False, 'loop_3f_N10.npz', n_detail=50)
        make_closed_loop_fixture(60, 2000, False, 'loop_3f_N60_config1.npz', n_detail=100)
