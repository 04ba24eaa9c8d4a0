"""The reference Runner's own configuration on the GPU (run.py 3f
--N_run=2000: N = 60, src/robotrunner.py:46; BASELINE configs[0]) -- the
Riccati kernel (hmpc_ric.hip) that serves 10 < N <= 64.

* every one of the reference run's 100 mpcontrol calls (101 QP solves)
  replayed through the C ABI on the reference's own inputs and linearisation
  (tests/golden/loop_3f_N60_config1.npz, recorded by make_golden.py through
  the reference's Mpc.mpcontrol; see tests/test_oracle_n60.py): u* and x*
  within 1e-6, every status solved;
* the whole 2000-step run through the device Runner (plant kernel + plan
  views + mpcontrol): states within 1e-6 of the reference loop, inputs within
  1e-5, all 100 calls solved;
* a 4096-instance N = 60 batch against the C port: equal statuses (the 25
  infeasible instances of the bench sample are certified infeasible on the
  CPU by qp_exact.min_violation), |du| <= 1e-6.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')
U_TOL = 1e-6


@pytest.fixture(scope='module')
def hm():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    return hmpc


@pytest.fixture(scope='module')
def loop():
    return np.load(os.path.join(GOLDEN, 'loop_3f_N60_config1.npz'))


def test_every_reference_call_replayed(hm, loop):
    import mpc_cvx_euler_3f
    from oracle import hmpc_oracle as ho
    g = loop
    N = int(g['N'])
    c0 = ho.runner_constants()
    # call 0: the init double solve through the drop-in Mpc
    mpc = mpc_cvx_euler_3f.Mpc(t=c0['t'], N=N, m=c0['m'], g=c0['g'], mu=1, Jinv=c0['Jinv'], rh=c0['rh'])
    u = mpc.mpcontrol(x_in=g['x_in'][0], x_ref_in=g['c0_x_ref'], pf=g['c0_pf'], C=g['C'][0], init=True)
    assert np.abs(u - g['c0_U']).max() <= U_TOL
    # calls 1..99 as one batch: each on the reference's own linearisation
    # (the time shift of the reference's previous x*, 3f :59-62)
    n = len(g['k'])
    x_in = np.stack([g['x_in'][c] for c in range(1, n)])
    x_lin = np.stack([np.vstack([g['x_in'][c], g[f'c{c - 1}_xstar'][2:], g[f'c{c - 1}_xstar'][-1:]])
                      for c in range(1, n)])
    x_ref = np.stack([g[f'c{c}_x_ref'] for c in range(1, n)])
    pf = np.stack([g[f'c{c}_pf'] for c in range(1, n)])
    C = np.stack([g['C'][c] for c in range(1, n)])
    cx = hm.Context('3f', N, t=c0['t'], m=c0['m'], g=c0['g'], mu=1.0, Jinv=c0['Jinv'], rh=c0['rh'])
    r = cx.solve_host(x_in, x_lin, x_ref, pf, C)
    cx.close()
    assert (r['status'] == 0).all()
    U = np.stack([g[f'c{c}_U'] for c in range(1, n)])
    X = np.stack([g[f'c{c}_xstar'] for c in range(1, n)])
    assert np.abs(r['u'] - U).max() <= U_TOL
    assert np.abs(r['x'] - X).max() <= U_TOL


def test_full_reference_run_on_device(hm, loop):
    import hmpc_runner
    g = loop
    n = len(g['k'])
    r = hmpc_runner.Runner(dt=1e-3, dyn='3f', curve=bool(g['curve']), N_run=int(g['N_run']),
                           N=int(g['N']), batch=1)
    out = r.run(n_periods=n)
    r.close()
    assert (out['status'] == 0).all()
    X = out['X_traj'][0]
    np.testing.assert_allclose(X[::20], g['X_traj_mpc'], rtol=0, atol=1e-6)
    np.testing.assert_allclose(out['f_hist'][0][::20], g['U0'], rtol=0, atol=1e-5)


def test_n60_batch_statuses_equal_port(hm):
    import hmpc_plan as hp
    from oracle import hmpc_oracle as ho
    from oracle import port
    N, B = 60, 4096
    inst = hp.sample_instances(B, N, curve=False, seed=2024)
    c = ho.runner_constants()
    cx = hm.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
    gpu = cx.solve_host(inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'], mu=inst['mu'])
    cx.close()
    ref = port.solve_batch('3f', N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                           mu=inst['mu'], nthreads=16)
    assert np.array_equal(gpu['status'], ref['status'])
    assert (ref['status'] == 0).sum() == B - 25
    ok = ref['status'] == 0
    assert np.abs(gpu['u'][ok] - ref['u'][ok]).max() <= U_TOL
    assert np.abs(gpu['x'][ok] - ref['x'][ok]).max() <= U_TOL
    assert (np.abs(gpu['obj'][ok] - ref['obj'][ok]) / np.abs(ref['obj'][ok])).max() <= 1e-8


def test_fused_fallback_equals_factorisation_kernel():
    """Horizons above 24 factorise in a kernel of their own when the
    per-instance K / Dinv blocks fit 4 GB (hmpc_ric.hip ric_kinst_stride);
    a larger batch (here 100 000 x N = 60: 4.5 GB) falls back to the fused
    solve kernel.  Both run the same phase-2 arithmetic, so the instances
    they share come out bit for bit equal, and equal to the C port."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import hmpc
    import hmpc_plan
    from oracle import port
    N, B, n = 60, 100_000, 48
    c = hmpc_plan.runner_constants()
    inst = hmpc_plan.sample_instances(B, N, curve=False, seed=61)
    keys = ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')

    def run(b):
        cx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])
        d = {k: torch.from_numpy(np.ascontiguousarray(inst[k][:b])).cuda() for k in keys}
        out = cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
        torch.cuda.synchronize()
        r = {k: out[k][:n].cpu().numpy() for k in ('u', 'x', 'obj', 'status')}
        cx.close()
        return r

    big, small = run(B), run(n)   # fused kernel / factorisation kernel + solve kernel
    for k in big:
        assert np.array_equal(big[k], small[k]), k
    ref = port.solve_batch('3f', N, *(inst[k][:n] for k in keys[:5]), mu=inst['mu'][:n], nthreads=16)
    assert np.array_equal(big['status'], ref['status'])
    ok = ref['status'] == 0
    assert np.abs(big['u'][ok] - ref['u'][ok]).max() <= 1e-6
