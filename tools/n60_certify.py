"""Certify every QP of the reference Runner's default run (3f, N = 60,
N_run = 2000: ``run.py 3f``) -- test infrastructure, CPU only.

The closed loop is driven by the C port (oracle/hmpc_port.c) as the Mpc; for
every one of its 101 solves the reference-form QP (oracle/hmpc_oracle.build_qp,
pinned bit for bit to the reference's own build_qp) is

  * checked against the port's (x*, u*): max violation of every row of
    l <= A z <= u -- a feasible point certifies the QP is feasible;
  * solved by oracle/qp_exact (IPM + polish + KKT certificate).

Writes the per-solve inputs to gpurun_out/loop_3f_N60_inputs.npz (scratch) when
--save is given.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from oracle import hmpc_oracle as ho  # noqa: E402
from oracle import hmpc_plant as hpl  # noqa: E402
from oracle import port, qp_exact  # noqa: E402


class PortMpc:
    """Mpc.mpcontrol (src/mpc_cvx_euler_3f.py:41-69) over the C port."""

    def __init__(self, N):
        self.N = N
        self.x_value = None
        self.log = []

    def _solve(self, x_in, x_lin, x_ref, pf, C):
        r = port.solve_batch('3f', self.N, x_in[None], x_lin[None], x_ref[None], pf[None], C[None])
        self.log.append(dict(x_in=x_in.copy(), x_lin=x_lin.copy(), x_ref=np.array(x_ref),
                             pf=np.array(pf), C=np.array(C), u=r['u'][0], x=r['x'][0],
                             obj=r['obj'][0], status=int(r['status'][0])))
        if r['status'][0] != 0:
            raise Exception('\n *** QP FAILED *** \n')
        return r['u'][0], r['x'][0]

    def mpcontrol(self, x_in, x_ref_in, pf, C, init):
        N = self.N
        xg = np.zeros((N + 1, 12))
        if init:
            xg[0] = x_in
            xg[1:] = x_ref_in
            _, xg = self._solve(x_in, xg, x_ref_in, pf, C)
        else:
            xg[0] = x_in
            xg[1:-1] = self.x_value[2:]
            xg[-1] = self.x_value[-1]
        u, x = self._solve(x_in, xg, x_ref_in, pf, C)
        self.x_value = x
        return u


def violation(qp, z):
    Az = qp['A'] @ z
    return float(max(np.max(qp['l'] - Az), np.max(Az - qp['u']), 0.0))


def main():
    save = "--save" in sys.argv
    only_last = "--last" in sys.argv
    N = 60
    orig = ho.OracleMpc
    holder = {}

    def factory(p, uref_mode='aliased'):
        m = PortMpc(p.N)
        holder['m'] = m
        return m

    ho.OracleMpc = factory
    try:
        out = hpl.run_closed_loop(N=N, N_run=2000, curve=False)
    finally:
        ho.OracleMpc = orig
    log = holder['m'].log
    print(f'{len(log)} solves; final state {out["X_traj"][-1][:3]}')
    p = ho.MpcParams.runner('3f', N)
    _, _, Gd = ho.constant_matrices(p)
    worst = []
    for i, s in enumerate(log):
        Ad, Bd = ho.gen_dt_dynamics(p, s['x_lin'], s['pf'])
        qp = ho.build_qp(p, s['x_in'], s['x_ref'], Ad, Bd, Gd, s['C'])
        z = np.concatenate([s['x'].ravel(), s['u'].ravel()])
        viol = violation(qp, z)
        t = time.time()
        sol = qp_exact.solve(qp['P'], qp['q'], qp['A'], qp['l'], qp['u'])
        el = time.time() - t
        du = np.nan
        if sol['x'] is not None:
            du = float(np.abs(sol['x'][(N + 1) * 12:] - s['u'].ravel()).max())
        worst.append((i, s['status'], sol['status'], viol, du))
        if sol['status'] != 'solved' or s['status'] != 0 or not (du < 1e-6):
            print(f'solve {i}: port status {s["status"]} violation {viol:.2e}; qp_exact '
                  f'{sol["status"]} ({sol["iters"]} it, {el:.1f}s) |du| {du:.2e}')
    print('max port violation', max(w[3] for w in worst), 'max |du|',
          np.nanmax([w[4] for w in worst]))
    if save:
        arrs = {k: np.array([s[k] for s in log]) for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'u', 'x',
                                                           'obj', 'status')}
        np.savez_compressed(os.path.join(ROOT, "gpurun_out", "loop_3f_N60_inputs.npz"), **arrs)


if __name__ == '__main__':
    main()
