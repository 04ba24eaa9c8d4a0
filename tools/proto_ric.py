"""Prototype (numpy) of the Riccati-factored condensed Hessian used by the
long-horizon kernel (csrc/hmpc_ric.hip): checks H^-1 n = M^-1 M^-T n against a
dense solve of the condensed Hessian the port builds.  Design aid, not a test.

H = 2 (Gamma' W Gamma + V) over u (6N), fixed variables (swing forces, 2f fy)
as identity rows/columns.  Backward Riccati with everything x2:
  P_N = 2*100*Q
  G_k = 2 V_k + B_k' P_{k+1} B_k,  F_k = B_k' P_{k+1} A_k,  K_k = G_k^-1 F_k
  P_k = 2 Q + A_k' P_{k+1} A_k - F_k' K_k
1/2 u'Hu = sum_k 1/2 (u_k + K_k x_k)' G_k (u_k + K_k x_k), x_0 = 0.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd'))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import hmpc_plan as hp  # noqa: E402
from oracle import hmpc_oracle as ho  # noqa: E402

Q = ho.Q_DIAG


def factor(Ad, Bd, free, N):
    """Kernel arithmetic: G = D D' (Cholesky), K = D^-T (D^-1 F), Ginv =
    D^-T D^-1 (explicit), P symmetric (lower triangle mirrored).  An LU
    inverse of G instead loses up to 1e-3 relative at N = 60."""
    P = 2 * 100 * np.diag(Q)
    K = np.zeros((N, 6, 12))
    Gi = np.zeros((N, 6, 6))
    for k in range(N - 1, -1, -1):
        B = Bd[k] * free[k][None, :]
        V = 2 * 0.001 * np.eye(6) if k < N - 1 else np.zeros((6, 6))
        G = V + B.T @ P @ B
        for c in range(6):
            if not free[k][c]:
                G[c, c] = 1.0
        F = B.T @ P @ Ad[k]
        D = np.linalg.cholesky(G)
        Di = np.linalg.solve(D, np.eye(6))     # lower triangular inverse
        Di = np.tril(Di)
        Gi[k] = Di.T @ Di
        K[k] = Di.T @ (Di @ F)
        P = 2 * np.diag(Q) + Ad[k].T @ P @ Ad[k] - F.T @ K[k]
        P = np.tril(P) + np.tril(P, -1).T
    return K, Gi


def hinv(Ad, Bd, free, K, Gi, n, N):
    n = n.reshape(N, 6)
    lam = np.zeros(12)
    mu = np.zeros((N, 6))
    for j in range(N - 1, -1, -1):
        B = Bd[j] * free[j][None, :]
        mu[j] = n[j] - B.T @ lam
        lam = Ad[j].T @ lam + K[j].T @ mu[j]
    w = np.einsum('kcd,kd->kc', Gi, mu)
    x = np.zeros(12)
    u = np.zeros((N, 6))
    for k in range(N):
        B = Bd[k] * free[k][None, :]
        u[k] = w[k] - K[k] @ x
        x = Ad[k] @ x + B @ u[k]
    return u.ravel()


def dense_H(Ad, Bd, free, N):
    NV = 6 * N
    Gm = np.zeros((12 * N, NV))
    for j in range(N):
        B = Bd[j] * free[j][None, :]
        blk = B
        for t in range(j, N):
            if t > j:
                blk = Ad[t] @ blk
            Gm[12 * t:12 * t + 12, 6 * j:6 * j + 6] = blk
    W = np.concatenate([Q * (100 if t == N - 1 else 1) for t in range(N)])
    H = 2 * Gm.T @ (W[:, None] * Gm)
    for v in range(NV):
        k, c = divmod(v, 6)
        if not free[k][c]:
            H[v, v] = 1.0
        elif k < N - 1:
            H[v, v] += 2 * 0.001
    return H


def main():
    for variant in ('3f', '2f'):
        for N in (10, 20, 60):
            inst = hp.sample_instances(3, N, curve=True, seed=5)
            p = ho.MpcParams.runner(variant, N)
            for i in range(3):
                Ad, Bd = ho.gen_dt_dynamics(p, inst['x_lin'][i], inst['pf'][i])
                C = inst['C'][i]
                free = np.ones((N, 6))
                free[C == 0, 0:3] = 0
                if variant == '2f':
                    free[:, 1] = 0
                K, Gi = factor(Ad, Bd, free, N)
                H = dense_H(Ad, Bd, free, N)
                rng = np.random.default_rng(i)
                n = rng.normal(size=6 * N) * free.ravel()
                a = hinv(Ad, Bd, free, K, Gi, n, N)
                b = np.linalg.solve(H, n)
                print(variant, N, i, 'rel err %.2e' % (np.abs(a - b).max() / np.abs(b).max()),
                      'cond %.1e' % np.linalg.cond(H))


if __name__ == '__main__':
    main()


# ---------------------------------------------------------------------------
# the dual active set of the kernel (range-space Goldfarb-Idnani with the
# Cholesky R'R of N_A' H^-1 N_A; H^-1 by the Riccati sweeps)
# ---------------------------------------------------------------------------
TAU = (7.78, 7.78, 4.0)
KTOL = 1e-10


def solve_ric(variant, N, x_in, x_lin, x_ref, pf, C, mu, uref_aliased=True, qmax=None, trace=False):
    p = ho.MpcParams.runner(variant, N)
    Ad, Bd = ho.gen_dt_dynamics(p, x_lin, pf)
    NV = 6 * N
    free = np.ones((N, 6))
    free[C == 0, 0:3] = 0
    if variant == '2f':
        free[:, 1] = 0
    dt, m, g = p.t, p.m, p.g
    zc = dt * dt / m
    # free response, gradient h = 2 Gamma' W (xbar - r) - 2 V ubar
    xb = np.zeros((N + 1, 12))
    xb[0] = x_in
    Gd = np.zeros(12)
    Gd[8] = -g * dt
    for k in range(N):
        xb[k + 1] = Ad[k] @ xb[k] + Gd
    a = np.zeros(12)
    h = np.zeros((N, 6))
    for t in range(N, 0, -1):
        W = Q * (100 if t == N else 1)
        a = W * (xb[t] - x_ref[t - 1]) + (Ad[t].T @ a if t < N else 0)
        i = t - 1
        B = Bd[i] * free[i][None, :]
        h[i] = 2 * B.T @ a
        if i < N - 1 and free[i][2]:
            ub = (2 * m * g if C[N - 1 if uref_aliased else i] != 0 else 0.0)
            h[i][2] -= 2 * 0.001 * ub
    K, Gi = factor(Ad, Bd, free, N)
    Hinv = lambda n: hinv(Ad, Bd, free, K, Gi, n, N)  # noqa: E731
    v = Hinv(-h.ravel())
    zb = xb[:, 2]

    def heights(u):   # z_k of the homogeneous response, k = 0..N
        uz = u.reshape(N, 6)[:, 2] * C
        z = np.zeros(N + 1)
        for k in range(2, N + 1):
            z[k] = zc * sum((k - 1 - j) * uz[j] for j in range(k - 1))
        return z

    def cons(idx):   # (normal, rhs) of constraint id = 4 v + slot: n'u >= b
        vv, sl = divmod(idx, 4)
        k, c = divmod(vv, 6)
        n = np.zeros(NV)
        if c >= 3:
            if sl == 0:
                n[vv] = 1; b = -TAU[c - 3]
            elif sl == 1:
                n[vv] = -1; b = -TAU[c - 3]
            else:
                for j in range(k - 1):
                    if C[j] != 0:
                        n[6 * j + 2] = zc * (k - 1 - j)
                b = 0.1 - zb[k]
        elif c == 2:
            n[vv] = 1 if sl == 0 else -1
            b = 0.0 if sl == 0 else -206.0
        else:
            n[vv] = -1 if sl == 0 else 1
            n[6 * k + 2] = mu
            b = 0.0
        return n, b

    ids = []
    for k in range(N):
        for c in range(6):
            vv = 6 * k + c
            if c >= 3:
                ids += [4 * vv, 4 * vv + 1] + ([4 * vv + 2] if (c == 3 and k >= 2) else [])
            elif C[k] != 0 and not (variant == '2f' and c == 1):
                ids += [4 * vv, 4 * vv + 1]
    allc = {i: cons(i) for i in ids}
    status = 0
    if x_in[2] - 0.1 < -KTOL or zb[1] - 0.1 < -KTOL:
        status = 2
    act, ua = [], []
    R = np.zeros((0, 0))
    it = 0
    maxit = 4 * NV + 50
    while status == 0:
        best, p_ = np.inf, None
        for i in ids:
            if i in act:
                continue
            n, b = allc[i]
            nn = np.linalg.norm(n)
            s = n @ v - b
            sc = s / nn if nn > 0 else (-np.inf if s < -KTOL else np.inf)
            if sc < best or (sc == best and i < p_):
                best, p_ = sc, i
        if not best < -KTOL:
            break
        n_p, b_p = allc[p_]
        s = Hinv(n_p)
        sn = n_p @ s
        uplus = 0.0
        while True:
            it += 1
            if it > maxit:
                status = 1
                break
            q = len(act)
            NA = np.array([allc[i][0] for i in act]).reshape(q, NV)
            cv = NA @ s
            y = np.linalg.solve(R.T, cv) if q else np.zeros(0)
            r = np.linalg.solve(R, y) if q else np.zeros(0)
            nz = n_p - NA.T @ r
            z = Hinv(nz) if q else s
            zn = nz @ z
            has_z = zn > 1e-12 * sn
            t1, kd = np.inf, -1
            for j in range(q):
                if r[j] > 0 and ua[j] / r[j] < t1:
                    t1, kd = ua[j] / r[j], j
            slack = n_p @ v - b_p
            t2 = -slack / zn if has_z else np.inf
            t = min(t1, t2)
            if not t < np.inf:
                status = 2
                break
            if has_z:
                v = v + t * z
            ua = [ua[j] - t * r[j] for j in range(q)]
            uplus += t
            if has_z and t == t2:
                if qmax is not None and q >= qmax:
                    status = 3
                    break
                Rn = np.zeros((q + 1, q + 1))
                Rn[:q, :q] = R
                Rn[:q, q] = y
                Rn[q, q] = np.sqrt(zn)
                R = Rn
                act.append(p_)
                ua.append(uplus)
                break
            # drop kd: delete column kd, re-triangularise by Givens
            act.pop(kd)
            ua.pop(kd)
            R = np.delete(R, kd, axis=1)
            for j in range(kd, q - 1):
                aa, bb = R[j, j], R[j + 1, j]
                hh = np.hypot(aa, bb)
                cg, sg = aa / hh, bb / hh
                rj, rj1 = R[j].copy(), R[j + 1].copy()
                R[j], R[j + 1] = cg * rj + sg * rj1, -sg * rj + cg * rj1
            R = R[:q - 1, :q - 1]
        if trace:
            print('it', it, 'q', len(act), 'best', best)
    u = v.reshape(N, 6) * (status == 0)
    return dict(u=u, status=status, iters=it, nact=len(act))


def compare(variant='3f', N=10, B=64, seed=0, curve=True, musweep=True):
    from oracle import port
    inst = hp.sample_instances(B, N, curve=curve, seed=seed, mu_sweep=(0.3, 1.2) if musweep else None)
    ref = port.solve_batch(variant, N, inst['x_in'], inst['x_lin'], inst['x_ref'], inst['pf'], inst['C'],
                           mu=inst['mu'], nthreads=8)
    du, bad, its, nacts = 0.0, 0, [], []
    for i in range(B):
        r = solve_ric(variant, N, inst['x_in'][i], inst['x_lin'][i], inst['x_ref'][i], inst['pf'][i],
                      inst['C'][i], inst['mu'][i])
        if r['status'] != ref['status'][i]:
            bad += 1
            continue
        if r['status'] == 0:
            du = max(du, np.abs(r['u'] - ref['u'][i]).max())
        its.append(r['iters'])
        nacts.append(r['nact'])
    print(f'{variant} N={N} B={B}: status mismatches {bad}, max|du| {du:.2e}, iters mean '
          f'{np.mean(its):.2f} max {max(its)}, active max {max(nacts)}')
