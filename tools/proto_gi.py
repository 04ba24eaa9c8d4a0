"""Design model of the device algorithm (numpy) -- development tool only.

Mirrors, step for step, what ``csrc/hmpc_kernels.hip`` does for ONE instance,
so that numerics (condensing, Cholesky, J = L^-T, Goldfarb-Idnani dual
active set with Householder adds / Givens drops) can be checked against the
oracle on the CPU before running on the GPU.  Not part of the product and
not the oracle.
"""
import numpy as np

NX, NU = 12, 6


def setup(p, x_in, x_lin, x_ref, pf, C, mu, uref_mode='aliased'):
    N, dt, m = p.N, p.t, p.m
    NV = NU * N
    # --- per-stage linearisation (kernel phase 1)
    cs = np.zeros((N, 2))
    Bd = np.zeros((N, 6, 6))          # rows 6..11 of Bd_k
    for k in range(N):
        c, s = np.cos(x_lin[k, 5]), np.sin(x_lin[k, 5])
        Rz = np.array([[c, s, 0], [-s, c, 0], [0, 0, 1.]])
        rf = p.rh + Rz @ (pf[k] - x_lin[k, 0:3])
        Jw = Rz @ p.Jinv @ Rz.T
        B = np.zeros((6, 6))
        if p.variant == '3f':
            B[0:3, 0:3] = np.eye(3) / m
            r = Rz.T @ rf
            rhat = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
            B[3:6, 0:3] = Jw @ rhat
        else:
            B[0:3, 0:3] = Rz.T / m
            rhat = np.array([[0, -rf[2], rf[1]], [rf[2], 0, -rf[0]], [-rf[1], rf[0], 0]])
            B[3:6, 0:3] = Jw @ Rz.T @ rhat
        B[3:6, 3:6] = Jw @ Rz.T
        Bd[k] = B * dt
        cs[k] = c, s

    def Ad_mul(k, x):          # Ad_k x
        c, s = cs[k]
        Rz = np.array([[c, s, 0], [-s, c, 0], [0, 0, 1.]])
        y = x.copy()
        y[0:3] += dt * x[6:9]
        y[3:6] += dt * (Rz @ x[9:12])
        return y

    def AdT_mul(k, x):         # Ad_k' x
        c, s = cs[k]
        Rz = np.array([[c, s, 0], [-s, c, 0], [0, 0, 1.]])
        y = x.copy()
        y[6:9] += dt * x[0:3]
        y[9:12] += dt * (Rz.T @ x[3:6])
        return y

    Gd = np.zeros(NX); Gd[8] = -p.g * dt
    # --- free response
    xb = np.zeros((N + 1, NX)); xb[0] = x_in
    for k in range(N):
        xb[k + 1] = Ad_mul(k, xb[k]) + Gd
    W = [np.array([50., 50., 2., 1., 1., 50., 1., 1., 1., 10., 10., 10.]) * (100 if k == N - 1 else 1)
         for k in range(N)]
    V = [np.full(6, 0.001) * (0 if k == N - 1 else 1) for k in range(N)]
    ubar = np.zeros((N, 6))
    for k in range(N):
        kk = N - 1 if uref_mode == 'aliased' else k
        ubar[k, 2] = 2 * p.m * p.g if C[kk] != 0 else 0
    # --- S recursion, Y_j = S_{j+1} Bd_j  (Bd nonzero rows 6..11)
    Y = np.zeros((N, NX, NU))
    S = np.diag(W[N - 1])
    for t in range(N, 0, -1):        # S_t
        if t < N:
            # S_t = W_{t-1} + Ad_t' S_{t+1} Ad_t
            T = np.array([AdT_mul(t, S[:, c]) for c in range(NX)]).T   # Ad_t' S
            M = T.T                                                      # S Ad_t
            S = np.diag(W[t - 1]) + np.array([AdT_mul(t, M[:, c]) for c in range(NX)]).T
        Y[t - 1] = S[:, 6:12] @ Bd[t - 1]
    # --- H lower rows, via Z propagation
    H = np.zeros((NV, NV))
    for v in range(NV):
        j, c = divmod(v, 6)
        Z = Y[j][:, c].copy()
        for i in range(j, -1, -1):
            if i < j:
                Z = AdT_mul(i + 1, Z)
            H[v, 6 * i:6 * i + 6] = 2 * Bd[i].T @ Z[6:12]
        H[v, v] += 2 * V[j][c]
    H = np.tril(H) + np.tril(H, -1).T
    # --- linear term via adjoint
    a = np.zeros((N + 2, NX))
    for t in range(N, 0, -1):
        a[t] = W[t - 1] * (xb[t] - x_ref[t - 1]) + (AdT_mul(t, a[t + 1]) if t < N else 0)
    h = np.zeros(NV)
    for j in range(N):
        h[6 * j:6 * j + 6] = 2 * Bd[j].T @ a[j + 1][6:12] - 2 * V[j] * ubar[j]
    # --- fixed variables
    fixed = np.zeros(NV, bool)
    for k in range(N):
        if C[k] == 0:
            fixed[6 * k + 0] = fixed[6 * k + 1] = fixed[6 * k + 2] = True
        if p.variant == '2f':
            fixed[6 * k + 1] = True
    H[fixed, :] = 0; H[:, fixed] = 0; H[fixed, fixed] = 1; h[fixed] = 0
    # --- constraints n'v >= b
    cons = []
    for k in range(N):
        for ax, lim in ((3, 7.78), (4, 7.78), (5, 4.0)):
            e = np.zeros(NV); e[6 * k + ax] = 1
            cons.append((e, -lim)); cons.append((-e, -lim))
        if C[k] != 0:
            e = np.zeros(NV); e[6 * k + 2] = 1
            cons.append((e, 0.0)); cons.append((-e, -206.0))
            for ax in ((0, 1) if p.variant == '3f' else (0,)):
                n1 = np.zeros(NV); n1[6 * k + ax] = -1; n1[6 * k + 2] = mu
                n2 = np.zeros(NV); n2[6 * k + ax] = 1; n2[6 * k + 2] = mu
                cons.append((n1, 0.0)); cons.append((n2, 0.0))
    infeasible_const = x_in[2] < 0.1 - 1e-12 or xb[1, 2] < 0.1 - 1e-12
    for k in range(2, N):
        n = np.zeros(NV)
        for j in range(k - 1):
            if not fixed[6 * j + 2]:
                n[6 * j + 2] = dt * Bd[j][2, 2] * (k - 1 - j)
        cons.append((n, 0.1 - xb[k, 2]))
    return dict(H=H, h=h, cons=cons, fixed=fixed, xb=xb, Bd=Bd, cs=cs, Gd=Gd, ubar=ubar,
                infeasible_const=infeasible_const, Ad_mul=Ad_mul, W=W, V=V)


def gi(H, h, cons, tol=1e-10, max_iter=500):
    NV = H.shape[0]
    L = np.linalg.cholesky(H)
    J = np.linalg.inv(L).T
    v = -J @ (J.T @ h)
    q = 0
    R = np.zeros((NV, NV))
    act, u = [], []
    norms = np.array([max(np.linalg.norm(n), 1e-300) for n, _ in cons])
    it = 0
    adds = drops = 0
    while True:
        s = np.array([n @ v - b for n, b in cons])
        sc = s / norms
        sc[act] = np.inf
        sc[norms < 1e-200] = np.where(s[norms < 1e-200] < -tol, -np.inf, np.inf)
        p = int(np.argmin(sc))
        if sc[p] >= -tol:
            return dict(v=v, status=0, act=act, u=u, iters=it, adds=adds, drops=drops)
        n_p, b_p = cons[p]
        u_plus = 0.0
        while True:
            it += 1
            if it > max_iter:
                return dict(v=v, status=3, act=act, u=u, iters=it, adds=adds, drops=drops)
            d = J.T @ n_p
            z = J[:, q:] @ d[q:]
            r = np.linalg.solve(np.triu(R[:q, :q]), d[:q]) if q else np.zeros(0)
            t1, k = np.inf, -1
            for j in range(q):
                if r[j] > 0:
                    ratio = u[j] / r[j]
                    if ratio < t1:
                        t1, k = ratio, j
            zn = d[q:] @ d[q:]
            s_p = n_p @ v - b_p
            t2 = -s_p / zn if zn > 1e-30 * max(1.0, d @ d) else np.inf
            t = min(t1, t2)
            if t == np.inf:
                return dict(v=v, status=2, act=act, u=u, iters=it, adds=adds, drops=drops)
            for j in range(q):
                u[j] -= t * r[j]
            u_plus += t
            if t2 < np.inf:
                v = v + t * z
            if t2 < np.inf and t == t2:
                # add p: Householder on d[q:]
                w = d[q:].copy()
                nrm = np.linalg.norm(w)
                alpha = -np.copysign(nrm, w[0])
                w[0] -= alpha
                ww = w @ w
                if ww > 0:
                    J[:, q:] -= np.outer(J[:, q:] @ w, w) * (2.0 / ww)
                R[:q, q] = d[:q]
                R[q, q] = alpha
                q += 1
                act.append(p); u.append(u_plus)
                adds += 1
                break
            # drop k
            drops += 1
            Rq = np.delete(R[:q, :q], k, axis=1)
            for l in range(k, q - 1):
                a_, b_ = Rq[l, l], Rq[l + 1, l]
                hh = np.hypot(a_, b_)
                c, s_ = a_ / hh, b_ / hh
                rl, rl1 = Rq[l].copy(), Rq[l + 1].copy()
                Rq[l], Rq[l + 1] = c * rl + s_ * rl1, -s_ * rl + c * rl1
                jl, jl1 = J[:, l].copy(), J[:, l + 1].copy()
                J[:, l], J[:, l + 1] = c * jl + s_ * jl1, -s_ * jl + c * jl1
            R[:] = 0
            R[:q - 1, :q - 1] = Rq[:q - 1]
            q -= 1
            del act[k]; del u[k]


def solve(p, x_in, x_lin, x_ref, pf, C, mu, uref_mode='aliased'):
    S = setup(p, x_in, x_lin, x_ref, pf, C, mu, uref_mode)
    if S['infeasible_const']:
        return dict(status=2)
    res = gi(S['H'], S['h'], S['cons'])
    v = res['v']
    u = v.reshape(p.N, 6)
    x = np.zeros((p.N + 1, NX)); x[0] = x_in
    obj = 0.0
    for k in range(p.N):
        x[k + 1] = S['Ad_mul'](k, x[k]) + np.concatenate([np.zeros(6), S['Bd'][k] @ u[k]]) + S['Gd']
        e = x[k + 1] - x_ref[k]
        du = u[k] - S['ubar'][k]
        obj += e @ (S['W'][k] * e) + du @ (S['V'][k] * du)
    res.update(u=u, x=x, obj=obj, H=S['H'], h=S['h'])
    return res
