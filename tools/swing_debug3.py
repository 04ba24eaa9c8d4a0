"""Swing-class debug 3 (the HMPC_SWING_DEBUG library): the kernel's v0, first
w = L^-1 n_p, first z = L^-T w and the first iteration's scalars against a
numpy condensing of the same all-swing QP (torques only)."""
import sys, os
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'hopper-mpc-inertial_amd')); sys.path.insert(0, ROOT)
import hmpc, hmpc_plan as hp
from oracle import hmpc_oracle as ho, port
N = 10
a = hp.sample_instances(4096, N, curve=True, seed=11, mu_sweep=(0.3, 1.2))
sw = np.where((a['C'] != 0).sum(1) == 0)[0]
keys = ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')
pr = port.solve_batch('3f', N, *[np.ascontiguousarray(a[k][sw]) for k in keys[:5]], mu=a['mu'][sw], nthreads=8)
hard = sw[pr['iters'] > 0][:8]
idx = np.repeat(hard, 2)
inst = {k: np.ascontiguousarray(a[k][idx]) for k in keys}
c = hp.runner_constants()
d = {k: torch.from_numpy(inst[k]).cuda() for k in keys}
cx = hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'], device=0)
print(cx.kernel_name)
o = cx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
torch.cuda.synchronize()
o = {k: v.cpu().numpy() for k, v in o.items()}
cx.close()
lim = np.tile([7.78, 7.78, 4.0], N)
for n, i in enumerate(idx):
    p = ho.MpcParams.runner('3f', N, mu=float(inst['mu'][n]))
    _, _, Gd = ho.constant_matrices(p)
    Ad, Bd = ho.gen_dt_dynamics(p, inst['x_lin'][n], inst['pf'][n])
    # condensed torque problem: x_{k+1} = xbar_{k+1} + sum_j Phi B_j u_j
    xbar = ho.rollout(p, inst['x_in'][n], np.zeros((N, 6)), Ad, Bd, Gd)
    G = np.zeros((N, 12, 3 * N))
    for k in range(N):
        for j in range(k + 1):
            M = Bd[j][:, 3:6]
            for l in range(j + 1, k + 1):
                M = Ad[l] @ M
            G[k, :, 3 * j:3 * j + 3] = M
    H = np.zeros((3 * N, 3 * N)); h = np.zeros(3 * N)
    for k in range(N):
        W = np.diag(ho.Q_DIAG * (100 if k == N - 1 else 1))
        H += 2 * G[k].T @ W @ G[k]
        h += 2 * G[k].T @ W @ (xbar[k + 1] - inst['x_ref'][n][k])
    for k in range(N - 1):
        H[3 * k:3 * k + 3, 3 * k:3 * k + 3] += 2 * 0.001 * np.eye(3)
    v0 = -np.linalg.solve(H, h)
    L = np.linalg.cholesky(H)
    xo = o['x'][n].ravel()
    g_v0, g_w, g_z, g_s = xo[0:30], xo[32:62], xo[64:94], xo[96:128]
    sc = np.concatenate([v0 + lim, lim - v0])
    ids = np.concatenate([4 * np.arange(30), 4 * np.arange(30) + 1])
    order = np.lexsort((ids, sc))
    pcpu = ids[order[0]]
    o_ = pcpu >> 2
    npv = np.zeros(30); npv[o_] = 1.0 if (pcpu & 3) == 0 else -1.0
    w = np.linalg.solve(L, npv); z = np.linalg.solve(L.T, w)
    print(f'n={n} inst {i} half {n % 2}: |v0-gpu| {np.abs(v0 - g_v0).max():.2e}  p cpu {pcpu} gpu {g_s[0]:.0f}  '
          f'wn2 cpu {w @ w:.6e} gpu {g_s[1]:.6e}  |w-gpu| {np.abs(w - g_w).max():.2e}  |z-gpu| {np.abs(z - g_z).max():.2e}')
    print(f'      t1 {g_s[2]:.4g} t2 {g_s[3]:.4g} sp {g_s[4]:.4g} (cpu {npv @ v0 - (-lim[o_]):.4g}) zn {g_s[5]:.4g} q {g_s[6]} bp {g_s[7]}  seq {g_s[8:20]}')
    print(f'      iters gpu {o["iters"][n]} port {pr["iters"][np.searchsorted(sw, i)]}')
