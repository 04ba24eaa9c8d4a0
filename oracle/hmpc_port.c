/*
 * TEST INFRASTRUCTURE ONLY -- never linked, loaded or called by the product
 * path (hopper-mpc-inertial_amd/).  Users: tests/ (second checker next to the
 * numpy oracle) and bench.py's cpu_baseline leg (the "port" CPU baseline,
 * OpenMP over instances).
 *
 * A plain-C restatement of the reference's per-timestep QP,
 *   Mpc.gen_dt_dynamics  src/mpc_cvx_euler_3f.py:71-94, 2f :70-94
 *   Mpc.build_qp         src/mpc_cvx_euler_3f.py:96-153, 2f :96-151
 *   Mpc.solve_qp         src/mpc_cvx_euler_3f.py:155-160 (cvxpy -> OSQP)
 * condensed DENSELY (explicit impulse-response matrix Gamma, H = 2 Gamma' W
 * Gamma + 2 V) and solved exactly by the classic Goldfarb-Idnani dual active
 * set method with an explicit J = L^-T Q (Givens updates).  Deliberately a
 * different formulation and a different solver organisation from the GPU
 * kernel (which condenses through a structured cost-to-go recursion and runs
 * a range-space active set), so agreement is evidence, not an echo.
 *
 * Pinning: tests/test_oracle_port.py checks this port against the golden
 * fixtures recorded from the reference's own build_qp (tests/golden/qp_*.npz,
 * u* within 1e-7, objective within 1e-9 relative) and against the numpy
 * oracle on freshly drawn instances.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define NX 12
#define NU 6

static const double QD[NX] = {50, 50, 2, 1, 1, 50, 1, 1, 1, 10, 10, 10}; /* 3f :35 */
#define RD 0.001    /* R = 0.001 I, :37           */
#define TERMQ 100.0 /* kf at k = N-1, :113        */
#define FZMAX 206.0 /* f_max[2], :20              */
#define ZMIN 0.1    /* z >= 0.1, :129             */
#define TOL 1e-10   /* scaled primal feasibility  */

enum { ST_SOLVED = 0, ST_MAXIT = 1, ST_INFEAS = 2, ST_NUMERICAL = 3 };

typedef struct {
  int variant, N, uref_aliased;
  double t, m, g, mu;
  const double *Jinv, *rh;
} prm;

/* ------------------------------------------------------------------------ */
/* gen_dt_dynamics: Ad (N,12,12), Bd (N,12,6), row-major                     */
/* ------------------------------------------------------------------------ */
static void mat3(const double* a, const double* b, double* c) { /* c = a b */
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      c[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}

static void dynamics(const prm* p, const double* xl, const double* pf, double* Ad, double* Bd) {
  const int N = p->N;
  const double dt = p->t;
  for (int k = 0; k < N; ++k) {
    const double psi = xl[12 * k + 5], c = cos(psi), s = sin(psi);
    const double Rz[9] = {c, s, 0, -s, c, 0, 0, 0, 1}; /* rz, src/utils.py:46-51 */
    const double RzT[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
    double d[3], rf[3], tmp[9], Jw[9], Bwt[9], Bwf[9], hw[9], w[3];
    for (int i = 0; i < 3; ++i) d[i] = pf[3 * k + i] - xl[12 * k + i];
    for (int i = 0; i < 3; ++i) rf[i] = p->rh[i] + Rz[3 * i] * d[0] + Rz[3 * i + 1] * d[1] + Rz[3 * i + 2] * d[2];
    mat3(Rz, p->Jinv, tmp);
    mat3(tmp, RzT, Jw); /* J_w_inv = Rz Jinv Rz'   (:86) */
    mat3(Jw, RzT, Bwt); /* B[9:12,3:6]             (:89) */
    if (p->variant == 3) {
      for (int i = 0; i < 3; ++i) w[i] = RzT[3 * i] * rf[0] + RzT[3 * i + 1] * rf[1] + RzT[3 * i + 2] * rf[2];
    } else {
      for (int i = 0; i < 3; ++i) w[i] = rf[i];
    }
    /* hat, src/utils.py:21-25 */
    hw[0] = 0; hw[1] = -w[2]; hw[2] = w[1];
    hw[3] = w[2]; hw[4] = 0; hw[5] = -w[0];
    hw[6] = -w[1]; hw[7] = w[0]; hw[8] = 0;
    if (p->variant == 3) mat3(Jw, hw, Bwf);  /* 3f :88: Jw hat(Rz' rf)     */
    else mat3(Bwt, hw, Bwf);                 /* 2f :88: Jw Rz' hat(rf)     */
    double* A = Ad + 144 * k;
    double* B = Bd + 72 * k;
    memset(A, 0, 144 * sizeof(double));
    memset(B, 0, 72 * sizeof(double));
    for (int i = 0; i < NX; ++i) A[13 * i] = 1.0;
    for (int i = 0; i < 3; ++i) {
      A[12 * i + 6 + i] += dt;                                   /* A[0:3,6:9] = I      */
      for (int j = 0; j < 3; ++j) A[12 * (3 + i) + 9 + j] += dt * Rz[3 * i + j]; /* A[3:6,9:12] = Rz */
    }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        const double bv = (p->variant == 3) ? (i == j ? 1.0 / p->m : 0.0) : RzT[3 * i + j] / p->m;
        B[6 * (6 + i) + j] = bv * dt;                 /* 3f :28 I/m; 2f :87 Rz'/m */
        B[6 * (9 + i) + j] = Bwf[3 * i + j] * dt;
        B[6 * (9 + i) + 3 + j] = Bwt[3 * i + j] * dt;
      }
  }
}

/* ------------------------------------------------------------------------ */
/* dense Goldfarb-Idnani:  min 1/2 x'Hx + h'x  s.t.  Cn x >= cb              */
/* ------------------------------------------------------------------------ */
typedef struct {
  int n, m;
  double *H, *J, *R, *d, *z, *r, *u, *x, *s;
  int* act;
  char* isact;
} gi_ws;

static int chol(int n, double* A) { /* lower L in place (row-major), 0 on success */
  for (int j = 0; j < n; ++j) {
    double s = A[n * j + j];
    for (int k = 0; k < j; ++k) s -= A[n * j + k] * A[n * j + k];
    if (!(s > 0.0)) return -1;
    const double ljj = sqrt(s);
    A[n * j + j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double t = A[n * i + j];
      for (int k = 0; k < j; ++k) t -= A[n * i + k] * A[n * j + k];
      A[n * i + j] = t / ljj;
    }
  }
  return 0;
}

static int gi_solve(gi_ws* w, const double* h, const double* Cn, const double* cb, double* cnorm,
                    int* iters) {
  const int n = w->n, m = w->m;
  double *L = w->H, *J = w->J, *R = w->R, *d = w->d, *z = w->z, *r = w->r, *u = w->u, *x = w->x;
  int* act = w->act;
  char* isact = w->isact;
  if (chol(n, L)) return ST_NUMERICAL;
  /* J = L^-T (upper): solve L Y = I, J = Y' */
  memset(J, 0, sizeof(double) * n * n);
  for (int c = 0; c < n; ++c) {
    for (int i = c; i < n; ++i) {
      double t = (i == c) ? 1.0 : 0.0;
      for (int k = c; k < i; ++k) t -= L[n * i + k] * J[n * c + k];  /* Y[i][c] stored at J[c][i] */
      J[n * c + i] = t / L[n * i + i];
    }
  }
  /* J currently holds Y' with Y = L^-1 (J[c][i] = Y[i][c]) -> that is L^-T, upper */
  /* x = -J J' h */
  for (int i = 0; i < n; ++i) {
    double t = 0.0;
    for (int k = 0; k < n; ++k) t += J[n * k + i] * h[k]; /* (J' h)_i */
    d[i] = t;
  }
  for (int i = 0; i < n; ++i) {
    double t = 0.0;
    for (int k = 0; k < n; ++k) t += J[n * i + k] * d[k];
    x[i] = -t;
  }
  for (int i = 0; i < m; ++i) {
    double t = 0.0;
    for (int k = 0; k < n; ++k) t += Cn[n * i + k] * Cn[n * i + k];
    cnorm[i] = sqrt(t);
    isact[i] = 0;
  }
  int q = 0, it = 0;
  const int maxit = 4 * (n + m) + 50;
  for (;;) {
    /* most violated constraint (scaled) */
    int p = -1;
    double best = -TOL;
    for (int i = 0; i < m; ++i) {
      if (isact[i]) continue;
      double s = -cb[i];
      for (int k = 0; k < n; ++k) s += Cn[n * i + k] * x[k];
      double sc;
      if (cnorm[i] > 0.0) sc = s / cnorm[i];
      else sc = (s < -TOL) ? -INFINITY : INFINITY;
      if (sc < best) { best = sc; p = i; }
    }
    if (p < 0) break;
    const double* np = Cn + (size_t)n * p;
    double uplus = 0.0;
    for (;;) {
      if (++it > maxit) { *iters = it; return ST_MAXIT; }
      /* d = J' n_p, z = J2 d2, r = R^-1 d1 */
      for (int i = 0; i < n; ++i) {
        double t = 0.0;
        for (int k = 0; k < n; ++k) t += J[n * k + i] * np[k];
        d[i] = t;
      }
      double zz = 0.0;
      for (int i = 0; i < n; ++i) {
        double t = 0.0;
        for (int k = q; k < n; ++k) t += J[n * i + k] * d[k];
        z[i] = t;
      }
      for (int k = q; k < n; ++k) zz += d[k] * d[k];
      for (int i = q - 1; i >= 0; --i) {
        double t = d[i];
        for (int k = i + 1; k < q; ++k) t -= R[n * i + k] * r[k];
        r[i] = t / R[n * i + i];
      }
      double t1 = INFINITY;
      int kd = -1;
      for (int j = 0; j < q; ++j)
        if (r[j] > 0.0 && u[j] / r[j] < t1) { t1 = u[j] / r[j]; kd = j; }
      double sp = -cb[p];
      for (int k = 0; k < n; ++k) sp += np[k] * x[k];
      double dd = 0.0;
      for (int k = 0; k < n; ++k) dd += d[k] * d[k];
      const int has_z = zz > 1e-24 * dd;
      const double t2 = has_z ? -sp / zz : INFINITY; /* n_p' z = |d2|^2 */
      const double t = t1 < t2 ? t1 : t2;
      if (!(t < INFINITY)) { *iters = it; return ST_INFEAS; }
      if (has_z)
        for (int i = 0; i < n; ++i) x[i] += t * z[i];
      for (int j = 0; j < q; ++j) u[j] -= t * r[j];
      uplus += t;
      if (has_z && t == t2) {
        /* add p: Givens from the bottom zero d[q+1..n-1]; J <- J G' */
        for (int j = n - 1; j > q; --j) {
          const double a = d[j - 1], b = d[j];
          const double hh = hypot(a, b);
          if (hh == 0.0) continue;
          const double c = a / hh, s = b / hh;
          d[j - 1] = hh;
          d[j] = 0.0;
          for (int k = 0; k < n; ++k) {
            const double x0 = J[n * k + j - 1], x1 = J[n * k + j];
            J[n * k + j - 1] = c * x0 + s * x1;
            J[n * k + j] = -s * x0 + c * x1;
          }
        }
        for (int i = 0; i <= q; ++i) R[n * i + q] = d[i];
        act[q] = p;
        u[q] = uplus;
        isact[p] = 1;
        ++q;
        break;
      }
      /* drop kd: delete column kd of R, restore the triangle by Givens */
      isact[act[kd]] = 0;
      for (int j = kd; j < q - 1; ++j) {
        act[j] = act[j + 1];
        u[j] = u[j + 1];
        for (int i = 0; i <= j + 1; ++i) R[n * i + j] = R[n * i + j + 1];
      }
      for (int j = kd; j < q - 1; ++j) {
        const double a = R[n * j + j], b = R[n * (j + 1) + j];
        const double hh = hypot(a, b);
        if (hh == 0.0) continue;
        const double c = a / hh, s = b / hh;
        for (int k = j; k < q - 1; ++k) {
          const double r0 = R[n * j + k], r1 = R[n * (j + 1) + k];
          R[n * j + k] = c * r0 + s * r1;
          R[n * (j + 1) + k] = -s * r0 + c * r1;
        }
        for (int k = 0; k < n; ++k) {
          const double x0 = J[n * k + j], x1 = J[n * k + j + 1];
          J[n * k + j] = c * x0 + s * x1;
          J[n * k + j + 1] = -s * x0 + c * x1;
        }
      }
      for (int i = 0; i < q; ++i) R[n * i + q - 1] = (i == q - 1) ? 0.0 : R[n * i + q - 1];
      --q;
    }
  }
  *iters = it;
  return ST_SOLVED;
}

/* ------------------------------------------------------------------------ */
/* one QP: dense condensing of build_qp, exact solve, rollout + objective    */
/* ------------------------------------------------------------------------ */
static double uref_z(const prm* p, const double* C, int k) { /* :107,131,138 (aliasing) */
  const int kk = p->uref_aliased ? p->N - 1 : k;
  return C[kk] != 0.0 ? 2.0 * p->m * p->g : 0.0;
}

static int solve_one(const prm* p, const double* x_in, const double* x_lin, const double* x_ref,
                     const double* pf, const double* C, double* u_out, double* x_out, double* obj_out,
                     int* iters_out) {
  const int N = p->N, NV = NU * N, NR = NX * N;
  const double dt = p->t;
  int status = ST_SOLVED;
  double* Ad = malloc(sizeof(double) * (144 * N + 72 * N + (size_t)NR * NV + NX * (N + 1)));
  double* Bd = Ad + 144 * N;
  double* Gm = Bd + 72 * N;   /* Gamma: row (t-1)*12 + r, column v, t = 1..N */
  double* xb = Gm + (size_t)NR * NV;
  dynamics(p, x_lin, pf, Ad, Bd);
  /* free response (Gd = [0..,-g dt,..] in row 8) */
  memcpy(xb, x_in, NX * sizeof(double));
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < NX; ++i) {
      double t = (i == 8) ? -p->g * dt : 0.0;
      for (int j = 0; j < NX; ++j) t += Ad[144 * k + 12 * i + j] * xb[NX * k + j];
      xb[NX * (k + 1) + i] = t;
    }
  /* Gamma */
  memset(Gm, 0, sizeof(double) * (size_t)NR * NV);
  for (int jst = 0; jst < N; ++jst)
    for (int c = 0; c < NU; ++c) {
      const int v = NU * jst + c;
      for (int r = 0; r < NX; ++r) Gm[(size_t)NV * (NX * jst + r) + v] = Bd[72 * jst + 6 * r + c];
      for (int t = jst + 1; t < N; ++t)
        for (int r = 0; r < NX; ++r) {
          double s = 0.0;
          for (int q = 0; q < NX; ++q) s += Ad[144 * t + 12 * r + q] * Gm[(size_t)NV * (NX * (t - 1) + q) + v];
          Gm[(size_t)NV * (NX * t + r) + v] = s;
        }
    }
  /* free variables: swing forces (:134-136) and 2f fy (2f :129) are fixed at 0 */
  int* fr = malloc(sizeof(int) * NV);
  int nf = 0;
  for (int v = 0; v < NV; ++v) {
    const int k = v / NU, c = v % NU;
    const int fixed = (c < 3 && C[k] == 0.0) || (p->variant == 2 && c == 1);
    if (!fixed) fr[nf++] = v;
  }
  /* H = 2 Gamma' W Gamma + 2 V, h = 2 Gamma' W (xbar - r) - 2 V ubar (cost :132,:139) */
  gi_ws w;
  const int mmax = 13 * N;   /* 6 torque + 2 fz + 4 friction rows per stage, N-1 z rows */
  w.n = nf;
  double* buf = malloc(sizeof(double) * ((size_t)3 * nf * nf + 6 * nf + 2 * (size_t)mmax + (size_t)mmax * nf + nf));
  w.H = buf;
  w.J = w.H + (size_t)nf * nf;
  w.R = w.J + (size_t)nf * nf;
  w.d = w.R + (size_t)nf * nf;
  w.z = w.d + nf;
  w.r = w.z + nf;
  w.u = w.r + nf;
  w.x = w.u + nf;
  w.s = w.x + nf;
  double* h = w.s + nf;
  double* cb = h + nf;
  double* cn = cb + mmax;
  double* Cn = cn + mmax;
  w.act = malloc(sizeof(int) * (nf + 1));
  w.isact = malloc(mmax);
  for (int a = 0; a < nf; ++a) {
    const int va = fr[a];
    for (int b2 = 0; b2 <= a; ++b2) {
      const int vb = fr[b2];
      double s = 0.0;
      for (int row = 0; row < NR; ++row) {
        const double ga = Gm[(size_t)NV * row + va];
        if (ga == 0.0) continue;
        const int t = row / NX;
        const double wt = QD[row % NX] * (t == N - 1 ? TERMQ : 1.0);
        s += ga * wt * Gm[(size_t)NV * row + vb];
      }
      s *= 2.0;
      if (a == b2 && va / NU != N - 1) s += 2.0 * RD;
      w.H[nf * a + b2] = s;
      w.H[nf * b2 + a] = s;
    }
    double s = 0.0;
    for (int row = 0; row < NR; ++row) {
      const int t = row / NX, r = row % NX;
      const double wt = QD[r] * (t == N - 1 ? TERMQ : 1.0);
      s += Gm[(size_t)NV * row + va] * wt * (xb[NX * (t + 1) + r] - x_ref[NX * t + r]);
    }
    h[a] = 2.0 * s;
    if (va % NU == 2 && va / NU != N - 1) h[a] -= 2.0 * RD * uref_z(p, C, va / NU);
  }
  /* constraints n'u >= b over the free variables */
  int m = 0;
  int* pos = malloc(sizeof(int) * NV); /* free index of variable v, or -1 */
  for (int v = 0; v < NV; ++v) pos[v] = -1;
  for (int a = 0; a < nf; ++a) pos[fr[a]] = a;
#define ROW_BEGIN() do { memset(Cn + (size_t)nf * m, 0, sizeof(double) * nf); } while (0)
#define COEF(v, val) do { if (pos[(v)] >= 0) Cn[(size_t)nf * m + pos[(v)]] += (val); } while (0)
  const double taulim[3] = {7.78, 7.78, 4.0}; /* :123-128 */
  for (int k = 0; k < N; ++k) {
    for (int a = 0; a < 3; ++a) {
      ROW_BEGIN(); COEF(NU * k + 3 + a, 1.0); cb[m++] = -taulim[a];
      ROW_BEGIN(); COEF(NU * k + 3 + a, -1.0); cb[m++] = -taulim[a];
    }
    if (C[k] != 0.0) { /* stance: :141-146 (2f :141-144) */
      ROW_BEGIN(); COEF(NU * k + 2, 1.0); cb[m++] = 0.0;
      ROW_BEGIN(); COEF(NU * k + 2, -1.0); cb[m++] = -FZMAX;
      const int nfr = (p->variant == 3) ? 2 : 1;
      for (int a = 0; a < nfr; ++a) {
        ROW_BEGIN(); COEF(NU * k + a, -1.0); COEF(NU * k + 2, p->mu); cb[m++] = 0.0;
        ROW_BEGIN(); COEF(NU * k + a, 1.0); COEF(NU * k + 2, p->mu); cb[m++] = 0.0;
      }
    }
  }
  /* z_k >= 0.1, k = 0..N-1 (:129): z_k = xbar_k[2] + Gamma row (k, 2) u */
  if (x_in[2] < ZMIN - TOL) status = ST_INFEAS;
  for (int k = 1; k < N && status == ST_SOLVED; ++k) {
    ROW_BEGIN();
    double nz = 0.0;
    for (int a = 0; a < nf; ++a) {
      const double gv = Gm[(size_t)NV * (NX * (k - 1) + 2) + fr[a]];
      Cn[(size_t)nf * m + a] = gv;
      nz += fabs(gv);
    }
    const double rhs = ZMIN - xb[NX * k + 2];
    if (nz == 0.0) {
      if (-rhs < -TOL) status = ST_INFEAS;   /* constant row violated */
      continue;
    }
    cb[m++] = rhs;
  }
#undef ROW_BEGIN
#undef COEF
  w.m = m;
  int iters = 0;
  if (status == ST_SOLVED) status = gi_solve(&w, h, Cn, cb, cn, &iters);
  /* u (fixed variables 0), x by rollout, objective on the trajectory */
  for (int v = 0; v < NV; ++v) u_out[v] = (pos[v] >= 0 && status == ST_SOLVED) ? w.x[pos[v]] : 0.0;
  double obj = 0.0;
  double* xx = x_out;
  memcpy(xx, x_in, NX * sizeof(double));
  for (int k = 0; k < N; ++k) {
    for (int i = 0; i < NX; ++i) {
      double t = (i == 8) ? -p->g * dt : 0.0;
      for (int j = 0; j < NX; ++j) t += Ad[144 * k + 12 * i + j] * xx[NX * k + j];
      for (int c = 0; c < NU; ++c) t += Bd[72 * k + 6 * i + c] * u_out[NU * k + c];
      xx[NX * (k + 1) + i] = t;
    }
    const double kf = (k == N - 1) ? TERMQ : 1.0, kuf = (k == N - 1) ? 0.0 : 1.0;
    for (int i = 0; i < NX; ++i) {
      const double e = xx[NX * (k + 1) + i] - x_ref[NX * k + i];
      obj += kf * QD[i] * e * e;
    }
    for (int c = 0; c < NU; ++c) {
      const double du = u_out[NU * k + c] - (c == 2 ? uref_z(p, C, k) : 0.0);
      obj += kuf * RD * du * du;
    }
  }
  *obj_out = obj;
  *iters_out = iters;
  free(w.act);
  free(w.isact);
  free(pos);
  free(buf);
  free(fr);
  free(Ad);
  return status;
}

/* ------------------------------------------------------------------------ */
/* exported                                                                  */
/* ------------------------------------------------------------------------ */
int hport_version(void) { return 10000; }

/* B instances (row-major batch arrays as in include/hmpc.h); mu may be NULL.
   Returns the number of instances solved (status 0). */
long hport_solve_batch(int variant, int N, double t, double m, double g, double mu_default,
                       const double* Jinv, const double* rh, int uref_aliased, long B,
                       const double* x_in, const double* x_lin, const double* x_ref,
                       const double* pf, const double* C, const double* mu, double* u, double* x,
                       double* obj, int* status, int* iters, int nthreads) {
  long solved = 0;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 8) num_threads(nthreads) reduction(+ : solved)
  for (long b = 0; b < B; ++b) {
    prm p = {variant, N, uref_aliased, t, m, g, mu ? mu[b] : mu_default, Jinv, rh};
    int it = 0;
    double ob = 0.0;
    const int st = solve_one(&p, x_in + 12 * b, x_lin + 12 * (N + 1) * b, x_ref + 12 * N * b,
                             pf + 3 * N * b, C + N * b, u + 6 * N * b, x + 12 * (N + 1) * b, &ob, &it);
    obj[b] = ob;
    status[b] = st;
    if (iters) iters[b] = it;
    solved += (st == ST_SOLVED);
  }
  return solved;
}
