// hmpc_cas.hip -- the reference's CasADi variant (src/mpc_cas_euler_3f.py,
// SURVEY.md 8f row 4) as the QP it actually builds, solved exactly on the
// GPU: one wavefront per instance, persistent grid.
//
// What the reference constructs (oracle/cas_oracle.py restates it; the
// problem data is pinned to a recording of the reference, tests/golden/
// cas_N10.npz):
//   min  sum_{k<N} |x_k - x_ref_k|^2 + 0.01 |u_k - 2 m g 1|^2        (:58-70)
//   s.t. x_0[i] = x_in[i] for i <= N, x_0[i] <= x_in[i] beyond      (:61,97-98)
//        x_{k+1} <= Ad x_k + Bd u_k + Gd   (one-sided, every row)     (:71-72,97-99)
//        +-fx - mu fz <= 0 every stage, +-fy - mu fz <= 0 last stage  (:73-76)
//        fx, fy in [-200 C, 200 C], fz in [0, 400 C]                  (:121-134)
// with the second-order discretisation M = I + A_bar t + t^2/2 A_bar^2 of
// [A B G] at the yaw of x_in (:44-50, :139) and the foot vector fixed at
// [0, 0, -0.2] (:39-41).  x_N is uncosted and only bounded above, so it is
// eliminated (reported on its dynamics bound); the remaining Hessian is
// DIAGONAL (2 on states, 0.02 on inputs) -- there is nothing to factorise.
//
// Solver: Goldfarb-Idnani dual active set in range-space form, R'R = N_A'
// H^-1 N_A (the Riccati kernel's scheme with H^-1 a diagonal scaling):
// s = H^-1 n_p is sparse, c = N_A's by sparse row dots (lane per active
// row), z = H^-1 (n_p - N_A r) by a per-variable gather over the <= 12 rows
// that can touch the variable.  R (capacity NV) lives in the workgroup's
// global slot.  N <= 11: the reference's lbg = 0 block then covers the
// initial condition only (N + 1 <= 12 rows), every dynamics row one-sided.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "hmpc_internal.h"
#include "hmpc_model.h"

namespace hmpc {

namespace {

constexpr int RT = 64;
constexpr int NVMAX = 18 * kCasNmax;               // 198 variables
constexpr int EV = (NVMAX + 63) / 64;              // variables per lane
constexpr int MMAX = 20 * kCasNmax + 2;            // 222 rows
constexpr int ER = (MMAX + 63) / 64;               // rows per lane
constexpr double kCasTol = 1e-10;

__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }
__device__ __forceinline__ void gsync() { __syncthreads(); }
__device__ __forceinline__ int loff(int r) { return (r * (r + 1)) >> 1; }

// per-instance data in LDS (doubles)
struct CasLay {
  int XIN, XR, CC, BD, RZ, GD, V, S, NB, Z, HI, RN, POS, ACT, UA, CB, SD, total;
  __host__ __device__ explicit CasLay(int N) {
    const int NV = 18 * N, M = 20 * N + 2;
    int o = 0;
    XIN = o; o += 12;
    XR = o; o += 12 * N;      // x_ref rows (cost)
    CC = o; o += (N + 1) & ~1;
    BD = o; o += 72;          // Bd (12 x 6)
    RZ = o; o += 10;          // rz(psi) (9) + mu
    GD = o; o += 12;          // Gd
    V = o; o += NV;           // primal iterate
    S = o; o += NV;           // H^-1 n_p
    NB = o; o += NV;          // n_p - N_A r
    Z = o; o += NV;           // H^-1 (n_p - N_A r)
    HI = o; o += NV;          // H^-1 diagonal (0: fixed variable)
    RN = o; o += M;           // row norms
    POS = o; o += M;          // active position of a row (int), -1 if inactive
    ACT = o; o += NV;         // active rows (int)
    UA = o; o += NV;          // multipliers
    CB = o; o += NV;          // r of the dual step
    SD = o; o += NV;          // subdiagonal of a drop
    total = o;
  }
};

// Rows (reference form n'z <= b); ids:
//   [0, 12(N-1))        dynamics (k, i) = 12 k + i, k <= N-2
//   D0 + i              initial condition x_0[i] <= x_in[i], i > N (D0 = 12(N-1))
//   F0 + 2k + s         friction +-fx_k - mu fz_k (F0 = D0 + 12)
//   F0 + 2N + s         friction +-fy_{N-1} - mu fz_{N-1}
//   B0 + 6k + j         bounds fx<=, -fx<=, fy<=, -fy<=, fz<=, -fz<= (B0 = F0 + 2N + 2)
// Variables: x_k[i] = 12 k + i (k < N), u_k[c] = 12 N + 6 k + c.
struct CasCtx {
  int N, NV, M, D0, F0, B0;
  double t, mu;
  const double* Bd;   // LDS
  const double* rz;   // LDS
  const double* xin;
  const double* cc;
};

template <typename F>
__device__ __forceinline__ void row_terms(const CasCtx& q, int id, F&& emit) {
  const int N = q.N;
  if (id < q.D0) {
    const int k = id / 12, i = id - 12 * k;
    emit(12 * (k + 1) + i, 1.0);
    emit(12 * k + i, -1.0);
    if (i < 3) emit(12 * k + 6 + i, -q.t);
    else if (i < 6) {
#pragma unroll
      for (int j = 0; j < 3; ++j) emit(12 * k + 9 + j, -q.t * q.rz[3 * (i - 3) + j]);
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const double b = q.Bd[6 * i + c];
      if (b != 0.0) emit(12 * N + 6 * k + c, -b);
    }
  } else if (id < q.F0) {
    emit(id - q.D0, 1.0);
  } else if (id < q.B0) {
    const int f = id - q.F0;
    const int k = f < 2 * N ? f >> 1 : N - 1;
    const int c = f < 2 * N ? 0 : 1;
    emit(12 * N + 6 * k + c, (f & 1) ? -1.0 : 1.0);
    emit(12 * N + 6 * k + 2, -q.mu);
  } else {
    const int f = id - q.B0, k = f / 6, j = f - 6 * k;
    emit(12 * N + 6 * k + (j >> 1), (j & 1) ? -1.0 : 1.0);
  }
}

__device__ __forceinline__ double row_rhs(const CasCtx& q, int id, const double* Gd) {
  if (id < q.D0) return Gd[id % 12];
  if (id < q.F0) return q.xin[id - q.D0];
  if (id < q.B0) return 0.0;
  const int f = id - q.B0, k = f / 6, j = f - 6 * k;
  if (j < 4) return 200.0 * q.cc[k];
  return j == 4 ? 400.0 * q.cc[k] : 0.0;
}

// a row exists (initial-condition rows only beyond N; bounds only for stance
// stages: a swing stage's forces are fixed at 0)
__device__ __forceinline__ bool row_live(const CasCtx& q, int id) {
  if (id < q.D0) return true;
  if (id < q.F0) return id - q.D0 > q.N;
  if (id < q.B0) return true;
  const int k = (id - q.B0) / 6;
  return q.cc[k] != 0.0;
}

// every row that can touch variable v, with its coefficient
template <typename F>
__device__ __forceinline__ void var_rows(const CasCtx& q, int v, F&& visit) {
  const int N = q.N;
  if (v < 12 * N) {
    const int k = v / 12, j = v - 12 * k;
    if (k >= 1) visit(12 * (k - 1) + j, 1.0);
    if (k <= N - 2) {
      visit(12 * k + j, -1.0);
      if (j >= 6 && j < 9) visit(12 * k + j - 6, -q.t);
      if (j >= 9) {
#pragma unroll
        for (int a = 0; a < 3; ++a) visit(12 * k + 3 + a, -q.t * q.rz[3 * a + j - 9]);
      }
    }
    if (k == 0 && j > N) visit(q.D0 + j, 1.0);
  } else {
    const int w = v - 12 * N, k = w / 6, c = w - 6 * k;
    if (k <= N - 2) {
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        const double b = q.Bd[6 * i + c];
        if (b != 0.0) visit(12 * k + i, -b);
      }
    }
    if (c == 0) { visit(q.F0 + 2 * k, 1.0); visit(q.F0 + 2 * k + 1, -1.0); }
    if (c == 2) { visit(q.F0 + 2 * k, -q.mu); visit(q.F0 + 2 * k + 1, -q.mu); }
    if (k == N - 1 && c == 1) { visit(q.F0 + 2 * N, 1.0); visit(q.F0 + 2 * N + 1, -1.0); }
    if (k == N - 1 && c == 2) { visit(q.F0 + 2 * N, -q.mu); visit(q.F0 + 2 * N + 1, -q.mu); }
    if (c < 3) { visit(q.B0 + 6 * k + 2 * c, 1.0); visit(q.B0 + 6 * k + 2 * c + 1, -1.0); }
  }
}

template <int ENT>
__device__ __forceinline__ double vget(const double (&v)[ENT], int i) {
  double r = v[0];
#pragma unroll
  for (int e = 1; e < ENT; ++e) r = ((i >> 6) == e) ? v[e] : r;
  return rdlane(r, i & 63);
}
template <int ENT>
__device__ __forceinline__ void vset(double (&v)[ENT], int i, double x) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int e = 0; e < ENT; ++e) v[e] = (64 * e + lane == i) ? x : v[e];
}

__device__ void cas_solve(const SolveArgs& a, int N, int64_t b, double* sm, double* Rm) {
  const CasLay L(N);
  int lane;
  asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"((int)threadIdx.x));
  const int NV = 18 * N, M = 20 * N + 2;
  const double t = a.dt, m = a.m, g = a.g;
  double* xin = sm + L.XIN;
  double* xr = sm + L.XR;
  double* cc = sm + L.CC;
  double* Bd = sm + L.BD;
  double* rz = sm + L.RZ;
  double* vv = sm + L.V;
  double* sv = sm + L.S;
  double* nb = sm + L.NB;
  double* zv = sm + L.Z;
  double* hi = sm + L.HI;
  double* rn = sm + L.RN;
  int* pos = reinterpret_cast<int*>(sm + L.POS);
  int* act = reinterpret_cast<int*>(sm + L.ACT);
  double* ua = sm + L.UA;
  double* cbv = sm + L.CB;
  double* sdg = sm + L.SD;

  // ---- loads, discretisation (lane 0: a 12x6 product, once per instance) ----
  const double* xrf = a.x_ref + b * a.xref_bs;
  if (lane < 12) xin[lane] = a.x_in[b * 12 + lane];
  for (int i = lane; i < 12 * N; i += RT) {
    const int r = i / 12, c = i - 12 * r;
    xr[i] = xrf[(int64_t)r * a.xref_rs + c];
  }
  for (int k = lane; k < N; k += RT) cc[k] = a.C[b * a.C_bs + k];
  const double mu = a.mu ? a.mu[b] : a.mu_default;
  wsync();
  double* Gd = sm + L.GD;
  {
    const double psi = xin[5];
    double sp, cp;
    sincos(psi, &sp, &cp);
    const double R[3][3] = {{cp, sp, 0.0}, {-sp, cp, 0.0}, {0.0, 0.0, 1.0}};   // rz (src/utils.py:46-51)
    // J_w^-1 = rz Jinv rz' (:38); B[9:12, 0:3] = Jw hat(rh + rf), B[9:12, 3:6] = Jw rz' (:39-43)
    double T[3][3], Jw[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        T[i][j] = R[i][0] * a.Jinv[j] + R[i][1] * a.Jinv[3 + j] + R[i][2] * a.Jinv[6 + j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Jw[i][j] = T[i][0] * R[j][0] + T[i][1] * R[j][1] + T[i][2] * R[j][2];
    const double w[3] = {a.rh[0], a.rh[1], a.rh[2] - 0.2};
    const double hw[3][3] = {{0.0, -w[2], w[1]}, {w[2], 0.0, -w[0]}, {-w[1], w[0], 0.0}};
    double B[12][6];
#pragma unroll
    for (int i = 0; i < 12; ++i)
#pragma unroll
      for (int c = 0; c < 6; ++c) B[i][c] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) B[6 + i][i] = 1.0 / m;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        B[9 + i][j] = Jw[i][0] * hw[0][j] + Jw[i][1] * hw[1][j] + Jw[i][2] * hw[2][j];
        B[9 + i][3 + j] = Jw[i][0] * R[j][0] + Jw[i][1] * R[j][1] + Jw[i][2] * R[j][2];
      }
    // Bd = B t + (t^2/2 A) B: A[0:3, 6:9] = I, A[3:6, 9:12] = rz (:26,37,47-49)
    const double h2 = 0.5 * (t * t);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 12; ++i)
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double acc = 0.0;
          if (i < 3) acc = h2 * B[6 + i][c];
          else if (i < 6)
            acc = (h2 * R[i - 3][0]) * B[9][c] + (h2 * R[i - 3][1]) * B[10][c] + (h2 * R[i - 3][2]) * B[11][c];
          Bd[6 * i + c] = B[i][c] * t + acc;
        }
#pragma unroll
      for (int e = 0; e < 9; ++e) rz[e] = R[e / 3][e % 3];
    }
    if (lane < 12) Gd[lane] = lane == 2 ? h2 * -g : (lane == 8 ? -g * t : 0.0);   // (t^2/2 A G)[2], G t (:50)
  }
  wsync();
  CasCtx q{N, NV, M, 12 * (N - 1), 12 * (N - 1) + 12, 12 * (N - 1) + 12 + 2 * N + 2, t, mu, Bd, rz, xin, cc};

  // ---- unconstrained optimum, H^-1 (fixed: x_0[i <= N], swing forces) ----
  const double ur = 2.0 * m * g;
  for (int v = lane; v < NV; v += RT) {
    double x0, h;
    if (v < 12 * N) {
      const int k = v / 12, j = v - 12 * k;
      const bool fixed = k == 0 && j <= N;
      x0 = fixed ? xin[j] : xr[v];
      h = fixed ? 0.0 : 0.5;
    } else {
      const int w = v - 12 * N, k = w / 6, c = w - 6 * k;
      const bool fixed = c < 3 && cc[k] == 0.0;
      x0 = fixed ? 0.0 : ur;
      h = fixed ? 0.0 : 50.0;
    }
    vv[v] = x0;
    hi[v] = h;
  }
  for (int id = lane; id < M; id += RT) {
    double s2 = 0.0;
    row_terms(q, id, [&](int, double c) { s2 = fma(c, c, s2); });
    rn[id] = sqrt(s2);
    pos[id] = -1;
  }
  wsync();

  // ---- dual active set ----
  auto rdot = [&](int id, const double* X) -> double {
    double s = 0.0;
    row_terms(q, id, [&](int v, double c) { s = fma(c, X[v], s); });
    return s;
  };
  int status = ST_SOLVED, iters = 0, qn = 0;
  const int max_iter = 4 * NV + 50;
  bool done = false;
  while (!done) {
    // most violated live, inactive row (scaled slack b - n'v < 0)
    double best = INFINITY;
    int bid = 0x7fffffff;
#pragma unroll
    for (int e = 0; e < ER; ++e) {
      const int id = 64 * e + lane;
      if (id < M && pos[id] < 0 && row_live(q, id) && rn[id] > 0.0)
        argmin_combine(best, bid, (row_rhs(q, id, Gd) - rdot(id, vv)) / rn[id], id);
    }
    wave_argmin(best, bid);
    if (!(best < -kCasTol)) break;
    const int p = uni(bid);
    const double bp = row_rhs(q, p, Gd);
    // GE form of p: n = -n_p, b = -b_p.  s = H^-1 n (sparse)
    for (int v = lane; v < NV; v += RT) sv[v] = 0.0;
    wsync();
    if (lane == 0) row_terms(q, p, [&](int v, double c) { sv[v] = -c * hi[v]; });
    wsync();
    double snl = 0.0;
    if (lane == 0) row_terms(q, p, [&](int v, double c) { snl = fma(c * c, hi[v], snl); });
    const double sn = rdlane(snl, 0);
    double uplus = 0.0;
    while (true) {
      if (++iters > max_iter) { status = ST_MAXIT; done = true; break; }
      // c = N_A' s (GE normals), y = R^-T c, r = R^-1 y
      double yv[EV], rv[EV];
#pragma unroll
      for (int e = 0; e < EV; ++e) {
        const int ai = 64 * e + lane;
        yv[e] = ai < qn ? -rdot(act[ai], sv) : 0.0;
      }
      for (int l = 0; l < qn; ++l) {
        const double yl = vget(yv, l) / Rm[loff(l) + l];
        vset(yv, l, yl);
#pragma unroll
        for (int e = 0; e < EV; ++e) {
          const int mm = 64 * e + lane;
          if (mm > l && mm < qn) yv[e] = fma(-Rm[loff(mm) + l], yl, yv[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < EV; ++e) rv[e] = yv[e];
      for (int l = qn - 1; l >= 0; --l) {
        const double rl = vget(rv, l) / Rm[loff(l) + l];
        vset(rv, l, rl);
#pragma unroll
        for (int e = 0; e < EV; ++e) {
          const int mm = 64 * e + lane;
          if (mm < l) rv[e] = fma(-Rm[loff(l) + mm], rl, rv[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < EV; ++e) {
        const int ai = 64 * e + lane;
        if (ai < qn) cbv[ai] = rv[e];
      }
      gsync();
      // nb = n_p - N_A r (GE), z = H^-1 nb, zn = nb' H^-1 nb
      double znl = 0.0;
      for (int v = lane; v < NV; v += RT) {
        double acc = 0.0;
        var_rows(q, v, [&](int id, double c) {
          if (id == p) acc -= c;
          const int ap = pos[id];
          if (ap >= 0) acc = fma(cbv[ap], c, acc);   // - r_a * (GE coef = -c)
        });
        nb[v] = acc;
        zv[v] = hi[v] * acc;
        znl = fma(acc * hi[v], acc, znl);
      }
      const double zn = wave_sum(znl);
      wsync();
      // step lengths
      double t1 = INFINITY;
      int kdrop = 0x7fffffff;
#pragma unroll
      for (int e = 0; e < EV; ++e) {
        const int ai = 64 * e + lane;
        if (ai < qn && rv[e] > 0.0) argmin_combine(t1, kdrop, ua[ai] / rv[e], ai);
      }
      wave_argmin(t1, kdrop);
      const double sp_ = -rdot(p, vv) + bp;   // GE slack of p (negative: violated)
      const bool has_z = zn > 1e-12 * sn;
      const double t2 = has_z ? -sp_ / zn : INFINITY;
      const double ts = t1 < t2 ? t1 : t2;
      if (!(ts < INFINITY)) { status = ST_INFEAS; done = true; break; }
      if (has_z)
        for (int v = lane; v < NV; v += RT) vv[v] = fma(ts, zv[v], vv[v]);
#pragma unroll
      for (int e = 0; e < EV; ++e) {
        const int ai = 64 * e + lane;
        if (ai < qn) ua[ai] = fma(-ts, rv[e], ua[ai]);
      }
      uplus += ts;
      gsync();
      if (has_z && ts == t2) {   // add p: R column [y; sqrt(zn)]
#pragma unroll
        for (int e = 0; e < EV; ++e) {
          const int ai = 64 * e + lane;
          if (ai < qn) Rm[loff(qn) + ai] = yv[e];
        }
        if (lane == 0) {
          Rm[loff(qn) + qn] = sqrt(zn);
          act[qn] = p;
          ua[qn] = uplus;
          pos[p] = qn;
        }
        ++qn;
        gsync();
        break;
      }
      // drop kdrop: delete its R column, restore the triangle by Givens
      {
        const int k = uni(kdrop);
        const int idk = act[k];
        for (int mm = k; mm + 1 < qn; ++mm) {
          for (int i0 = 0; i0 <= mm + 1; i0 += RT) {
            const int i = i0 + lane;
            const double val = i <= mm + 1 ? Rm[loff(mm + 1) + i] : 0.0;
            gsync();
            if (i <= mm) Rm[loff(mm) + i] = val;
            if (i == mm + 1) sdg[mm] = val;
            gsync();
          }
        }
        for (int i0 = k; i0 + 1 < qn; i0 += RT) {
          const int i = i0 + lane;
          int an = 0;
          double un = 0.0;
          if (i + 1 < qn) { an = act[i + 1]; un = ua[i + 1]; }
          gsync();
          if (i + 1 < qn) { act[i] = an; ua[i] = un; pos[an] = i; }
          gsync();
        }
        if (lane == 0) pos[idk] = -1;
        for (int l = k; l + 1 < qn; ++l) {
          const double aa = Rm[loff(l) + l], bb = sdg[l];
          const double hh = sqrt(aa * aa + bb * bb);
          const double cg = hh != 0.0 ? aa / hh : 1.0, sg = hh != 0.0 ? bb / hh : 0.0;
          gsync();
          if (lane == 0) Rm[loff(l) + l] = hh;
          for (int i0 = 0; i0 < qn; i0 += RT) {
            const int mcol = i0 + lane;
            if (mcol > l && mcol + 1 < qn) {
              const double rl = Rm[loff(mcol) + l], rl1 = Rm[loff(mcol) + l + 1];
              Rm[loff(mcol) + l] = cg * rl + sg * rl1;
              Rm[loff(mcol) + l + 1] = -sg * rl + cg * rl1;
            }
          }
          gsync();
        }
        --qn;
        gsync();
      }
    }
  }

  // ---- outputs: u*, x* (x_N on its dynamics bound), objective ----
  const int nx = 12 * N;
  for (int v = lane; v < 6 * N; v += RT) a.u[b * 6 * N + v] = vv[nx + v];
  double objl = 0.0;
  for (int v = lane; v < NV; v += RT) {
    const double d = v < nx ? vv[v] - xr[v] : vv[v] - ur;
    objl = fma(v < nx ? d : 0.01 * d, d, objl);
  }
  const double objv = wave_sum(objl);
  if (a.x) {
    double* xo = a.x + b * 12 * (N + 1);
    for (int v = lane; v < nx; v += RT) xo[v] = vv[v];
    if (lane < 12) {
      const int i = lane, k = N - 1;
      double xn = vv[12 * k + i] + Gd[i];
      if (i < 3) xn = fma(t, vv[12 * k + 6 + i], xn);
      else if (i < 6)
        for (int j = 0; j < 3; ++j) xn = fma(t * rz[3 * (i - 3) + j], vv[12 * k + 9 + j], xn);
      for (int c = 0; c < 6; ++c) xn = fma(Bd[6 * i + c], vv[nx + 6 * k + c], xn);
      xo[12 * N + i] = xn;
    }
  }
  if (lane == 0) {
    if (a.obj) a.obj[b] = objv;
    a.status[b] = status;
    if (a.iters) a.iters[b] = iters;
      if (a.active) a.active[b] = qn;
  }
}

__global__ void __launch_bounds__(RT) cas_kernel(SolveArgs a, int N) {
  extern __shared__ __attribute__((aligned(16))) double cas_sm[];
  double* Rm = a.kws + (int64_t)blockIdx.x * a.kws_stride;
  while (true) {
    int b = 0;
    if (threadIdx.x == 0) b = atomicAdd(a.work, 1);
    b = __builtin_amdgcn_readfirstlane(b);
    if (b >= a.B) break;
    cas_solve(a, N, (int64_t)b, cas_sm, Rm);
    __syncthreads();
  }
}

}  // namespace

size_t cas_lds_bytes(int N) { return (size_t)CasLay(N).total * sizeof(double); }
int64_t cas_ws_stride(int N) {
  const int64_t nv = 18 * (int64_t)N;
  return ((nv * (nv + 1) / 2) + 15) & ~(int64_t)15;
}
int cas_groups(int N) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, cas_kernel, RT, cas_lds_bytes(N)) != hipSuccess ||
      per < 1)
    per = 1;
  return cus * per;
}
bool launch_solve_cas(int N, const SolveArgs& a, hipStream_t s) {
  if (N < 1 || N > kCasNmax) return false;
  if (a.B <= 0) return true;
  if (!a.work || !a.kws || a.ric_groups < 1) return false;
  const unsigned g = (unsigned)(a.B < a.ric_groups ? a.B : a.ric_groups);
  hipLaunchKernelGGL(cas_kernel, dim3(g), dim3(RT), cas_lds_bytes(N), s, a, N);
  return true;
}

}  // namespace hmpc
