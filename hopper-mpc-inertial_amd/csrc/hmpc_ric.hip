// hmpc_ric.hip -- the per-timestep QP of Mpc.build_qp/solve_qp
// (src/mpc_cvx_euler_3f.py:96-160; 2f :96-158) for any horizon
// 1 <= N <= kRicNmax, the Runner's own N = 60 (src/robotrunner.py:46)
// included, without forming the condensed Hessian.
//
// One wavefront solves one instance.  The condensed Hessian over the inputs
// (states eliminated through the dynamics, NV = 6N variables),
//     H = 2 (Gamma' W Gamma + V),
// is never built: a backward Riccati recursion over the stages factors it as
// H = M'M with (M u)_k = D_k'(u_k + K_k x_k), x the state response to u
// (x_0 = 0), G_k = D_k D_k' = 2V_k + B_k'P_{k+1}B_k, K_k = G_k^-1 B_k'P_{k+1}A_k,
// P_k = 2Q + A_k'P_{k+1}A_k - F_k'K_k (P_N = 2*100 Q) -- O(N nx^3) instead of
// the dense O((6N)^3).  H^-1 n is then two sweeps over the stages:
//     backward  mu_j = n_j - B_j'lam_{j+1},  lam_j = A_j'lam_{j+1} + K_j'mu_j
//     per stage w_j = G_j^-1 mu_j
//     forward   u_k = w_k - K_k x_k,          x_{k+1} = A_k x_k + B_k u_k
// (lanes 0..11 hold the 12 state/adjoint rows; every other per-stage step runs
// lane-per-stage).
//
// The dual active set is Goldfarb-Idnani in range-space form with the
// Cholesky R'R = N_A' H^-1 N_A of the active normals (no NV x q basis): one
// iteration for constraint p computes s = H^-1 n_p (once per p), c = N_A's,
// r = (R'R)^-1 c, z = H^-1 (n_p - N_A r) and steps exactly as the classic
// method; an add appends [R^-T c; sqrt(n_z'z)] to R, a drop re-triangularises
// R by Givens rotations.  Constraints (one id = 4 v + slot per variable v):
// torque box (:123-128), fz box + friction pyramid (:141-146), z >= 0.1 (:129:
// z_k = free response + sum_{j<=k-2} dt (dt/m)(k-1-j) fz_j); swing and 2f fy
// equalities (:134-136, 2f :129) are fixed variables (zero columns of B_k).
//
// R lives in LDS with a capacity ric_qcap(N); an instance whose active set
// outgrows it is handed to the overflow pass (capacity 6N, R in global
// memory) instead of failing.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "hmpc_internal.h"
#include "hmpc_model.h"

namespace hmpc {

namespace {

constexpr int RT = 64;   // one wavefront per workgroup

// LDS layout (in doubles) for a runtime horizon N and active-set capacity cap
// (R in LDS only when r_lds).
struct RicLay {
  int XIN, CC, CS, BW, ZB, ZN, ZD, MISC, VV, SV, ZV, NB, MU, KM, GI, UA, ACT, CB, GV, SD, RM, U0, total;
  __host__ __device__ RicLay(int N, int cap, bool r_lds) {
    const int NV = 6 * N;
    auto up2 = [](int x) { return (x + 1) & ~1; };   // 16-B alignment of every array
    int o = 0;
    XIN = o; o += 12;
    CC = o; o = up2(o + N);
    CS = o; o += 2 * N;
    BW = o; o += 18 * N;
    ZB = o; o = up2(o + N + 1);   // free-response heights z_k, k = 0..N
    ZN = o; o = up2(o + N);       // |n| of the z row of stage k
    ZD = o; o = up2(o + N);       // z-row dots of s = H^-1 n_p
    MISC = o; o += 8;
    VV = o; o += NV;              // primal iterate
    SV = o; o += NV;              // s = H^-1 n_p
    ZV = o; o += NV;              // z = H^-1 (n_p - N_A r)
    NB = o; o += NV;              // right-hand side of H^-1 (n_p, n_p - N_A r)
    MU = o; o += NV;              // sweep scratch (mu, then G^-1 mu)
    KM = o; o += 72 * N;          // K_k [6][12]
    GI = o; o = up2(o + 21 * N);  // G_k^-1, packed lower triangle
    UA = o; o = up2(o + cap);     // active multipliers
    ACT = o; o = up2(o + cap);    // active ids (int)
    CB = o; o = up2(o + cap);     // scratch
    GV = o; o += 2 * up2(cap);    // Givens of a drop
    SD = o; o = up2(o + cap);     // subdiagonal scratch
    U0 = o;                       // union: x_ref (12N) | Riccati scratch (468)
    o += (12 * N > 468 ? 12 * N : 468);
    RM = o; if (r_lds) o = up2(o + cap * (cap + 1) / 2);   // packed upper R
    total = o;
  }
};

// Riccati scratch inside the union
constexpr int PS_OFF = 0, M1_OFF = 144, TS_OFF = 288, FS_OFF = 360, GS_OFF = 432;

__device__ __forceinline__ int loff(int r) { return (r * (r + 1)) >> 1; }

__device__ __forceinline__ void wsync() { __syncthreads(); }

// inclusive prefix sum over the wave (lane order)
__device__ __forceinline__ double wave_scan(double x) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

// entry i (uniform) of a lane-distributed vector (entry i in lane i % 64,
// register i / 64)
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

template <int VAR, int ENT>
__device__ void ric_solve(const SolveArgs& a, const int N, const int64_t b, double* sm, double* Rm,
                          const int cap) {
  const RicLay L(N, cap, false);
  const int lane = threadIdx.x;
  const int NV = 6 * N;
  const double dt = a.dt, dtm = dt / a.m;
  const double zc = dt * dtm;   // coefficient scale of fz_j in z_k
  double* xin = sm + L.XIN;
  double* cc = sm + L.CC;
  double* cs = sm + L.CS;
  double* bw = sm + L.BW;
  double* zb = sm + L.ZB;
  double* znrm = sm + L.ZN;
  double* zd = sm + L.ZD;
  double* vv = sm + L.VV;
  double* sv = sm + L.SV;
  double* zv = sm + L.ZV;
  double* nb = sm + L.NB;
  double* mu_ = sm + L.MU;
  double* km = sm + L.KM;
  double* gi = sm + L.GI;
  double* ua = sm + L.UA;
  int* act = reinterpret_cast<int*>(sm + L.ACT);
  double* gv = sm + L.GV;
  double* sdg = sm + L.SD;
  double* un = sm + L.U0;

  // ---------------- phase 0: loads + gen_dt_dynamics (lane k < N) ----------
  // x_ref / pf / C may be strided views of a resident plan (path_plan_grab,
  // src/robotrunner.py:228-230); x_lin rows per shift_mode (3f :50-62)
  const double* xrf = a.x_ref + b * a.xref_bs;
  const double mu = a.mu ? a.mu[b] : a.mu_default;
  if (lane < 12) xin[lane] = a.x_in[b * 12 + lane];
  for (int i = lane; i < 12 * N; i += RT) {
    const int r = i / 12, c = i - 12 * r;
    un[i] = xrf[(int64_t)r * a.xref_rs + c];
  }
  for (int k = lane; k < N; k += RT) {
    cc[k] = a.C[b * a.C_bs + k];
    const double* row;
    if (k == 0 && a.shift_mode != 0) row = a.x_in + b * 12;
    else if (a.shift_mode == 1) row = xrf + (int64_t)(k - 1) * a.xref_rs;
    else if (a.shift_mode == 2) row = a.x_lin + b * 12 * (N + 1) + 12 * (k + 1);
    else row = a.x_lin + b * 12 * (N + 1) + 12 * k;
    const double p[3] = {row[0], row[1], row[2]};
    const double* pfr = a.pf + b * a.pf_bs + (int64_t)k * a.pf_rs;
    const double pfk[3] = {pfr[0], pfr[1], pfr[2]};
    stage_dynamics_vals<VAR, double>(k, row[5], p, pfk, a.Jinv, a.rh, dt, cs, bw);
  }
  wsync();

  // ---------------- phase 1: free response, d_t, adjoint, gradient ----------
  // lane r < 12 holds component r.  d_t = kf Q (xbar_t - r_{t-1}) overwrites
  // x_ref row t-1; the gradient h = 2 Gamma' W (xbar - r) - 2 V ubar goes to
  // NB as -h (the right-hand side of the unconstrained optimum).
  {
    double xr = lane < 12 ? xin[lane] : 0.0;
    const double qr = qdiag(lane);
    if (lane == 2) zb[0] = xr;
    for (int k = 0; k < N; ++k) {
      xr = ad_lane(xr, dt, cs[2 * k], cs[2 * k + 1]) + ((lane == 8) ? -a.g * dt : 0.0);
      const double kf = (k == N - 1) ? kTermQ : 1.0;
      if (lane < 12) un[12 * k + lane] = kf * qr * (xr - un[12 * k + lane]);
      if (lane == 2) zb[k + 1] = xr;
    }
    wsync();
    const double ubar_alias = (cc[N - 1] != 0.0) ? 2.0 * a.m * a.g : 0.0;
    double ar = lane < 12 ? un[12 * (N - 1) + lane] : 0.0;   // a_N = d_N
    for (int t = N; t >= 1; --t) {
      const int i = t - 1;
      const double a6 = rdlane(ar, 6), a7 = rdlane(ar, 7), a8 = rdlane(ar, 8);
      const double a9 = rdlane(ar, 9), a10 = rdlane(ar, 10), a11 = rdlane(ar, 11);
      if (lane < 6) {
        const int c = lane;
        const double cp = cs[2 * i], sp = cs[2 * i + 1];
        const double* bwi = bw + 18 * i;
        double acc = bwi[c] * a9 + bwi[6 + c] * a10 + bwi[12 + c] * a11;
        if (c < 3)
          acc += bv<VAR>(0, c, dtm, cp, sp) * a6 + bv<VAR>(1, c, dtm, cp, sp) * a7 +
                 bv<VAR>(2, c, dtm, cp, sp) * a8;
        const bool stance = cc[i] != 0.0;
        const bool fr = c >= 3 || (stance && !(VAR == 2 && c == 1));
        double h = fr ? 2.0 * acc : 0.0;
        if (fr && c == 2 && i < N - 1) {
          const double ub = a.uref_aliased ? ubar_alias : (stance ? 2.0 * a.m * a.g : 0.0);
          h -= 2.0 * kRdiag * ub;
        }
        nb[6 * i + c] = -h;
      }
      if (t >= 2) {
        ar = adt_lane(ar, dt, cs[2 * i], cs[2 * i + 1]) + (lane < 12 ? un[12 * (t - 2) + lane] : 0.0);
      }
    }
  }
  wsync();

  // ---------------- phase 2: Riccati factorisation -------------------------
  int status = ST_SOLVED;
  {
    double* P = un + PS_OFF;    // P_{k+1}, 12 x 12 full
    double* M1 = un + M1_OFF;   // P A
    double* T = un + TS_OFF;    // P B, 12 x 6
    double* F = un + FS_OFF;    // B'P A, 6 x 12
    double* G = un + GS_OFF;    // 6 x 6
    for (int e = lane; e < 144; e += RT) {
      const int i = e / 12, j = e - 12 * i;
      P[e] = (i == j) ? 2.0 * kTermQ * kQ[i] : 0.0;
    }
    wsync();
    double nbad = 0.0;
    for (int k = N - 1; k >= 0; --k) {
      const double cp = cs[2 * k], sp = cs[2 * k + 1];
      const bool stance = cc[k] != 0.0;
      const double* bwk = bw + 18 * k;
      // B[r][c] (rows 6..11), zero columns for fixed variables
      auto bent = [&](int r, int c) -> double {
        const bool fr = c >= 3 || (stance && !(VAR == 2 && c == 1));
        if (!fr) return 0.0;
        if (r < 9) return c < 3 ? bv<VAR>(r - 6, c, dtm, cp, sp) : 0.0;
        return bwk[6 * (r - 9) + c];
      };
      // (a) T = P B
      for (int e = lane; e < 72; e += RT) {
        const int i = e / 6, c = e - 6 * i;
        double acc = 0.0;
#pragma unroll
        for (int r = 6; r < 12; ++r) acc = fma(P[12 * i + r], bent(r, c), acc);
        T[e] = acc;
      }
      wsync();
      // (b) G = 2V + B'T (identity rows for fixed variables), F = T'A
      for (int e = lane; e < 108; e += RT) {
        if (e < 36) {
          const int c = e / 6, d = e - 6 * c;
          double acc = 0.0;
#pragma unroll
          for (int r = 6; r < 12; ++r) acc = fma(bent(r, c), T[6 * r + d], acc);
          const bool frc = c >= 3 || (stance && !(VAR == 2 && c == 1));
          if (c == d) acc = frc ? acc + ((k < N - 1) ? 2.0 * kRdiag : 0.0) : 1.0;
          G[e] = acc;
        } else {
          const int e2 = e - 36, c = e2 / 12, j = e2 - 12 * c;
          double f = T[6 * j + c];
          if (j >= 6 && j < 9) f = fma(dt, T[6 * (j - 6) + c], f);
          else if (j == 9) f += dt * (cp * T[18 + c] - sp * T[24 + c]);
          else if (j == 10) f += dt * (sp * T[18 + c] + cp * T[24 + c]);
          else if (j == 11) f = fma(dt, T[30 + c], f);
          F[e2] = f;
        }
      }
      wsync();
      // (c) G = D D' (every lane, redundantly), Dinv; G^-1 = Dinv'Dinv packed
      // (lanes e < 21); K = Dinv'(Dinv F) (lanes j < 12, one column each)
      double D[21], Di[21];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
#pragma unroll
        for (int d = 0; d <= c; ++d) {
          double s = G[6 * c + d];
#pragma unroll
          for (int m = 0; m < d; ++m) s = fma(-D[loff(c) + m], D[loff(d) + m], s);
          if (d == c) {
            nbad += (s > 0.0) ? 0.0 : 1.0;
            D[loff(c) + c] = sqrt(s > 0.0 ? s : 1.0);
          } else {
            D[loff(c) + d] = s / D[loff(d) + d];
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) {   // column c of Dinv: forward substitution of e_c
        Di[loff(c) + c] = 1.0 / D[loff(c) + c];
#pragma unroll
        for (int r = c + 1; r < 6; ++r) {
          double s = 0.0;
#pragma unroll
          for (int m = c; m < r; ++m) s = fma(D[loff(r) + m], Di[loff(m) + c], s);
          Di[loff(r) + c] = -s / D[loff(r) + r];
        }
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) {
#pragma unroll
        for (int d = 0; d <= c; ++d) {
          double s = 0.0;
#pragma unroll
          for (int m = c; m < 6; ++m) s = fma(Di[loff(m) + c], Di[loff(m) + d], s);
          if (lane == 0) gi[21 * k + loff(c) + d] = s;
        }
      }
      if (lane < 12) {
        const int j = lane;
        double y[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double s = 0.0;
#pragma unroll
          for (int m = 0; m <= c; ++m) s = fma(Di[loff(c) + m], F[12 * m + j], s);
          y[c] = s;
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double s = 0.0;
#pragma unroll
          for (int m = c; m < 6; ++m) s = fma(Di[loff(m) + c], y[m], s);
          km[72 * k + 12 * c + j] = s;
        }
      }
      wsync();
      if (k == 0) break;
      // (d) P_k = 2Q + A'(P A) - F'K, lower triangle computed, mirrored
      for (int e = lane; e < 144; e += RT) {
        const int i = e / 12, j = e - 12 * i;
        double m1 = P[e];
        if (j >= 6 && j < 9) m1 = fma(dt, P[12 * i + j - 6], m1);
        else if (j == 9) m1 += dt * (cp * P[12 * i + 3] - sp * P[12 * i + 4]);
        else if (j == 10) m1 += dt * (sp * P[12 * i + 3] + cp * P[12 * i + 4]);
        else if (j == 11) m1 = fma(dt, P[12 * i + 5], m1);
        M1[e] = m1;
      }
      wsync();
      for (int e = lane; e < 78; e += RT) {
        int i = 0;
        while (loff(i + 1) <= e) ++i;
        const int j = e - loff(i);
        double pn = M1[12 * i + j];
        if (i >= 6 && i < 9) pn = fma(dt, M1[12 * (i - 6) + j], pn);
        else if (i == 9) pn += dt * (cp * M1[36 + j] - sp * M1[48 + j]);
        else if (i == 10) pn += dt * (sp * M1[36 + j] + cp * M1[48 + j]);
        else if (i == 11) pn = fma(dt, M1[60 + j], pn);
#pragma unroll
        for (int c = 0; c < 6; ++c) pn = fma(-F[12 * c + i], km[72 * k + 12 * c + j], pn);
        if (i == j) pn += 2.0 * kQ[i];
        P[12 * i + j] = pn;
        P[12 * j + i] = pn;
      }
      wsync();
    }
    if (nbad != 0.0) status = ST_NUMERICAL;
  }

  // ---------------- H^-1 by two sweeps ----------------------------------------
  // dst = H^-1 NB (NB kept; MU scratch)
  auto hinv = [&](double* dst) __attribute__((always_inline)) {
    double lam = 0.0;
    for (int j = N - 1; j >= 0; --j) {
      const double cp = cs[2 * j], sp = cs[2 * j + 1];
      const bool stance = cc[j] != 0.0;
      const double l6 = rdlane(lam, 6), l7 = rdlane(lam, 7), l8 = rdlane(lam, 8);
      const double l9 = rdlane(lam, 9), l10 = rdlane(lam, 10), l11 = rdlane(lam, 11);
      double m = 0.0;
      if (lane < 6) {
        const int c = lane;
        const double* bwj = bw + 18 * j;
        double bc = bwj[c] * l9 + bwj[6 + c] * l10 + bwj[12 + c] * l11;
        if (c < 3)
          bc += bv<VAR>(0, c, dtm, cp, sp) * l6 + bv<VAR>(1, c, dtm, cp, sp) * l7 +
                bv<VAR>(2, c, dtm, cp, sp) * l8;
        const bool fr = c >= 3 || (stance && !(VAR == 2 && c == 1));
        m = nb[6 * j + c] - (fr ? bc : 0.0);
        mu_[6 * j + c] = m;
      }
      if (j == 0) break;
      const double m0 = rdlane(m, 0), m1 = rdlane(m, 1), m2 = rdlane(m, 2);
      const double m3 = rdlane(m, 3), m4 = rdlane(m, 4), m5 = rdlane(m, 5);
      double nl = adt_lane(lam, dt, cp, sp);
      if (lane < 12) {
        const double* kj = km + 72 * j + lane;
        nl += ((kj[0] * m0 + kj[12] * m1) + (kj[24] * m2 + kj[36] * m3)) + (kj[48] * m4 + kj[60] * m5);
      }
      lam = lane < 12 ? nl : 0.0;
    }
    wsync();
    for (int j = lane; j < N; j += RT) {
      double mv[6], w[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) mv[c] = mu_[6 * j + c];
      const double* g = gi + 21 * j;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        double s = 0.0;
#pragma unroll
        for (int d = 0; d < 6; ++d) s = fma(g[c >= d ? loff(c) + d : loff(d) + c], mv[d], s);
        w[c] = s;
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) mu_[6 * j + c] = w[c];
    }
    wsync();
    double x = 0.0;
    for (int k = 0; k < N; ++k) {
      const double cp = cs[2 * k], sp = cs[2 * k + 1];
      double xs[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) xs[i] = rdlane(x, i);
      double u = 0.0;
      if (lane < 6) {
        const double* kr = km + 72 * k + 12 * lane;
        double a0 = mu_[6 * k + lane], a1 = 0.0;
#pragma unroll
        for (int c = 0; c < 12; c += 2) {
          a0 = fma(-kr[c], xs[c], a0);
          a1 = fma(-kr[c + 1], xs[c + 1], a1);
        }
        u = a0 + a1;
        dst[6 * k + lane] = u;
      }
      const double u0 = rdlane(u, 0), u1 = rdlane(u, 1), u2 = rdlane(u, 2);
      const double u3 = rdlane(u, 3), u4 = rdlane(u, 4), u5 = rdlane(u, 5);
      double nx = ad_lane(x, dt, cp, sp);
      if (lane >= 6 && lane < 9) {
        const int r = lane - 6;
        nx += bv<VAR>(r, 0, dtm, cp, sp) * u0 + bv<VAR>(r, 1, dtm, cp, sp) * u1 +
              bv<VAR>(r, 2, dtm, cp, sp) * u2;
      } else if (lane >= 9 && lane < 12) {
        const double* bwr = bw + 18 * k + 6 * (lane - 9);
        nx += ((bwr[0] * u0 + bwr[1] * u1) + (bwr[2] * u2 + bwr[3] * u3)) + (bwr[4] * u4 + bwr[5] * u5);
      }
      x = lane < 12 ? nx : 0.0;
    }
    wsync();
  };
  // sum over all NV entries of X .* Y (lane-per-stage), wave-uniform
  auto vdot = [&](const double* X, const double* Y) -> double {
    double s = 0.0;
    for (int j = lane; j < N; j += RT) {
#pragma unroll
      for (int c = 0; c < 6; ++c) s = fma(X[6 * j + c], Y[6 * j + c], s);
    }
    return wave_sum(s);
  };
  // lane k: sum_{j <= k-2} zc (k-1-j) C_j X[fz_j] (the z-row of stage k over X)
  auto zdot = [&](const double* X) -> double {
    const double aj = (lane < N && cc[lane] != 0.0) ? X[6 * lane + 2] : 0.0;
    const double s1 = wave_scan(aj), s2 = wave_scan(aj * (double)lane);
    const double t1 = __shfl_up(s1, 2), t2 = __shfl_up(s2, 2);
    return lane >= 2 ? zc * ((double)(lane - 1) * t1 - t2) : 0.0;
  };

  // ---------------- phase 3: unconstrained optimum v0 = -H^-1 h --------------
  hinv(vv);
  // |n| of the z rows (lane k): zc sqrt(sum_{j <= k-2, stance} (k-1-j)^2)
  if (lane < N) {
    double s2 = 0.0;
    for (int j = 0; j + 2 <= lane; ++j) {
      const double cz = (double)(lane - 1 - j);
      if (cc[j] != 0.0) s2 = fma(cz, cz, s2);
    }
    znrm[lane] = zc * sqrt(s2);
  }
  wsync();

  // ---------------- phase 4: dual active set --------------------------------
  int iters = 0;
  if (xin[2] - kZmin < -kTol || zb[1] - kZmin < -kTol) status = ST_INFEAS;   // constant rows z_0, z_1
  const int max_iter = 4 * NV + 50;
  const bool stance_me = lane < N && cc[lane] != 0.0;
  const double inv01 = 1.0 / sqrt(1.0 + mu * mu);
  int amask = 0;   // active (c, slot) bits 4c + slot of my stage
  int q = 0;
  // coefficient of constraint id on the 6 entries of stage j (acc += s * n)
  auto add_coef = [&](int id, int j, double s, double (&acc)[6]) __attribute__((always_inline)) {
    const int v = id >> 2, sl = id & 3, k = v / 6, c = v - 6 * k;
    double e[6] = {0, 0, 0, 0, 0, 0};
    if (c >= 3) {
      if (sl < 2) {
        if (j == k) {
#pragma unroll
          for (int t = 3; t < 6; ++t) e[t] = (t == c) ? (sl == 0 ? 1.0 : -1.0) : 0.0;
        }
      } else if (j <= k - 2 && cc[j] != 0.0) {
        e[2] = zc * (double)(k - 1 - j);
      }
    } else if (c == 2) {
      if (j == k) e[2] = sl == 0 ? 1.0 : -1.0;
    } else if (j == k) {
      e[0] = (c == 0) ? (sl == 0 ? -1.0 : 1.0) : 0.0;
      e[1] = (c == 1) ? (sl == 0 ? -1.0 : 1.0) : 0.0;
      e[2] = mu;
    }
#pragma unroll
    for (int t = 0; t < 6; ++t) acc[t] = fma(s, e[t], acc[t]);
  };
  auto rhs_of = [&](int id) -> double {
    const int v = id >> 2, sl = id & 3, k = v / 6, c = v - 6 * k;
    if (c >= 3) return sl < 2 ? -tau_lim(c) : kZmin - zb[k];
    if (c == 2) return sl == 0 ? 0.0 : -kFzMax;
    return 0.0;
  };
  // n_id' X for an id, given X and the z-row dots ZX of X in lane k (uniform
  // id; every lane returns the value)
  auto cdot = [&](int id, const double* X, double zx) -> double {
    const int v = id >> 2, sl = id & 3, k = v / 6, c = v - 6 * k;
    if (c >= 3) return sl < 2 ? (sl == 0 ? X[v] : -X[v]) : rdlane(zx, k);
    if (c == 2) return sl == 0 ? X[v] : -X[v];
    return (sl == 0 ? -X[v] : X[v]) + mu * X[6 * k + 2];
  };

  bool done = status != ST_SOLVED;
  while (!done) {
    // ---- slacks of my stage's constraints; the most violated ----
    const double vz = zdot(vv);
    double best = INFINITY;
    int bid = 0x7fffffff;
    if (lane < N) {
      const int k = lane;
      double u[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) u[c] = vv[6 * k + c];
#pragma unroll
      for (int c = 3; c < 6; ++c) {
        const double lim = tau_lim(c);
        const int v = 6 * k + c;
        if (!(amask & (1 << (4 * c)))) argmin_combine(best, bid, u[c] + lim, 4 * v);
        if (!(amask & (1 << (4 * c + 1)))) argmin_combine(best, bid, lim - u[c], 4 * v + 1);
      }
      if (k >= 2 && !(amask & (1 << 14))) {
        const double zrow = (zb[k] - kZmin) + vz;
        const double zn = znrm[k];
        const double s2 = zn > 0.0 ? zrow / zn : ((zrow < -kTol) ? -INFINITY : INFINITY);
        argmin_combine(best, bid, s2, 4 * (6 * k + 3) + 2);
      }
      if (stance_me) {
        const int v = 6 * k + 2;
        if (!(amask & (1 << 8))) argmin_combine(best, bid, u[2], 4 * v);
        if (!(amask & (1 << 9))) argmin_combine(best, bid, kFzMax - u[2], 4 * v + 1);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          if (VAR == 2 && c == 1) continue;
          const int vc = 6 * k + c;
          if (!(amask & (1 << (4 * c)))) argmin_combine(best, bid, (mu * u[2] - u[c]) * inv01, 4 * vc);
          if (!(amask & (1 << (4 * c + 1)))) argmin_combine(best, bid, (mu * u[2] + u[c]) * inv01, 4 * vc + 1);
        }
      }
    }
    wave_argmin(best, bid);
    if (!(best < -kTol)) break;   // primal feasible: optimal
    const int p = uni(bid);
    const double bp = rhs_of(p);
    // n_p -> NB
    for (int j = lane; j < N; j += RT) {
      double acc[6] = {0, 0, 0, 0, 0, 0};
      add_coef(p, j, 1.0, acc);
#pragma unroll
      for (int c = 0; c < 6; ++c) nb[6 * j + c] = acc[c];
    }
    wsync();
    hinv(sv);                     // s = H^-1 n_p
    const double sn = vdot(nb, sv);
    const double szd = zdot(sv);
    if (lane < N) zd[lane] = szd;
    wsync();
    double uplus = 0.0;
    // ---- inner loop: step towards satisfying constraint p ----
    while (true) {
      if (++iters > max_iter) { status = ST_MAXIT; done = true; break; }
      // c = N_A' s, y = R^-T c, r = R^-1 y  (entry a in lane a % 64)
      double yv[ENT], rv[ENT];
#pragma unroll
      for (int e = 0; e < ENT; ++e) {
        const int ai = 64 * e + lane;
        double cvl = 0.0;
        if (ai < q) {
          const int id = act[ai];
          const int v = id >> 2, sl = id & 3, k = v / 6, c = v - 6 * k;
          if (c >= 3) cvl = sl < 2 ? (sl == 0 ? sv[v] : -sv[v]) : zd[k];
          else if (c == 2) cvl = sl == 0 ? sv[v] : -sv[v];
          else cvl = (sl == 0 ? -sv[v] : sv[v]) + mu * sv[6 * k + 2];
        }
        yv[e] = cvl;
      }
      for (int l = 0; l < q; ++l) {   // forward substitution with R'
        const double yl = vget(yv, l) / Rm[loff(l) + l];
        vset(yv, l, yl);
#pragma unroll
        for (int e = 0; e < ENT; ++e) {
          const int m = 64 * e + lane;
          if (m > l && m < q) yv[e] = fma(-Rm[loff(m) + l], yl, yv[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < ENT; ++e) rv[e] = yv[e];
      for (int l = q - 1; l >= 0; --l) {   // back substitution with R
        const double rl = vget(rv, l) / Rm[loff(l) + l];
        vset(rv, l, rl);
#pragma unroll
        for (int e = 0; e < ENT; ++e) {
          const int m = 64 * e + lane;
          if (m < l) rv[e] = fma(-Rm[loff(l) + m], rl, rv[e]);
        }
      }
      // z = H^-1 (n_p - N_A r), n_z' z
      const double* zsrc = sv;
      double zn = sn;
      if (q > 0) {
        for (int j = lane; j < N; j += RT) {
          double acc[6] = {0, 0, 0, 0, 0, 0};
          add_coef(p, j, 1.0, acc);
          for (int ai = 0; ai < q; ++ai) add_coef(act[ai], j, -vget(rv, ai), acc);
#pragma unroll
          for (int c = 0; c < 6; ++c) nb[6 * j + c] = acc[c];
        }
        // (the vget above is wave-uniform: every lane runs the same trip count
        // when N <= 64)
        wsync();
        hinv(zv);
        zsrc = zv;
        zn = vdot(nb, zv);
      }
      // partial step t1 (drop candidate) over r > 0
      double t1 = INFINITY;
      int kdrop = 0x7fffffff;
#pragma unroll
      for (int e = 0; e < ENT; ++e) {
        const int ai = 64 * e + lane;
        if (ai < q && rv[e] > 0.0) argmin_combine(t1, kdrop, ua[ai] / rv[e], ai);
      }
      wave_argmin(t1, kdrop);
      // full step t2
      const double sp_ = cdot(p, vv, zdot(vv)) - bp;
      const bool has_z = zn > 1e-12 * sn;
      const double t2 = has_z ? -sp_ / zn : INFINITY;
      const double t = t1 < t2 ? t1 : t2;
      if (!(t < INFINITY)) { status = ST_INFEAS; done = true; break; }
      if (has_z)
        for (int i = lane; i < NV; i += RT) vv[i] = fma(t, zsrc[i], vv[i]);
#pragma unroll
      for (int e = 0; e < ENT; ++e) {
        const int ai = 64 * e + lane;
        if (ai < q) ua[ai] = fma(-t, rv[e], ua[ai]);
      }
      uplus += t;
      wsync();
      if (has_z && t == t2) {
        // ---- add p: R column [y; sqrt(n_z'z)] ----
        if (q >= cap) {
          status = a.ovf_count ? ST_OVERFLOW : ST_NUMERICAL;
          done = true;
          break;
        }
#pragma unroll
        for (int e = 0; e < ENT; ++e) {
          const int ai = 64 * e + lane;
          if (ai < q) Rm[loff(q) + ai] = yv[e];
        }
        if (lane == 0) {
          Rm[loff(q) + q] = sqrt(zn);
          act[q] = p;
          ua[q] = uplus;
        }
        if (lane == (p >> 2) / 6) amask |= 1 << (4 * ((p >> 2) % 6) + (p & 3));
        ++q;
        wsync();
        break;
      }
      // ---- drop kdrop: delete its column of R, restore the triangle ----
      {
        const int k = uni(kdrop);
        const int idk = act[k];
        if (lane == (idk >> 2) / 6) amask &= ~(1 << (4 * ((idk >> 2) % 6) + (idk & 3)));
        for (int m = k; m + 1 < q; ++m) {   // shift columns m+1 -> m, keep subdiagonals
          for (int i0 = 0; i0 <= m + 1; i0 += RT) {
            const int i = i0 + lane;
            const double val = i <= m + 1 ? Rm[loff(m + 1) + i] : 0.0;
            wsync();
            if (i <= m) Rm[loff(m) + i] = val;
            if (i == m + 1) sdg[m] = val;
            wsync();
          }
        }
        for (int i0 = k; i0 + 1 < q; i0 += RT) {   // shift the active list
          const int i = i0 + lane;
          int an = 0;
          double un_ = 0.0;
          if (i + 1 < q) { an = act[i + 1]; un_ = ua[i + 1]; }
          wsync();
          if (i + 1 < q) { act[i] = an; ua[i] = un_; }
          wsync();
        }
        for (int l = k; l + 1 < q; ++l) {   // Givens on rows (l, l+1)
          const double aa = Rm[loff(l) + l], bb = sdg[l];
          const double hh = sqrt(aa * aa + bb * bb);
          const double cg = hh != 0.0 ? aa / hh : 1.0, sg = hh != 0.0 ? bb / hh : 0.0;
          wsync();
          if (lane == 0) Rm[loff(l) + l] = hh;
          for (int i0 = 0; i0 < q; i0 += RT) {
            const int mcol = i0 + lane;   // columns m > l hold rows l, l+1
            if (mcol > l && mcol + 1 < q) {
              const double rl = Rm[loff(mcol) + l], rl1 = Rm[loff(mcol) + l + 1];
              Rm[loff(mcol) + l] = cg * rl + sg * rl1;
              Rm[loff(mcol) + l + 1] = -sg * rl + cg * rl1;
            }
          }
          wsync();
        }
        q = q - 1;
        wsync();
      }
    }
  }

  // ---------------- phase 5: outputs ---------------------------------------
  // overflowed instances are re-solved by the overflow pass: write nothing
  // but the status (x_prev may be this solve's input)
  if (status == ST_OVERFLOW) {
    if (lane == 0) {
      a.status[b] = ST_OVERFLOW;
      const int slot = atomicAdd(a.ovf_count, 1);
      a.ovf_list[slot] = (int32_t)b;
    }
    return;
  }
  // x_ref again (its LDS copy is gone) into the union, x* staged over SV..
  for (int i = lane; i < 12 * N; i += RT) {
    const int r = i / 12, c = i - 12 * r;
    un[i] = xrf[(int64_t)r * a.xref_rs + c];
  }
  for (int i = lane; i < NV; i += RT) {
    const int j = i / 6, c = i - 6 * j;
    const bool fr = c >= 3 || (cc[j] != 0.0 && !(VAR == 2 && c == 1));
    const double u = (status == ST_SOLVED && fr) ? vv[i] : 0.0;
    vv[i] = u;
    a.u[b * NV + i] = u;
  }
  wsync();
  double* xo = sv;   // 12 (N+1) <= 4 NV doubles (SV, ZV, NB, MU)
  {
    double xr = lane < 12 ? xin[lane] : 0.0;
    if (lane < 12) xo[lane] = xr;
    const double qr = qdiag(lane);
    const double ub_alias = (cc[N - 1] != 0.0) ? 2.0 * a.m * a.g : 0.0;
    double objl = 0.0;
    for (int k = 0; k < N; ++k) {
      const double cp = cs[2 * k], sp = cs[2 * k + 1];
      const double* uk = vv + 6 * k;
      const double u0 = uk[0], u1 = uk[1], u2 = uk[2], u3 = uk[3], u4 = uk[4], u5 = uk[5];
      double nx = ad_lane(xr, dt, cp, sp) + ((lane == 8) ? -a.g * dt : 0.0);
      if (lane >= 6 && lane < 9) {
        const int r = lane - 6;
        nx += bv<VAR>(r, 0, dtm, cp, sp) * u0 + bv<VAR>(r, 1, dtm, cp, sp) * u1 + bv<VAR>(r, 2, dtm, cp, sp) * u2;
      } else if (lane >= 9 && lane < 12) {
        const double* bwr = bw + 18 * k + 6 * (lane - 9);
        nx += ((bwr[0] * u0 + bwr[1] * u1) + (bwr[2] * u2 + bwr[3] * u3)) + (bwr[4] * u4 + bwr[5] * u5);
      }
      xr = lane < 12 ? nx : 0.0;
      const double kf = (k == N - 1) ? kTermQ : 1.0;
      const double e = lane < 12 ? xr - un[12 * k + lane] : 0.0;
      objl = fma(kf * qr * e, e, objl);
      if (k < N - 1 && lane < 6) {
        const double ub = a.uref_aliased ? ub_alias : ((cc[k] != 0.0) ? 2.0 * a.m * a.g : 0.0);
        const double du = uk[lane] - (lane == 2 ? ub : 0.0);
        objl = fma(kRdiag * du, du, objl);
      }
      if (lane < 12) xo[12 * (k + 1) + lane] = xr;
    }
    const double objv = wave_sum(objl);
    wsync();
    if (a.x)
      for (int i = lane; i < 12 * (N + 1); i += RT) a.x[b * 12 * (N + 1) + i] = xo[i];
    if (lane == 0) {
      if (a.obj) a.obj[b] = objv;
      a.status[b] = status;
      if (a.iters) a.iters[b] = iters;
    }
  }
}

template <int VAR>
__global__ void __launch_bounds__(RT) ric_kernel(SolveArgs a, int N, int cap) {
  extern __shared__ __attribute__((aligned(16))) double ric_sm[];
  const RicLay L(N, cap, true);
  ric_solve<VAR, 1>(a, N, (int64_t)blockIdx.x, ric_sm, ric_sm + L.RM, cap);
}

// the overflow pass: instances listed in a.ovf_list, capacity 6N, R in the
// global workspace (one block of rws_stride doubles per workgroup)
template <int VAR>
__global__ void __launch_bounds__(RT) ric_overflow_kernel(SolveArgs a, int N) {
  extern __shared__ __attribute__((aligned(16))) double ric_sm[];
  const int n = *a.ovf_count;
  double* Rm = a.rws + (int64_t)blockIdx.x * a.rws_stride;
  SolveArgs a2 = a;
  a2.ovf_count = nullptr;   // no further overflow: capacity is 6N
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int64_t b = a.ovf_list[i];
    ric_solve<VAR, (6 * kRicNmax + 63) / 64>(a2, N, b, ric_sm, Rm, 6 * N);
    __syncthreads();
  }
}

template <typename K>
bool set_lds(K kern, size_t bytes) {
  if (bytes <= 65536) return true;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess;
}

}  // namespace

size_t ric_lds_bytes(int N, int qcap) {
  const RicLay L(N, qcap > 0 ? qcap : 6 * N, qcap > 0);
  return (size_t)L.total * sizeof(double);
}

bool launch_solve_ric(int variant, int N, const SolveArgs& a, hipStream_t s) {
  if (N < 1 || N > kRicNmax || (variant != 2 && variant != 3)) return false;
  if (a.B <= 0) return true;
  const int cap = ric_qcap(N);
  const size_t lds = ric_lds_bytes(N, cap);
  if (variant == 3) {
    if (!set_lds(ric_kernel<3>, lds)) return false;
    hipLaunchKernelGGL(ric_kernel<3>, dim3((unsigned)a.B), dim3(RT), lds, s, a, N, cap);
  } else {
    if (!set_lds(ric_kernel<2>, lds)) return false;
    hipLaunchKernelGGL(ric_kernel<2>, dim3((unsigned)a.B), dim3(RT), lds, s, a, N, cap);
  }
  return true;
}

bool launch_solve_ric_overflow(int variant, int N, const SolveArgs& a, int groups, hipStream_t s) {
  if (N < 1 || N > kRicNmax || !a.ovf_count || !a.ovf_list || !a.rws || groups < 1) return false;
  const size_t lds = ric_lds_bytes(N, 0);
  if (variant == 3) {
    if (!set_lds(ric_overflow_kernel<3>, lds)) return false;
    hipLaunchKernelGGL(ric_overflow_kernel<3>, dim3((unsigned)groups), dim3(RT), lds, s, a, N);
  } else if (variant == 2) {
    if (!set_lds(ric_overflow_kernel<2>, lds)) return false;
    hipLaunchKernelGGL(ric_overflow_kernel<2>, dim3((unsigned)groups), dim3(RT), lds, s, a, N);
  } else {
    return false;
  }
  return true;
}

}  // namespace hmpc
