// hmpc_model.h -- the reference's MPC model pieces shared by the solve
// kernels (hmpc_kernels.hip: one wavefront per instance for the compiled
// horizons; hmpc_wide.hip: any other horizon).  Device code only.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace hmpc {

// ----------------------------------------------------------------------------
// constants of Mpc.__init__ / build_qp (src/mpc_cvx_euler_3f.py:20,35,37,113-129)
// ----------------------------------------------------------------------------
constexpr double kQ[12] = {50, 50, 2, 1, 1, 50, 1, 1, 1, 10, 10, 10};   // :35
constexpr double kRdiag = 0.001;   // R = 0.001 I   (:37)
constexpr double kTermQ = 100.0;   // kf at k = N-1 (:113)
constexpr double kFzMax = 206.0;   // f_max[2]      (:20)
constexpr double kZmin = 0.1;      //               (:129)
constexpr double kTol = 1e-10;     // scaled primal feasibility tolerance
__device__ __forceinline__ double tau_lim(int c) { return c == 5 ? 4.0 : 7.78; }   // :123-128

constexpr int ST_SOLVED = 0, ST_MAXIT = 1, ST_INFEAS = 2, ST_NUMERICAL = 3;

// ----------------------------------------------------------------------------
// cross-lane helpers (wave64; W waves per workgroup)
// ----------------------------------------------------------------------------
__device__ __forceinline__ double rdlane(double x, int l) {
  long long b = __double_as_longlong(x);
  int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float rdlane(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// 1/sqrt(p) to ~1 ulp without the IEEE sqrt + divide sequences (two dependent
// chains of ~15 f64 ops each): hardware v_rsq_f64 estimate, then one
// third-order correction y (1 + e/2 + 3e^2/8), e = 1 - p y^2.
__device__ __forceinline__ double rsq_nr(double p) {
  const double y = __builtin_amdgcn_rsq(p);
  const double e = fma(-(p * y), y, 1.0);
  return fma(y * e, fma(0.375, e, 0.5), y);
}
__device__ __forceinline__ float rsq_nr(float p) {   // fp32: v_rsq_f32 + one Newton step
  const float y = __builtin_amdgcn_rsqf(p);
  return y * fmaf(-0.5f * p * y, y, 1.5f);
}

// x of lane (r + D) within r's row of 16 lanes (D < 0: lane r - |D|); a DPP
// row shift -- a VALU modifier, no LDS round trip like a bpermute.  Lanes
// whose source falls outside their row read 0.
template <int D>
__device__ __forceinline__ int row_shift(int x) {
  static_assert(D != 0 && D > -16 && D < 16, "row shift");
  constexpr int ctrl = D > 0 ? 0x100 + D : 0x110 - D;   // row_shl:D / row_shr:-D
  return __builtin_amdgcn_update_dpp(0, x, ctrl, 0xf, 0xf, true);
}
template <int D>
__device__ __forceinline__ double row_shift(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = row_shift<D>((int)(b & 0xffffffffLL)), hi = row_shift<D>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int D>
__device__ __forceinline__ float row_shift(float x) {
  return __int_as_float(row_shift<D>(__float_as_int(x)));
}

// DPP lane permutes within a row of 16 lanes (VALU modifiers: no LDS round
// trip, unlike the bpermute behind __shfl_xor).
// (mov_dpp: no "old" operand -- every control used here reads a valid lane of
// the row, so the old value was never selected, but update_dpp(0, ...) made
// the compiler materialise the 0 in two v_movs per 64-bit permute)
template <int CTRL>
__device__ __forceinline__ int dpp(int x) { return __builtin_amdgcn_mov_dpp(x, CTRL, 0xf, 0xf, false); }
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = dpp<CTRL>((int)(b & 0xffffffffLL)), hi = dpp<CTRL>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float x) { return __int_as_float(dpp<CTRL>(__float_as_int(x))); }
constexpr int kDppXor1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // lane i <-> 7-i within each half row
constexpr int kDppMirror = 0x140;      // lane i <-> 15-i within each row

// Sum over the wave, returned wave-uniform: a DPP butterfly inside each row
// of 16 lanes (xor 1, xor 2, half mirror, mirror: every lane then holds its
// row's sum), then the four row sums by readlane.  Call with every lane
// active (lanes without data contribute 0).
template <typename R>
__device__ __forceinline__ R wave_sum(R x) {
  x += dpp<kDppXor1>(x);
  x += dpp<kDppXor2>(x);
  x += dpp<kDppHalfMirror>(x);
  x += dpp<kDppMirror>(x);
  return (rdlane(x, 0) + rdlane(x, 16)) + (rdlane(x, 32) + rdlane(x, 48));
}

template <typename R>
__device__ __forceinline__ void argmin_combine(R& v, int& i, R v2, int i2) {
  if (v2 < v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
// the same, branch-free (selects, not an exec-masked branch per combine:
// the dense kernels, round 5; the Riccati kernels keep the branch form,
// which their register allocation at the 2-wave cap is tuned to)
template <typename R>
__device__ __forceinline__ void argmin_combine_sel(R& v, int& i, R v2, int i2) {
  const bool take = (v2 < v) | ((v2 == v) & (i2 < i));
  v = take ? v2 : v;
  i = take ? i2 : i;
}

// (min v, its smallest i) over the wave, wave-uniform; the same row butterfly
// + readlane shape as wave_sum.  Lexicographic (v, i) minimum: independent of
// the combining order.
template <bool SEL = false, typename R>
__device__ __forceinline__ void wave_argmin(R& v, int& i) {
  auto comb = [](R& a, int& ia, R b, int ib) __attribute__((always_inline)) {
    if constexpr (SEL) argmin_combine_sel(a, ia, b, ib);
    else argmin_combine(a, ia, b, ib);
  };
  comb(v, i, dpp<kDppXor1>(v), dpp<kDppXor1>(i));
  comb(v, i, dpp<kDppXor2>(v), dpp<kDppXor2>(i));
  comb(v, i, dpp<kDppHalfMirror>(v), dpp<kDppHalfMirror>(i));
  comb(v, i, dpp<kDppMirror>(v), dpp<kDppMirror>(i));
  R vb = rdlane(v, 0);
  int ib = __builtin_amdgcn_readlane(i, 0);
  comb(vb, ib, rdlane(v, 16), __builtin_amdgcn_readlane(i, 16));
  comb(vb, ib, rdlane(v, 32), __builtin_amdgcn_readlane(i, 32));
  comb(vb, ib, rdlane(v, 48), __builtin_amdgcn_readlane(i, 48));
  v = vb;
  i = ib;
}

// S_t storage order (22 entries):
//   0..8   per axis a: [pp, pv, vv] at 3a    (p_a = x[a], v_a = x[6+a])
//   9..11  yaw: [tt, tw, ww]                 (theta_z = x[5], w_z = x[11])
//   12..21 roll/pitch block y = (x3, x4, x9, x10):
//          P00 P01 P11 M00 M01 M10 M11 Q00 Q01 Q11  (M_ij = S[x(3+i)][x(9+j)])
// f = S e for the structured S (full 12 rows).  LOWER0: e[0..5] are zero
// (an input impulse), so their products are skipped rather than multiplied
// by a zero the compiler may not fold away.
template <bool LOWER0 = false, typename R>
__device__ __forceinline__ void s_times(const R* s, const R (&e)[12], R (&f)[12]) {
  const R P00 = s[12], P01 = s[13], P11 = s[14], M00 = s[15], M01 = s[16], M10 = s[17],
               M11 = s[18], Q00 = s[19], Q01 = s[20], Q11 = s[21];
  if constexpr (LOWER0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      f[a] = s[3 * a + 1] * e[6 + a];
      f[6 + a] = s[3 * a + 2] * e[6 + a];
    }
    f[5] = s[10] * e[11];
    f[11] = s[11] * e[11];
    f[3] = M00 * e[9] + M01 * e[10];
    f[4] = M10 * e[9] + M11 * e[10];
    f[9] = Q00 * e[9] + Q01 * e[10];
    f[10] = Q01 * e[9] + Q11 * e[10];
    return;
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    f[a] = s[3 * a] * e[a] + s[3 * a + 1] * e[6 + a];
    f[6 + a] = s[3 * a + 1] * e[a] + s[3 * a + 2] * e[6 + a];
  }
  f[5] = s[9] * e[5] + s[10] * e[11];
  f[11] = s[10] * e[5] + s[11] * e[11];
  f[3] = P00 * e[3] + P01 * e[4] + M00 * e[9] + M01 * e[10];
  f[4] = P01 * e[3] + P11 * e[4] + M10 * e[9] + M11 * e[10];
  f[9] = M00 * e[3] + M10 * e[4] + Q00 * e[9] + Q01 * e[10];
  f[10] = M01 * e[3] + M11 * e[4] + Q01 * e[9] + Q11 * e[10];
}

// x <- Ad x with Ad = I + dt A(psi): p += dt v; theta += dt Rz(psi) w
// (src/mpc_cvx_euler_3f.py:27,87,91; rz of src/utils.py:46-51)
template <typename R>
__device__ __forceinline__ void ad_times(R (&x)[12], R dt, R cp, R sp) {
#pragma unroll
  for (int a = 0; a < 3; ++a) x[a] = fma(dt, x[6 + a], x[a]);
  const R w0 = x[9], w1 = x[10];
  x[3] = x[3] + ((cp * dt) * w0 + (sp * dt) * w1);
  x[4] = x[4] + ((-sp * dt) * w0 + (cp * dt) * w1);
  x[5] = fma(dt, x[11], x[5]);
}
// g <- Ad' g
template <typename R>
__device__ __forceinline__ void adt_times(R (&g)[12], R dt, R cp, R sp) {
#pragma unroll
  for (int a = 0; a < 3; ++a) g[6 + a] = fma(dt, g[a], g[6 + a]);
  const R g3 = g[3], g4 = g[4];
  g[9] = g[9] + ((cp * dt) * g3 + (-sp * dt) * g4);
  g[10] = g[10] + ((sp * dt) * g3 + (cp * dt) * g4);
  g[11] = fma(dt, g[5], g[11]);
}

// The same two maps lane-parallel: lane r < 12 holds component r.  The
// cross terms come from other lanes (readlane / DPP row shift); lanes >= 12 pass
// their value through unchanged.  Branch-free: d_r = al_r x[r+-6] + sp beta_r
// with per-lane 0/1 coefficients (no per-lane selects of the terms).  r is
// the caller's lane (an opaque copy keeps the coefficients from being hoisted
// out of a persistent loop).
template <typename R>
__device__ __forceinline__ R ad_lane(R x, R dt, R cp, R sp, int r = threadIdx.x) {
  // r < 3: v; r = 3, 4: Rz w (cp w0 + sp w1, cp w1 - sp w0); r = 5: w2
  const R xv = row_shift<6>(x);   // x[r+6] for r < 6
  const R w0 = rdlane(x, 9), w1 = rdlane(x, 10);
  const R k1 = (r == 3 || r == 4) ? R(1) : R(0);
  const R k0 = (r < 6 && r != 3 && r != 4) ? R(1) : R(0);
  const R s1 = (r == 3) ? R(1) : R(0), s0 = (r == 4) ? R(-1) : R(0);
  const R d = fma(fma(k1, cp, k0), xv, sp * fma(s1, w1, s0 * w0));
  return fma(dt, d, x);
}
template <typename R>
__device__ __forceinline__ R adt_lane(R g, R dt, R cp, R sp, int r = threadIdx.x) {
  // 6 <= r < 9: g[r-6]; r = 9, 10: Rz' (cp g3 - sp g4, sp g3 + cp g4); r = 11: g5
  const R gv = row_shift<-6>(g);  // g[r-6] for 6 <= r < 12
  const R g3 = rdlane(g, 3), g4 = rdlane(g, 4);
  const R k1 = (r == 9 || r == 10) ? R(1) : R(0);
  const R k0 = (r >= 6 && r < 12 && r != 9 && r != 10) ? R(1) : R(0);
  const R s3 = (r == 10) ? R(1) : R(0), s4 = (r == 9) ? R(-1) : R(0);
  const R d = fma(fma(k1, cp, k0), gv, sp * fma(s3, g3, s4 * g4));
  return fma(dt, d, g);
}
// The select form of the same maps: fewer live lane constants, for the
// generic kernel whose register budget is already spent (the coefficient form
// above spills there)
template <typename R>
__device__ __forceinline__ R ad_lane_sel(R x, R dt, R cp, R sp) {
  const int r = threadIdx.x;
  const R xv = row_shift<6>(x);
  const R w0 = rdlane(x, 9), w1 = rdlane(x, 10), w2 = rdlane(x, 11);
  R d = R(0);
  d = (r < 3) ? xv : d;
  d = (r == 3) ? (cp * w0 + sp * w1) : d;
  d = (r == 4) ? (cp * w1 - sp * w0) : d;
  d = (r == 5) ? w2 : d;
  return fma(dt, d, x);
}
template <typename R>
__device__ __forceinline__ R adt_lane_sel(R g, R dt, R cp, R sp) {
  const int r = threadIdx.x;
  const R gv = row_shift<-6>(g);
  const R g3 = rdlane(g, 3), g4 = rdlane(g, 4), g5 = rdlane(g, 5);
  R d = R(0);
  d = (r >= 6 && r < 9) ? gv : d;
  d = (r == 9) ? (cp * g3 - sp * g4) : d;
  d = (r == 10) ? (sp * g3 + cp * g4) : d;
  d = (r == 11) ? g5 : d;
  return fma(dt, d, g);
}
__device__ __forceinline__ double qdiag(int r) {   // Q[r][r], 0 beyond the state
  return (r == 0 || r == 1 || r == 5) ? 50.0 : (r == 2 ? 2.0 : (r >= 9 && r < 12) ? 10.0 : (r < 12 ? 1.0 : 0.0));
}

// rows 6..8 of Bd_k, column c2 (< 3): 3f dt/m I (:28), 2f Rz'(psi) dt/m (2f :87)
template <int VAR, typename R>
__device__ __forceinline__ R bv(int r, int c2, R dtm, R cp, R sp) {
  if constexpr (VAR == 3) {
    return r == c2 ? dtm : R(0);
  } else {
    // Rz' = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
    if (r == 2 || c2 == 2) return (r == c2) ? dtm : R(0);
    if (r == c2) return cp * dtm;
    return (r == 0) ? -sp * dtm : sp * dtm;
  }
}

// 2 Bd_j[:, c2]' y[6..11]  (rows 0..5 of Bd are zero)
template <int VAR, typename R>
__device__ __forceinline__ R bd_dot(int c2, const R (&y)[12], const R* bw, R dtm,
                                         R cp, R sp) {
  R acc = R(0);
  if constexpr (VAR == 3) {   // dt/m I: one product (no FMAs by structural zeros)
    if (c2 < 3) acc = dtm * y[6 + c2];
  } else if (c2 < 3) {
#pragma unroll
    for (int r = 0; r < 3; ++r) acc = fma(bv<VAR>(r, c2, dtm, cp, sp), y[6 + r], acc);
  }
#pragma unroll
  for (int r = 0; r < 3; ++r) acc = fma(bw[6 * r + c2], y[9 + r], acc);
  return R(2) * acc;
}

// Mpc.gen_dt_dynamics for stage k (3f :71-94, 2f :70-94): cos/sin of the
// linearisation yaw and rows 9..11 of Bd_k (rows 6..8 are bv(); the rest of
// Bd_k is zero).  xlin: [N][12] linearisation rows, pf: [N][3].
// Same from values: psi = x_lin[k][5], p = x_lin[k][0:3], pfk = pf[k].
template <int VAR, typename R>
__device__ __forceinline__ void stage_dynamics_vals(int k, R psi, const R (&p)[3], const R (&pfk)[3],
                                                    const double (&Jinv)[9], const double (&rh)[3],
                                                    R dt, R* cs, R* bwo) {
  R sp, cp;
  if constexpr (sizeof(R) == 4) sincosf(psi, &sp, &cp);
  else sincos(psi, &sp, &cp);
  // rz(psi) = [[c, s, 0], [-s, c, 0], [0, 0, 1]]   (src/utils.py:46-51)
  const R Rz[3][3] = {{cp, sp, R(0)}, {-sp, cp, R(0)}, {R(0), R(0), R(1)}};
  R d[3], rf[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) d[i] = pfk[i] - p[i];
  // rf = rh + Rz (pf - p)   (:84)
#pragma unroll
  for (int i = 0; i < 3; ++i) rf[i] = R(rh[i]) + (Rz[i][0] * d[0] + Rz[i][1] * d[1] + Rz[i][2] * d[2]);
  R T[3][3], Jw[3][3], RzT[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) RzT[i][j] = Rz[j][i];
  // J_w_inv = Rz Jinv Rz'   (:86)
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      T[i][j] = Rz[i][0] * R(Jinv[0 * 3 + j]) + Rz[i][1] * R(Jinv[1 * 3 + j]) + Rz[i][2] * R(Jinv[2 * 3 + j]);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) Jw[i][j] = T[i][0] * RzT[0][j] + T[i][1] * RzT[1][j] + T[i][2] * RzT[2][j];
  R Bwt[3][3], Bwf[3][3];
  // B[9:12, 3:6] = J_w_inv Rz'   (:89)
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) Bwt[i][j] = Jw[i][0] * RzT[0][j] + Jw[i][1] * RzT[1][j] + Jw[i][2] * RzT[2][j];
  R w[3];
  if constexpr (VAR == 3) {   // rhat = hat(Rz' rf); B[9:12,0:3] = Jw rhat   (:85,88)
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = RzT[i][0] * rf[0] + RzT[i][1] * rf[1] + RzT[i][2] * rf[2];
  } else {                    // rhat = hat(rf); B[9:12,0:3] = (Jw Rz') rhat   (2f :84,88)
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = rf[i];
  }
  // hat (src/utils.py:21-25)
  const R hw[3][3] = {{R(0), -w[2], w[1]}, {w[2], R(0), -w[0]}, {-w[1], w[0], R(0)}};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if constexpr (VAR == 3)
        Bwf[i][j] = Jw[i][0] * hw[0][j] + Jw[i][1] * hw[1][j] + Jw[i][2] * hw[2][j];
      else
        Bwf[i][j] = Bwt[i][0] * hw[0][j] + Bwt[i][1] * hw[1][j] + Bwt[i][2] * hw[2][j];
    }
  R* bw = bwo + 18 * k;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      bw[i * 6 + j] = Bwf[i][j] * dt;
      bw[i * 6 + 3 + j] = Bwt[i][j] * dt;
    }
  cs[2 * k] = cp;
  cs[2 * k + 1] = sp;
}

template <int VAR, typename R>
__device__ __forceinline__ void stage_dynamics(int k, const R* xlin, const R* pf,
                                               const double (&Jinv)[9], const double (&rh)[3], R dt,
                                               R* cs, R* bwo) {
  const R p[3] = {xlin[12 * k], xlin[12 * k + 1], xlin[12 * k + 2]};
  const R pfk[3] = {pf[3 * k], pf[3 * k + 1], pf[3 * k + 2]};
  stage_dynamics_vals<VAR, R>(k, xlin[12 * k + 5], p, pfk, Jinv, rh, dt, cs, bwo);
}

}  // namespace hmpc
