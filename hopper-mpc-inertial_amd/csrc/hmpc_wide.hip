// hmpc_wide.hip -- the same QP for horizons without a dedicated kernel
// (the Runner's default N = 60, src/robotrunner.py:46, and any other
// 1 <= N <= kWideNmax).
//
// The one-wavefront kernel (hmpc_kernels.hip) keeps a row of the condensed
// Hessian in registers and the whole factor in LDS; at N = 60 the factor
// alone is 520 KB.  Here one 256-thread workgroup solves an instance out of a
// per-workgroup global workspace (WideLayout, L2-resident), fixed variables
// are compacted away first (swing forces, 2f fy: NF <= NV free variables),
// and the dual active set is the classic Goldfarb-Idnani form with an
// explicit J = L^-T Q, whose every step is a parallel sweep over J:
//
//   0  inputs -> workspace (plan views as in the fast kernel)
//   1  gen_dt_dynamics per stage (3f :71-94, 2f :70-94)
//   2  free response, cost-to-go S_t, adjoint (wave 0; same recursions as the
//      fast kernel's phase 2)
//   3  free-variable map; Hessian rows over the free variables (thread per
//      row: g_j = Ad_{j+1}' g_{j+1} from S_{i+1} B_i e_c) and gradient
//   4  Cholesky H = L L' (right-looking, trailing rows updated coalesced)
//   5  J = L^-T (thread per column of L^-1, independent forward substitutions)
//   6  Goldfarb-Idnani: d = J' n_p from the <= N nonzeros of n_p (rows of
//      J), z = J2 d2 (wave-per-row dot products), adds by ONE Householder
//      reflection of J's trailing columns (two parallel passes; Givens would
//      be NF - q dependent rotations), drops by Givens on R and J
//   7  outputs as the fast kernel (x* rollout, objective)
//
// Constraints and tolerances are those of the fast kernel (one id per
// variable and slot: torque box :123-128, fz box + friction :141-146,
// z >= 0.1 :129).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "hmpc_internal.h"
#include "hmpc_model.h"

namespace hmpc {

namespace {

constexpr int WT = 256;               // threads per workgroup
constexpr int WW = WT / 64;           // waves
constexpr int NVMAX = 6 * kWideNmax;  // LDS vectors
constexpr int kPanelElems = 6144;     // NV x PB: PB = 16 up to NV = 384, else 8
constexpr int QL = 78;                // active-set capacity: R (QL x QL) lives in the panel buffer

template <typename T>
struct Shared {
  T red[WW];
  int ired[WW];
  T vec[NVMAX];   // a broadcast vector (Cholesky column, d, Householder v)
  T vec2[NVMAX];
  T pan[kPanelElems];   // Cholesky panel (rows k0.., PB columns)
  T npv[kWideNmax + 2];   // n_p: <= N nonzeros (z rows), else <= 2
  int npi[kWideNmax + 2];
  int npn;
  int nf;
  int p;
  int kd;
  int flag;
  T best, bp, t1, sp, gc, gs;
};

template <typename T>
__device__ T block_sum(T x, Shared<T>& sh) {
  x = wave_sum(x);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh.red[threadIdx.x >> 6] = x;
  __syncthreads();
  T s = T(0);
#pragma unroll
  for (int w = 0; w < WW; ++w) s += sh.red[w];
  return s;
}

template <typename T>
__device__ void block_argmin(T& v, int& i, Shared<T>& sh) {
  wave_argmin(v, i);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sh.red[threadIdx.x >> 6] = v;
    sh.ired[threadIdx.x >> 6] = i;
  }
  __syncthreads();
  v = sh.red[0];
  i = sh.ired[0];
#pragma unroll
  for (int w = 1; w < WW; ++w) argmin_combine(v, i, sh.red[w], sh.ired[w]);
}

// out[i] = sum_{k in [k0, n)} M[i*ld + k] vec[k] for rows i < n: one wave per
// row, lanes over k (coalesced), then a wave reduction.
template <typename T>
__device__ void rows_dot(const T* M, int ld, int n, int k0, const T* vec, T* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < n; i += WW) {
    const T* row = M + (int64_t)i * ld;
    T acc = T(0);
    for (int k = k0 + lane; k < n; k += 64) acc = fma(row[k], vec[k], acc);
    acc = wave_sum(acc);
    if (lane == 0) out[i] = acc;
  }
}

__device__ __forceinline__ void gfence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

#ifdef HMPC_STAMPS
#define WSTAMP(i) (wst[i] = __builtin_amdgcn_s_memtime())
#else
#define WSTAMP(i) ((void)0)
#endif

template <int VAR, typename T>
__device__ void wide_solve(const SolveArgs& a, const int N, const int64_t b, T* ws, Shared<T>& sh) {
#ifdef HMPC_STAMPS
  long long wst[10] = {0};
#endif
  WSTAMP(0);
  const WideLayout Lw(N);
  const int tid = threadIdx.x;
  const int NV = 6 * N;
  const T dt = T(a.dt), dtm = dt / T(a.m);
  T* xin = ws + Lw.XIN;
  T* cc = ws + Lw.CC;
  T* cs = ws + Lw.CS;
  T* bw = ws + Lw.BW;
  T* zb = ws + Lw.ZB;
  T* xl = ws + Lw.XL;
  T* xr = ws + Lw.XR;
  T* pf = ws + Lw.PF;
  T* ss = ws + Lw.SS;
  T* dg = ws + Lw.DG;
  T* aj = ws + Lw.AJ;
  T* hv = ws + Lw.HV;
  T* xv = ws + Lw.XV;
  T* dv = ws + Lw.DV;
  T* zv = ws + Lw.ZV;
  T* wv = ws + Lw.WV;
  T* uo = ws + Lw.UO;
  T* rv = ws + Lw.RV;
  T* ua = ws + Lw.UA;
  int* fr = reinterpret_cast<int*>(ws + Lw.FR);
  int* pos = reinterpret_cast<int*>(ws + Lw.POS);
  int* act = reinterpret_cast<int*>(ws + Lw.ACT);
  int* isa = reinterpret_cast<int*>(ws + Lw.ISA);
  T* H = ws + Lw.H;
  T* J = ws + Lw.J;
  const int ld = NV;   // row stride of H, J, R
  // feasibility / degeneracy thresholds scaled to the arithmetic
  const T tol = sizeof(T) == 4 ? T(1e-4) : T(kTol);
  const T tiny = sizeof(T) == 4 ? T(1e-12) : T(1e-24);

  // ---------------- 0: inputs ------------------------------------------------
  {
    const double* xrf = a.x_ref + b * a.xref_bs;
    for (int i = tid; i < 12; i += WT) xin[i] = a.x_in[b * 12 + i];
    for (int i = tid; i < 12 * N; i += WT) xr[i] = xrf[(int64_t)(i / 12) * a.xref_rs + i % 12];
    for (int i = tid; i < 3 * N; i += WT) pf[i] = a.pf[b * a.pf_bs + (int64_t)(i / 3) * a.pf_rs + i % 3];
    for (int i = tid; i < N; i += WT) cc[i] = a.C[b * a.C_bs + i];
    gfence();
    __syncthreads();
    const double* xp = a.x_lin + b * 12 * (N + 1);
    for (int i = tid; i < 12 * N; i += WT) {
      const int r = i / 12, c = i - 12 * r;
      T v;
      if (a.shift_mode == 0) v = xp[i];
      else if (a.shift_mode == 1) v = r == 0 ? xin[c] : xr[i - 12];   // [x_in; x_ref] (3f :52-53)
      else v = r == 0 ? xin[c] : xp[(r + 1) * 12 + c];               // time shift (3f :59-62)
      xl[i] = v;
    }
    gfence();
    __syncthreads();
  }
  WSTAMP(1);
  // ---------------- 1: gen_dt_dynamics --------------------------------------
  for (int k = tid; k < N; k += WT) stage_dynamics<VAR>(k, xl, pf, a.Jinv, a.rh, dt, cs, bw);
  gfence();
  __syncthreads();
  WSTAMP(2);
  // ---------------- 2: free response, S_t, adjoint (wave 0) -----------------
  if (tid < 64) {
    T xrr = tid < 12 ? xin[tid] : T(0.0);
    const T qr = T(qdiag(tid));
    T s[22];
#pragma unroll
    for (int a3 = 0; a3 < 3; ++a3) {
      s[3 * a3] = T(kTermQ) * T(kQ[a3]);
      s[3 * a3 + 1] = T(0.0);
      s[3 * a3 + 2] = T(kTermQ) * T(kQ[6 + a3]);
    }
    s[9] = T(kTermQ) * T(kQ[5]); s[10] = T(0.0); s[11] = T(kTermQ) * T(kQ[11]);
    s[12] = T(kTermQ) * T(kQ[3]); s[13] = T(0.0); s[14] = T(kTermQ) * T(kQ[4]);
    s[15] = s[16] = s[17] = s[18] = T(0.0);
    s[19] = T(kTermQ) * T(kQ[9]); s[20] = T(0.0); s[21] = T(kTermQ) * T(kQ[10]);
    if (tid == 2) zb[0] = xrr;
    if (tid == 0)
      for (int e = 0; e < 22; ++e) ss[22 * (N - 1) + e] = s[e];
    for (int k = 0; k < N; ++k) {
      const T cp = cs[2 * k], sp = cs[2 * k + 1];
      xrr = ad_lane_sel(xrr, dt, cp, sp) + ((tid == 8) ? -T(a.g) * dt : T(0.0));
      const T kf = (k == N - 1) ? T(kTermQ) : T(1.0);
      if (tid < 12) dg[12 * k + tid] = kf * qr * (xrr - xr[12 * k + tid]);
      if (tid == 2) zb[k + 1] = xrr;
      const int t = N - 1 - k;
      if (t >= 1) {
        const T ct = cs[2 * t], st = cs[2 * t + 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int o = 3 * q;
          const T aa = s[o], bb = s[o + 1], cc2 = s[o + 2];
          s[o + 1] = fma(dt, aa, bb);
          s[o + 2] = cc2 + dt * (T(2.0) * bb + dt * aa);
        }
        const T D00 = ct * dt, D01 = st * dt, D10 = -st * dt, D11 = ct * dt;
        const T P00 = s[12], P01 = s[13], P11 = s[14];
        const T M00 = s[15], M01 = s[16], M10 = s[17], M11 = s[18];
        const T N00 = M00 + (P00 * D00 + P01 * D10), N01 = M01 + (P00 * D01 + P01 * D11);
        const T N10 = M10 + (P01 * D00 + P11 * D10), N11 = M11 + (P01 * D01 + P11 * D11);
        const T A00 = D00 * N00 + D10 * N10, A01 = D00 * N01 + D10 * N11;
        const T A11 = D01 * N01 + D11 * N11;
        const T B00 = M00 * D00 + M10 * D10, B01 = M00 * D01 + M10 * D11;
        const T B11 = M01 * D01 + M11 * D11;
        s[19] += A00 + B00;
        s[20] += A01 + B01;
        s[21] += A11 + B11;
        s[15] = N00; s[16] = N01; s[17] = N10; s[18] = N11;
#pragma unroll
        for (int a3 = 0; a3 < 3; ++a3) {
          s[3 * a3] += T(kQ[a3]);
          s[3 * a3 + 2] += T(kQ[6 + a3]);
        }
        s[9] += T(kQ[5]); s[11] += T(kQ[11]);
        s[12] += T(kQ[3]); s[14] += T(kQ[4]);
        s[19] += T(kQ[9]); s[21] += T(kQ[10]);
        if (tid == 0)
          for (int e = 0; e < 22; ++e) ss[22 * (t - 1) + e] = s[e];
      }
    }
    gfence();
    T ar = tid < 12 ? dg[12 * (N - 1) + tid] : T(0.0);
    if (tid >= 6 && tid < 12) aj[6 * (N - 1) + tid - 6] = ar;
    for (int t = N - 1; t >= 1; --t) {
      ar = adt_lane_sel(ar, dt, cs[2 * t], cs[2 * t + 1]) + (tid < 12 ? dg[12 * (t - 1) + tid] : T(0.0));
      if (tid >= 6 && tid < 12) aj[6 * (t - 1) + tid - 6] = ar;
    }
  }
  WSTAMP(3);
  // ---------------- 3: free variables, Hessian rows, gradient ----------------
  if (tid == 0) {
    int nf = 0;
    for (int v = 0; v < NV; ++v) {
      const int k = v / 6, c = v - 6 * k;
      const bool fixed = (c < 3 && cc[k] == T(0.0)) || (VAR == 2 && c == 1);   // :134-136, 2f :129
      pos[v] = fixed ? -1 : nf;
      if (!fixed) fr[nf++] = v;
    }
    sh.nf = nf;
  }
  gfence();
  __syncthreads();
  const int NF = sh.nf;
  const T ubar_alias = (cc[N - 1] != T(0.0)) ? T(2.0) * T(a.m) * T(a.g) : T(0.0);
  for (int r = tid; r < NF; r += WT) {
    const int v = fr[r];
    const int ii = v / 6, ci = v - 6 * ii;
    const T cpi = cs[2 * ii], spi = cs[2 * ii + 1];
    const T* bwi = bw + 18 * ii;
    T e0[12], f[12], g[12];
    for (int q = 0; q < 6; ++q) e0[q] = T(0.0);
    for (int q = 0; q < 3; ++q) e0[6 + q] = ci < 3 ? bv<VAR>(q, ci, dtm, cpi, spi) : T(0.0);
    for (int q = 0; q < 3; ++q) e0[9 + q] = bwi[6 * q + ci];
    s_times(ss + 22 * ii, e0, f);
    T* Hr = H + (int64_t)r * ld;
    for (int c2 = 0; c2 <= ci; ++c2) {   // diagonal block, columns <= mine
      const int pw = pos[6 * ii + c2];
      if (pw < 0) continue;
      T hd = bd_dot<VAR>(c2, f, bwi, dtm, cpi, spi);
      if (c2 == ci && ii != N - 1) hd += T(2.0) * T(kRdiag);
      Hr[pw] = hd;
    }
    T hacc = T(0.0);
    for (int q = 0; q < 6; ++q) hacc = fma(e0[6 + q], aj[6 * ii + q], hacc);
    for (int q = 0; q < 12; ++q) g[q] = f[q];
    for (int j = ii - 1; j >= 0; --j) {
      adt_times(g, dt, cs[2 * (j + 1)], cs[2 * (j + 1) + 1]);
      const T cp = cs[2 * j], sp = cs[2 * j + 1];
      for (int c2 = 0; c2 < 6; ++c2) {
        const int pw = pos[6 * j + c2];
        if (pw >= 0) Hr[pw] = bd_dot<VAR>(c2, g, bw + 18 * j, dtm, cp, sp);
      }
    }
    T ub = T(0.0);
    if (ci == 2) ub = a.uref_aliased ? ubar_alias : ((cc[ii] != T(0.0)) ? T(2.0) * T(a.m) * T(a.g) : T(0.0));
    const T Vj = (ii == N - 1) ? T(0.0) : T(kRdiag);
    hv[r] = T(2.0) * hacc - T(2.0) * Vj * ub;
  }
  gfence();
  __syncthreads();

  int status = ST_SOLVED;
  WSTAMP(4);
  // ---------------- 4: Cholesky --------------------------------------------
  // Blocked right-looking: a panel of PB columns is factored in LDS, written
  // back, and the trailing lower triangle gets one rank-PB update by 4 x 4
  // register tiles -- one pass over the trailing matrix per panel instead
  // of one per column.
  {
    const int PB = NV <= 384 ? 16 : 8;
    T* P = sh.pan;
    for (int k0 = 0; k0 < NF && status == ST_SOLVED; k0 += PB) {
      const int pw = NF - k0 < PB ? NF - k0 : PB;
      const int m = NF - k0;
      for (int e = tid; e < m * PB; e += WT) {
        const int r = e / PB, c = e - PB * r;
        P[e] = (c < pw && c <= r) ? H[(int64_t)(k0 + r) * ld + k0 + c] : T(0);
      }
      __syncthreads();
      for (int c = 0; c < pw; ++c) {
        const T piv = P[c * PB + c];
        if (!(piv > T(0))) { status = ST_NUMERICAL; break; }   // uniform
        const T lkk = sqrt(piv), rl = T(1) / lkk;
        __syncthreads();   // every thread has read the pivot
        for (int r = c + 1 + tid; r < m; r += WT) P[r * PB + c] *= rl;
        if (tid == 0) P[c * PB + c] = lkk;
        __syncthreads();
        const int nc = pw - c - 1;
        if (nc > 0) {
          for (int e = tid; e < (m - c - 1) * nc; e += WT) {
            const int rr = c + 1 + e / nc, cc = c + 1 + e % nc;
            if (rr >= cc) P[rr * PB + cc] = fma(-P[rr * PB + c], P[cc * PB + c], P[rr * PB + cc]);
          }
          __syncthreads();
        }
      }
      if (status != ST_SOLVED) break;
      for (int e = tid; e < m * PB; e += WT) {
        const int r = e / PB, c = e - PB * r;
        if (c < pw && c <= r) H[(int64_t)(k0 + r) * ld + k0 + c] = P[e];
      }
      // trailing rank-pw update of rows/cols >= k0 + pw, 4 x 4 tiles
      const int t0 = k0 + pw, mt = NF - t0;
      const int T4 = (mt + 3) / 4;
      const int ntile = T4 * (T4 + 1) / 2;
      for (int tp = tid; tp < ntile; tp += WT) {
        int ti = (int)((sqrtf(8.0f * (float)tp + 1.0f) - 1.0f) * 0.5f);
        while (ti * (ti + 1) / 2 > tp) --ti;
        while ((ti + 1) * (ti + 2) / 2 <= tp) ++ti;
        const int tj = tp - ti * (ti + 1) / 2;
        const int i0 = t0 + 4 * ti, j0 = t0 + 4 * tj;
        T acc[4][4];
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
          for (int b2 = 0; b2 < 4; ++b2) acc[a2][b2] = T(0);
        for (int c = 0; c < pw; ++c) {
          T av[4], bvv[4];
#pragma unroll
          for (int a2 = 0; a2 < 4; ++a2) {
            const int ri = i0 + a2 - k0, rj = j0 + a2 - k0;
            av[a2] = ri < m ? P[ri * PB + c] : T(0);
            bvv[a2] = rj < m ? P[rj * PB + c] : T(0);
          }
#pragma unroll
          for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
            for (int b2 = 0; b2 < 4; ++b2) acc[a2][b2] = fma(av[a2], bvv[b2], acc[a2][b2]);
        }
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2) {
          const int ii = i0 + a2;
          if (ii >= NF) continue;
          T* Hi = H + (int64_t)ii * ld;
#pragma unroll
          for (int b2 = 0; b2 < 4; ++b2) {
            const int jj = j0 + b2;
            if (jj <= ii) Hi[jj] -= acc[a2][b2];
          }
        }
      }
      gfence();
      __syncthreads();
    }
  }
  WSTAMP(5);
  // ---------------- 5: J = L^-T (row c of J = column c of L^-1) -------------
  // Y = L^-1 by blocks of rows: a block's rows first take the contribution of
  // every earlier block (4 x 4 register tiles over rows of L staged in LDS and
  // rows of J = Y'), then a short forward substitution inside the block, one
  // thread per column (no barrier: a column's entries are that thread's).
  if (status == ST_SOLVED) {
    for (int64_t e = tid; e < (int64_t)NF * ld; e += WT) J[e] = T(0);
    gfence();
    __syncthreads();
    const int RB = NV <= 384 ? 16 : 8;
    T* Lb = sh.pan;   // rows rb..re-1 of L, columns 0..re-1 (stride re)
    for (int rb = 0; rb < NF; rb += RB) {
      const int re = NF - rb < RB ? NF : rb + RB;
      const int h = re - rb;
      for (int e = tid; e < h * re; e += WT) {
        const int r = e / re, k = e - re * r;
        Lb[e] = (k <= rb + r) ? H[(int64_t)(rb + r) * ld + k] : T(0);
      }
      __syncthreads();
      // A: J[c][rb + r] = delta(rb + r, c) - sum_{k < rb} L[rb + r][k] Y[k][c]
      const int TC = (re + 3) / 4, TR = (h + 3) / 4;
      for (int tp = tid; tp < TR * TC; tp += WT) {
        const int tr = tp / TC, tc = tp - TC * tr;
        const int r0 = 4 * tr, c0 = 4 * tc;
        T acc[4][4];
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
          for (int b2 = 0; b2 < 4; ++b2) acc[a2][b2] = T(0);
        const T* Jc[4];
#pragma unroll
        for (int b2 = 0; b2 < 4; ++b2) Jc[b2] = J + (int64_t)(c0 + b2 < re ? c0 + b2 : c0) * ld;
        for (int k = c0; k < rb; ++k) {   // Y[k][c] = 0 for k < c
          T av[4], bvv[4];
#pragma unroll
          for (int a2 = 0; a2 < 4; ++a2) av[a2] = r0 + a2 < h ? Lb[(r0 + a2) * re + k] : T(0);
#pragma unroll
          for (int b2 = 0; b2 < 4; ++b2) bvv[b2] = Jc[b2][k];
#pragma unroll
          for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
            for (int b2 = 0; b2 < 4; ++b2) acc[a2][b2] = fma(av[a2], bvv[b2], acc[a2][b2]);
        }
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2) {
          const int r = rb + r0 + a2;
          if (r0 + a2 >= h) continue;
#pragma unroll
          for (int b2 = 0; b2 < 4; ++b2) {
            const int c = c0 + b2;
            if (c < re) J[(int64_t)c * ld + r] = ((r == c) ? T(1) : T(0)) - acc[a2][b2];
          }
        }
      }
      gfence();
      __syncthreads();
      // B: forward substitution inside the block, column c per thread, the
      // block's entries of the column in registers (rows above c are 0 and
      // stay 0, so every column runs the same unrolled triangle)
      for (int c = tid; c < re; c += WT) {
        T* Jcol = J + (int64_t)c * ld + rb;
        T y[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = r < h ? Jcol[r] : T(0);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (r < h) {
            const T* Lr = Lb + r * re + rb;
            T acc = y[r];
#pragma unroll
            for (int k = 0; k < r; ++k) acc = fma(-Lr[k], y[k], acc);
            y[r] = acc / Lr[r];
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (r < h) Jcol[r] = y[r];
      }
      gfence();
      __syncthreads();
    }
  }
  WSTAMP(6);
  // ---------------- 6: Goldfarb-Idnani -------------------------------------
  int iters = 0;
  T* Rl = sh.pan;   // R, q x q upper, stride QL (the Cholesky panel buffer is free now)
  const T mu = T(a.mu ? a.mu[b] : a.mu_default);
  const T zc = dt * dtm;   // coefficient scale of fz_j in z_k (Bd[8][2] = dt/m)
  if (xin[2] - T(kZmin) < -tol || zb[1] - T(kZmin) < -tol) status = ST_INFEAS;   // constant rows z_0, z_1
  if (status == ST_SOLVED) {
    // x = -J J' h
    for (int i = tid; i < NF; i += WT) {
      T acc = T(0.0);
      for (int k = 0; k <= i; ++k) acc = fma(J[(int64_t)k * ld + i], hv[k], acc);
      sh.vec[i] = acc;
    }
    for (int i = tid; i < 4 * NV; i += WT) isa[i] = 0;
    __syncthreads();
    rows_dot(J, ld, NF, 0, sh.vec, xv);
    gfence();
    __syncthreads();
    for (int i = tid; i < NF; i += WT) xv[i] = -xv[i];
    gfence();
    __syncthreads();
  }
  int q = 0;
  const int max_iter = 4 * NV + 50;
  bool done = status != ST_SOLVED;
  while (!done) {
    // ---- slacks of every constraint; the most violated one ----
    T best = INFINITY;
    int bid = 0x7fffffff;
    for (int v = tid; v < NV; v += WT) {
      const int j = v / 6, c = v - 6 * j;
      const bool stance = cc[j] != T(0.0);
      const T xvv = pos[v] >= 0 ? xv[pos[v]] : T(0.0);
      T s0 = INFINITY, s1 = INFINITY, s2 = INFINITY;
      if (c >= 3) {
        const T lim = T(tau_lim(c));
        s0 = xvv + lim;
        s1 = lim - xvv;
        if (c == 3 && j >= 2) {
          T z1 = T(0.0), n2 = T(0.0);
          for (int jj = 0; jj <= j - 2; ++jj) {
            if (cc[jj] == T(0.0)) continue;
            const T cz = zc * (T)(j - 1 - jj);
            z1 = fma(cz, xv[pos[6 * jj + 2]], z1);
            n2 = fma(cz, cz, n2);
          }
          const T zrow = (zb[j] - T(kZmin)) + z1;
          s2 = n2 > T(0.0) ? zrow / sqrt(n2) : ((zrow < -tol) ? -INFINITY : INFINITY);
        }
      } else if (stance && !(VAR == 2 && c == 1)) {
        const T fz = xv[pos[6 * j + 2]];
        if (c == 2) {
          s0 = fz;
          s1 = T(kFzMax) - fz;
        } else {
          const T inv = T(1.0) / sqrt(T(1.0) + mu * mu);
          s0 = (mu * fz - xvv) * inv;
          s1 = (mu * fz + xvv) * inv;
        }
      }
      if (!isa[4 * v]) argmin_combine(best, bid, s0, 4 * v);
      if (!isa[4 * v + 1]) argmin_combine(best, bid, s1, 4 * v + 1);
      if (!isa[4 * v + 2]) argmin_combine(best, bid, s2, 4 * v + 2);
    }
    block_argmin(best, bid, sh);
    if (!(best < -tol)) break;   // primal feasible: optimal
    const int p = bid;
    // n_p as (free index, coefficient) pairs and its rhs b_p
    if (tid == 0) {
      const int v = p >> 2, sl = p & 3, j = v / 6, c = v - 6 * j;
      int n = 0;
      T bp = T(0.0);
      if (c >= 3) {
        if (sl < 2) {
          sh.npi[n] = pos[v]; sh.npv[n++] = sl == 0 ? T(1.0) : -T(1.0);
          bp = -T(tau_lim(c));
        } else {
          for (int jj = 0; jj <= j - 2; ++jj)
            if (cc[jj] != T(0.0)) { sh.npi[n] = pos[6 * jj + 2]; sh.npv[n++] = zc * (T)(j - 1 - jj); }
          bp = T(kZmin) - zb[j];
        }
      } else if (c == 2) {
        sh.npi[n] = pos[v]; sh.npv[n++] = sl == 0 ? T(1.0) : -T(1.0);
        bp = sl == 0 ? T(0.0) : -T(kFzMax);
      } else {
        sh.npi[n] = pos[v]; sh.npv[n++] = sl == 0 ? -T(1.0) : T(1.0);
        sh.npi[n] = pos[6 * j + 2]; sh.npv[n++] = mu;
      }
      sh.npn = n;
      sh.bp = bp;
    }
    __syncthreads();
    const int npn = sh.npn;
    const T bp = sh.bp;
    T uplus = T(0.0);
    while (true) {
      if (++iters > max_iter) { status = ST_MAXIT; done = true; break; }
      // d = J' n_p (a combination of <= N rows of J)
      for (int i = tid; i < NF; i += WT) {
        T acc = T(0.0);
        for (int e = 0; e < npn; ++e) acc = fma(sh.npv[e], J[(int64_t)sh.npi[e] * ld + i], acc);
        sh.vec[i] = acc;
        dv[i] = acc;
      }
      __syncthreads();
      // z = J2 d2, |d2|^2, |d|^2
      rows_dot(J, ld, NF, q, sh.vec, zv);
      T zz = T(0.0), dd = T(0.0);
      for (int i = tid; i < NF; i += WT) {
        const T di = sh.vec[i];
        dd = fma(di, di, dd);
        if (i >= q) zz = fma(di, di, zz);
      }
      zz = block_sum(zz, sh);
      dd = block_sum(dd, sh);
      gfence();
      __syncthreads();
      // r = R^-1 d1, the drop candidate and n_p' x - b_p (q, n_p small: one thread)
      if (tid == 0) {
        for (int i = q - 1; i >= 0; --i) {
          T t = sh.vec[i];
          for (int k = i + 1; k < q; ++k) t = fma(-Rl[i * QL + k], rv[k], t);
          rv[i] = t / Rl[i * QL + i];
        }
        T t1 = INFINITY;
        int kd = -1;
        for (int j = 0; j < q; ++j)
          if (rv[j] > T(0.0) && ua[j] / rv[j] < t1) { t1 = ua[j] / rv[j]; kd = j; }
        T sp = -bp;
        for (int e = 0; e < npn; ++e) sp = fma(sh.npv[e], xv[sh.npi[e]], sp);
        sh.t1 = t1;
        sh.kd = kd;
        sh.sp = sp;
      }
      gfence();
      __syncthreads();
      const T t1 = sh.t1, sp = sh.sp;
      const int kd = sh.kd;
      const bool has_z = zz > tiny * dd;
      const T t2 = has_z ? -sp / zz : INFINITY;   // n_p' z = |d2|^2
      const T t = t1 < t2 ? t1 : t2;
      if (!(t < INFINITY)) { status = ST_INFEAS; done = true; break; }
      if (has_z)
        for (int i = tid; i < NF; i += WT) xv[i] = fma(t, zv[i], xv[i]);
      if (tid == 0)
        for (int j = 0; j < q; ++j) ua[j] = fma(-t, rv[j], ua[j]);
      uplus += t;
      gfence();
      __syncthreads();
      if (has_z && t == t2) {
        // ---- add p: one Householder reflection maps d2 onto alpha e_q ----
        if (q >= QL) { status = ST_NUMERICAL; done = true; break; }   // uniform
        const T dq = sh.vec[q];
        const T alpha = sqrt(zz);
        const T sg = dq >= T(0.0) ? T(1.0) : -T(1.0);
        const T beta = T(1.0) / (alpha * (alpha + fabs(dq)));   // 2 / v'v
        for (int k = q + tid; k < NF; k += WT) sh.vec2[k] = (k == q) ? dq + sg * alpha : sh.vec[k];
        __syncthreads();
        rows_dot(J, ld, NF, q, sh.vec2, wv);   // w = J2 v
        gfence();
        __syncthreads();
        // J2 <- J2 (I - beta v v'); column q flips sign when sg > 0 so that
        // the new R diagonal is +alpha
        // (a thread per column k, rows streamed: coalesced over k, independent
        // rows in flight)
        for (int k = q + tid; k < NF; k += WT) {
          const T vk = beta * sh.vec2[k];
          const bool flip = (k == q && sg > T(0));
          T* Jk = J + k;
#pragma unroll 4
          for (int i = 0; i < NF; ++i) {
            const T x = fma(-wv[i], vk, Jk[(int64_t)i * ld]);
            Jk[(int64_t)i * ld] = flip ? -x : x;
          }
        }
        for (int i = tid; i < q; i += WT) Rl[i * QL + q] = sh.vec[i];
        if (tid == 0) {
          Rl[q * QL + q] = alpha;
          act[q] = p;
          ua[q] = uplus;
          isa[p] = 1;
        }
        ++q;
        gfence();
        __syncthreads();
        break;
      }
      // ---- drop kd: delete column kd of R, restore the triangle ----
      if (tid == 0) {
        isa[act[kd]] = 0;
        for (int j = kd; j < q - 1; ++j) {
          act[j] = act[j + 1];
          ua[j] = ua[j + 1];
          for (int i = 0; i <= j + 1; ++i) Rl[i * QL + j] = Rl[i * QL + j + 1];
        }
      }
      gfence();
      __syncthreads();
      for (int j = kd; j < q - 1; ++j) {
        if (tid == 0) {
          const T aa = Rl[j * QL + j], bb = Rl[(j + 1) * QL + j];
          const T hh = sqrt(aa * aa + bb * bb);
          T c = T(1.0), s = T(0.0);
          if (hh != T(0.0)) { c = aa / hh; s = bb / hh; }
          for (int k = j; k < q - 1; ++k) {
            const T r0 = Rl[j * QL + k], r1 = Rl[(j + 1) * QL + k];
            Rl[j * QL + k] = c * r0 + s * r1;
            Rl[(j + 1) * QL + k] = -s * r0 + c * r1;
          }
          sh.gc = c;
          sh.gs = s;
        }
        gfence();
        __syncthreads();
        const T c = sh.gc, s = sh.gs;
        for (int i = tid; i < NF; i += WT) {
          T* Ji = J + (int64_t)i * ld;
          const T x0 = Ji[j], x1 = Ji[j + 1];
          Ji[j] = c * x0 + s * x1;
          Ji[j + 1] = -s * x0 + c * x1;
        }
        gfence();
        __syncthreads();
      }
      if (tid == 0)
        for (int i = 0; i < q; ++i) Rl[i * QL + q - 1] = T(0.0);
      --q;
      gfence();
      __syncthreads();
    }
  }
  WSTAMP(7);
  // ---------------- 7: outputs ---------------------------------------------
  for (int v = tid; v < NV; v += WT) {
    const T u = (status == ST_SOLVED && pos[v] >= 0) ? xv[pos[v]] : T(0.0);
    uo[v] = u;
    a.u[b * NV + v] = u;
  }
  gfence();
  __syncthreads();
  double* xo = a.x ? a.x + b * 12 * (N + 1) : nullptr;
  if (tid < 64) {
    T xrr = tid < 12 ? xin[tid] : T(0.0);
    if (xo && tid < 12) xo[tid] = xrr;
    const T qr = T(qdiag(tid));
    const int rw = (tid >= 9 && tid < 12) ? tid - 9 : 0;
    const int rvv = (tid >= 6 && tid < 9) ? tid - 6 : 0;
    T objl = T(0.0);
    for (int k = 0; k < N; ++k) {
      const T cp = cs[2 * k], sp = cs[2 * k + 1];
      const T* bwr = bw + 18 * k + 6 * rw;
      const T* uk = uo + 6 * k;
      T bw_u = T(0.0);
      for (int c = 0; c < 6; ++c) bw_u = fma(bwr[c], uk[c], bw_u);
      T bv_u;
      if constexpr (VAR == 3) {
        bv_u = dtm * uk[rvv];
      } else {   // Rz' dt/m
        const T u0 = uk[0], u1 = uk[1], u2 = uk[2];
        bv_u = (rvv == 0) ? dtm * (cp * u0 - sp * u1) : ((rvv == 1) ? dtm * (sp * u0 + cp * u1) : dtm * u2);
      }
      const T bu = (tid >= 9 && tid < 12) ? bw_u : ((tid >= 6 && tid < 9) ? bv_u : T(0.0));
      xrr = ad_lane_sel(xrr, dt, cp, sp) + bu + ((tid == 8) ? -T(a.g) * dt : T(0.0));
      const T kf = (k == N - 1) ? T(kTermQ) : T(1.0);
      const T e = xrr - (tid < 12 ? xr[12 * k + tid] : T(0.0));
      objl = fma(kf * qr * e, e, objl);
      if (k < N - 1 && tid < 6) {
        const T ubz = a.uref_aliased ? ((cc[N - 1] != T(0.0)) ? T(2.0) * T(a.m) * T(a.g) : T(0.0))
                                          : ((cc[k] != T(0.0)) ? T(2.0) * T(a.m) * T(a.g) : T(0.0));
        const T du = uk[tid] - (tid == 2 ? ubz : T(0.0));
        objl = fma(kRdiag * du, du, objl);
      }
      if (xo && tid < 12) xo[12 * (k + 1) + tid] = xrr;
    }
    const T objv = wave_sum(objl);
#ifdef HMPC_STAMPS
    WSTAMP(8);
    if (xo && tid == 0)
      for (int i = 0; i < 9; ++i) reinterpret_cast<long long*>(xo)[i] = wst[i];
#endif
    if (tid == 0) {
      if (a.obj) a.obj[b] = objv;
      a.status[b] = status;
      if (a.iters) a.iters[b] = iters;
      if (a.active) a.active[b] = q;
    }
  }
}

template <int VAR, typename T>
__global__ void __launch_bounds__(WT, 2) wide_kernel(SolveArgs a, int N) {
  __shared__ Shared<T> sh;
  T* ws = reinterpret_cast<T*>(a.ws) + (int64_t)blockIdx.x * a.ws_stride;
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    wide_solve<VAR, T>(a, N, b, ws, sh);
    gfence();
    __syncthreads();
  }
}

}  // namespace

bool launch_solve_wide(int variant, int N, const SolveArgs& a, hipStream_t s) {
  if (N < 1 || N > kWideNmax || !a.ws || a.ws_groups < 1) return false;
  if (a.B <= 0) return true;
  const int64_t g = a.B < a.ws_groups ? a.B : a.ws_groups;
  const bool f32 = a.precision == 1 || a.precision == 5;
  if (variant == 3) {
    if (f32) hipLaunchKernelGGL((wide_kernel<3, float>), dim3((unsigned)g), dim3(WT), 0, s, a, N);
    else hipLaunchKernelGGL((wide_kernel<3, double>), dim3((unsigned)g), dim3(WT), 0, s, a, N);
    return true;
  }
  if (variant == 2) {
    if (f32) hipLaunchKernelGGL((wide_kernel<2, float>), dim3((unsigned)g), dim3(WT), 0, s, a, N);
    else hipLaunchKernelGGL((wide_kernel<2, double>), dim3((unsigned)g), dim3(WT), 0, s, a, N);
    return true;
  }
  return false;
}

}  // namespace hmpc
