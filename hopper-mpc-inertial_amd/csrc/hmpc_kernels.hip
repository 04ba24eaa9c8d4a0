// hmpc_kernels.hip -- batched MPC/QP solve for MI355X (gfx950), fp64.
//
// One workgroup of W = ceil(6N/64) wavefronts solves ONE QP instance of the
// reference's Mpc.build_qp/solve_qp (src/mpc_cvx_euler_3f.py:96-160; 2f
// :96-158) to its exact optimum.  Lane v of the workgroup owns decision
// variable v = 6*k + c of the CONDENSED problem (states eliminated through
// the dynamics), i.e. row v of every NV x NV matrix lives in lane v's
// registers.  Phases (see DESIGN.md "Kernel"):
//
//   0  coalesced load of the instance's inputs into LDS
//   1  per-stage linearisation = Mpc.gen_dt_dynamics (3f :71-94, 2f :70-94)
//   2  free response  xbar_{k+1} = Ad_k xbar_k + Gd
//   3  backward Riccati-like sweep S_t = W_{t-1} + Ad_t' S_{t+1} Ad_t,
//      Y_j = S_{j+1} Bd_j
//   4  condensed Hessian rows H[v,:] and gradient h[v] (adjoint sweep)
//   5  Cholesky H = L L'   (rows in registers, one LDS column per step)
//   6  J = L^-T            (row v of J built in lane v)
//   7  unconstrained optimum v0 = -H^-1 h (two triangular sweeps)
//   8  Goldfarb-Idnani dual active set: the most violated constraint enters,
//      Householder update of J on add, Givens on drop.  Constraints: torque
//      box (:123-128), fz box + friction pyramid (:141-146), z >= 0.1
//      (:129, dense rows over fz through the dynamics); swing / 2f fy
//      equalities (:134-136, 2f :129) are eliminated as fixed variables.
//   9  outputs: u* (coalesced), x* by forward simulation, objective incl.
//      its constant term evaluated on (x*, u*), status, iterations.
//
// No MFMA: every product is a tiny dense block or a rank-1 update.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <utility>

#include "hmpc_internal.h"

namespace hmpc {

// compile-time loop: f(std::integral_constant<int, i>) for i in [Begin, End).
// Every index into a register-resident row (Jr[]) goes through this, so no
// row ever lands in scratch memory.
template <int Begin, typename F, int... Is>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Begin + Is>{}), ...);
}
template <int Begin, int End, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (End > Begin) sfor_impl<Begin>(std::make_integer_sequence<int, End - Begin>{}, f);
}
// Same, with a scheduling fence every CH iterations: keeps the scheduler from
// hoisting every LDS load of a long unrolled loop ahead of its FMAs (which
// would need ~NV extra VGPRs on top of the register-resident row).
template <int CH, int Begin, int End, typename F>
__device__ __forceinline__ void sfor_chunked(F&& f) {
  sfor<Begin, End>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    f(ic);
    if constexpr (((i - Begin) % CH) == CH - 1) __builtin_amdgcn_sched_barrier(0);
  });
}

// Empty asm that claims to read and write x: pins the value into a VGPR pair
// at this point.  Used at step boundaries of the unrolled factorisations so
// the compiler cannot sink a step's FMAs past the next step's loads (which
// doubled the live set and spilled the register-resident row to scratch).
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }
// A wave-uniform 0 the compiler cannot see through.  Added to the LDS
// address of an iteration's loads, it keeps those loads from being hoisted
// above the (volatile, hence ordered) point where it is produced -- the
// scheduler otherwise pulls every iteration's loads of a read-only LDS region
// to the top of a fully unrolled loop and spills.
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}
template <int NV>
__device__ __forceinline__ void pin_row(double (&r)[NV]) {
  sfor<0, NV>([&](auto jc) __attribute__((always_inline)) { pin(r[decltype(jc)::value]); });
}

// row[j] += alpha * x[j] for j in [Begin, End), x in LDS.  Loads are issued
// in chunks of CH behind an opaque zero, and every updated element is pinned,
// so at most CH loaded values are live beside the row.
template <int Begin, int End, int CH, int NV>
__device__ __forceinline__ void row_axpy(double (&row)[NV], double alpha, const double* x) {
  sfor<Begin, End>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    if constexpr (((j - Begin) % CH) == 0) x += opaque_zero();
    row[j] = fma(alpha, x[j], row[j]);
    pin(row[j]);
  });
}
// sum_j row[j] * x[j] for j in [Begin, End), x in LDS, chunked as above.
template <int Begin, int End, int CH, int NV>
__device__ __forceinline__ double row_dot(const double (&row)[NV], const double* x) {
  double s0 = 0.0, s1 = 0.0;
  sfor<Begin, End>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    if constexpr (((j - Begin) % CH) == 0) {
      x += opaque_zero();
      pin(s0);
      pin(s1);
    }
    if constexpr ((j & 1) == 0) s0 = fma(row[j], x[j], s0);
    else s1 = fma(row[j], x[j], s1);
  });
  return s0 + s1;
}

// ----------------------------------------------------------------------------
// constants of Mpc.__init__ / build_qp (src/mpc_cvx_euler_3f.py:20,35,37,113-129)
// ----------------------------------------------------------------------------
__device__ __forceinline__ double qdiag(int c) {   // Q = diag(50,50,2,1,1,50,1,1,1,10,10,10)
  return (c == 0 || c == 1 || c == 5) ? 50.0 : (c == 2 ? 2.0 : (c >= 9 ? 10.0 : 1.0));
}
constexpr double kRdiag = 0.001;   // R = 0.001 I
constexpr double kTermQ = 100.0;   // kf at k = N-1
constexpr double kFzMax = 206.0;   // f_max[2]
constexpr double kZmin = 0.1;
constexpr double kTol = 1e-10;     // scaled primal feasibility tolerance
__device__ __forceinline__ double tau_lim(int c) { return c == 5 ? 4.0 : 7.78; }

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

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

__device__ __forceinline__ void argmin_combine(double& v, int& i, double v2, int i2) {
  if (v2 < v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

__device__ __forceinline__ void wave_argmin(double& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double v2 = __shfl_xor(v, o, 64);
    int i2 = __shfl_xor(i, o, 64);
    argmin_combine(v, i, v2, i2);
  }
}

template <int W>
struct Blk {
  // `red` must hold >= 2*W doubles; every call is bracketed by barriers so
  // consecutive calls may reuse it.
  __device__ static double sum(double x, double* red) {
    x = wave_sum(x);
    if constexpr (W == 1) {
      return x;
    } else {
      __syncthreads();
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
      __syncthreads();
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < W; ++w) s += red[w];
      return s;
    }
  }
  __device__ static void argmin(double& v, int& i, double* red) {
    wave_argmin(v, i);
    if constexpr (W > 1) {
      __syncthreads();
      if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = v;
        reinterpret_cast<int*>(red + W)[threadIdx.x >> 6] = i;
      }
      __syncthreads();
      v = red[0];
      i = reinterpret_cast<int*>(red + W)[0];
#pragma unroll
      for (int w = 1; w < W; ++w) argmin_combine(v, i, red[w], reinterpret_cast<int*>(red + W)[w]);
    }
  }
  // value of x in lane l (l uniform)
  __device__ static double bcast(double x, int l, double* red) {
    if constexpr (W == 1) {
      return rdlane(x, l);
    } else {
      __syncthreads();
      if ((int)threadIdx.x == l) red[0] = x;
      __syncthreads();
      return red[0];
    }
  }
  // rank of this lane among lanes with flag set, and the total count
  __device__ static void rank(bool flag, int& r, int& cnt, double* red) {
    unsigned long long m = __ballot(flag);
    int lane = threadIdx.x & 63;
    r = __popcll(m & ((1ull << lane) - 1ull));
    cnt = __popcll(m);
    if constexpr (W > 1) {
      int* ired = reinterpret_cast<int*>(red);
      __syncthreads();
      if (lane == 0) ired[threadIdx.x >> 6] = cnt;
      __syncthreads();
      int off = 0, tot = 0;
      int me = threadIdx.x >> 6;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        int c = ired[w];
        if (w < me) off += c;
        tot += c;
      }
      r += off;
      cnt = tot;
    }
  }
};

// ----------------------------------------------------------------------------
// LDS layout (in doubles), one instance per workgroup
// ----------------------------------------------------------------------------
template <int N>
struct Lay {
  static constexpr int NV = 6 * N;
  static constexpr int W = (NV + 63) / 64;
  static constexpr int NT = 64 * W;
  static constexpr int NSLOT = 4;
  static constexpr int e2(int n) { return (n + 1) & ~1; }
  // persistent
  static constexpr int XIN = 0;
  static constexpr int CC = XIN + 12;
  static constexpr int CS = CC + e2(N);
  static constexpr int BD = CS + 2 * N;           // rows 6..11 of Bd_k: [k][a][col] 6x6
  static constexpr int XBAR = BD + 36 * N;         // [(N+1)][12]
  static constexpr int DZ = XBAR + 12 * (N + 1);   // [NT]
  static constexpr int XS = DZ + NT;               // [NT]
  static constexpr int RED = XS + NT;              // [16]
  static constexpr int UA = RED + 16;              // [NV] multipliers of active constraints
  static constexpr int RV = UA + NV;               // [NV]
  static constexpr int ACT = RV + NV;              // [NV] (int storage)
  static constexpr int SD = ACT + NV;              // [NV] subdiagonal scratch for drops
  static constexpr int U0 = SD + NV;               // start of the union
  // union A (phases 0-4)
  static constexpr int XLIN = U0;                  // [(N+1)][12]
  static constexpr int XREF = XLIN + 12 * (N + 1); // [N][12]
  static constexpr int PF = XREF + 12 * N;         // [N][3]
  static constexpr int SB = PF + e2(3 * N);        // [2][144]
  static constexpr int YY = SB + 288;              // [N][12][6]
  static constexpr int ADJ = YY + 72 * N;          // [(N+1)][12]
  static constexpr int ENDA = ADJ + 12 * (N + 1);
  // union B (phases 5-9)
  static constexpr int LP = U0;                    // packed lower L, row r at r(r+1)/2; later R
  static constexpr int LPS = e2(NV * (NV + 1) / 2 + NT);
  static constexpr int INVD = LP + LPS;            // [NV]
  static constexpr int COL = INVD + e2(NV);        // [2][NT]   (also final x* staging)
  static constexpr int SLOT = COL + 2 * NT;        // [NSLOT][NV]
  static constexpr int ENDB = SLOT + (NSLOT + 1) * NV;   // + one pad row
  static constexpr int XOUT = COL;                 // [(N+1)][12] <= 2*NT + NSLOT*NV
  static constexpr int TOTAL = ENDA > ENDB ? ENDA : ENDB;
  static_assert(12 * (N + 1) <= 2 * NT + NSLOT * NV, "x* staging does not fit");
};

__device__ __forceinline__ int loff(int r) { return (r * (r + 1)) >> 1; }

// ----------------------------------------------------------------------------
// the kernel
// ----------------------------------------------------------------------------
#ifndef HMPC_WAVES_PER_EU
#define HMPC_WAVES_PER_EU(W) ((W) == 1 ? 2 : 1)
#endif
template <int VAR, int N>
__global__ void __launch_bounds__(Lay<N>::NT, HMPC_WAVES_PER_EU(Lay<N>::W))
solve_kernel(SolveArgs a) {
  using L = Lay<N>;
  constexpr int NV = L::NV;
  constexpr int W = L::W;
  constexpr int NT = L::NT;
  using B = Blk<W>;
  __shared__ double sm[L::TOTAL];
  double* red = sm + L::RED;

  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x;
  const double dt = a.dt;
  const double mu = a.mu ? a.mu[b] : a.mu_default;

  // ---------------- phase 0: coalesced loads --------------------------------
  for (int i = tid; i < 12; i += NT) sm[L::XIN + i] = a.x_in[b * 12 + i];
  for (int i = tid; i < 12 * N; i += NT) sm[L::XREF + i] = a.x_ref[b * 12 * N + i];
  for (int i = tid; i < 3 * N; i += NT) sm[L::PF + i] = a.pf[b * 3 * N + i];
  for (int i = tid; i < N; i += NT) sm[L::CC + i] = a.C[b * N + i];
  if (a.shift_mode == 0) {
    for (int i = tid; i < 12 * (N + 1); i += NT) sm[L::XLIN + i] = a.x_lin[b * 12 * (N + 1) + i];
  } else if (a.shift_mode == 1) {   // [x_in; x_ref]          (3f :52-53)
    for (int i = tid; i < 12 * (N + 1); i += NT)
      sm[L::XLIN + i] = i < 12 ? a.x_in[b * 12 + i] : a.x_ref[b * 12 * N + i - 12];
  } else {                          // [x_in; x_prev[2:]; x_prev[N]]  (3f :59-62)
    const double* xp = a.x_lin + b * 12 * (N + 1);
    for (int i = tid; i < 12 * (N + 1); i += NT) {
      int r = i / 12, c = i - 12 * r;
      double v;
      if (r == 0) v = a.x_in[b * 12 + c];
      else if (r < N) v = xp[(r + 1) * 12 + c];
      else v = xp[N * 12 + c];
      sm[L::XLIN + i] = v;
    }
  }
  __syncthreads();

  // ---------------- phase 1: gen_dt_dynamics (lane k < N) -------------------
  if (tid < N) {
    const int k = tid;
    const double psi = sm[L::XLIN + 12 * k + 5];
    double sp, cp;
    sincos(psi, &sp, &cp);
    // rz(psi) = [[c, s, 0], [-s, c, 0], [0, 0, 1]]   (src/utils.py:46-51)
    const double Rz[3][3] = {{cp, sp, 0.0}, {-sp, cp, 0.0}, {0.0, 0.0, 1.0}};
    double d[3], rf[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] = sm[L::PF + 3 * k + i] - sm[L::XLIN + 12 * k + i];
#pragma unroll
    for (int i = 0; i < 3; ++i) rf[i] = a.rh[i] + (Rz[i][0] * d[0] + Rz[i][1] * d[1] + Rz[i][2] * d[2]);
    double T[3][3], Jw[3][3], RzT[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) RzT[i][j] = Rz[j][i];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        T[i][j] = Rz[i][0] * a.Jinv[0 * 3 + j] + Rz[i][1] * a.Jinv[1 * 3 + j] + Rz[i][2] * a.Jinv[2 * 3 + j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Jw[i][j] = T[i][0] * RzT[0][j] + T[i][1] * RzT[1][j] + T[i][2] * RzT[2][j];
    double Bwt[3][3], Bwf[3][3], Bvf[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Bwt[i][j] = Jw[i][0] * RzT[0][j] + Jw[i][1] * RzT[1][j] + Jw[i][2] * RzT[2][j];
    double w[3];
    if constexpr (VAR == 3) {   // rhat = hat(Rz' rf); B[9:12,0:3] = Jw rhat; B[6:9,0:3] = I/m
#pragma unroll
      for (int i = 0; i < 3; ++i) w[i] = RzT[i][0] * rf[0] + RzT[i][1] * rf[1] + RzT[i][2] * rf[2];
    } else {                    // rhat = hat(rf); B[9:12,0:3] = (Jw Rz') rhat; B[6:9,0:3] = Rz'/m
#pragma unroll
      for (int i = 0; i < 3; ++i) w[i] = rf[i];
    }
    const double hw[3][3] = {{0.0, -w[2], w[1]}, {w[2], 0.0, -w[0]}, {-w[1], w[0], 0.0}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if constexpr (VAR == 3)
          Bwf[i][j] = Jw[i][0] * hw[0][j] + Jw[i][1] * hw[1][j] + Jw[i][2] * hw[2][j];
        else
          Bwf[i][j] = Bwt[i][0] * hw[0][j] + Bwt[i][1] * hw[1][j] + Bwt[i][2] * hw[2][j];
      }
    const double im = 1.0 / a.m;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Bvf[i][j] = (VAR == 3) ? (i == j ? im : 0.0) : RzT[i][j] / a.m;
    double* bd = sm + L::BD + 36 * k;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        bd[i * 6 + j] = Bvf[i][j] * dt;
        bd[i * 6 + 3 + j] = 0.0;
        bd[(3 + i) * 6 + j] = Bwf[i][j] * dt;
        bd[(3 + i) * 6 + 3 + j] = Bwt[i][j] * dt;
      }
    sm[L::CS + 2 * k] = cp;
    sm[L::CS + 2 * k + 1] = sp;
  }
  __syncthreads();

  // ---------------- phase 2: free response (lanes 0..11 of wave 0) ----------
  {
    double xv = tid < 12 ? sm[L::XIN + tid] : 0.0;
    if (tid < 12) sm[L::XBAR + tid] = xv;
    for (int k = 0; k < N; ++k) {
      const double cp = sm[L::CS + 2 * k], sp = sm[L::CS + 2 * k + 1];
      const double vsrc = __shfl(xv, (tid + 6) & 63, 64);
      const double w0 = __shfl(xv, 9, 64), w1 = __shfl(xv, 10, 64), w2 = __shfl(xv, 11, 64);
      double nx = xv;
      if (tid < 3) nx = xv + dt * vsrc;
      else if (tid == 3) nx = xv + ((cp * dt) * w0 + (sp * dt) * w1);
      else if (tid == 4) nx = xv + ((-sp * dt) * w0 + (cp * dt) * w1);
      else if (tid == 5) nx = xv + dt * w2;
      else if (tid == 8) nx = xv + (-a.g * dt);
      xv = nx;
      if (tid < 12) sm[L::XBAR + 12 * (k + 1) + tid] = xv;
    }
  }
  // (XBAR is consumed after the next barrier)

  // ---------------- phase 3: S sweep, Y_j = S_{j+1} Bd_j --------------------
  {
    // S_N = W_{N-1} = kTermQ * Q
    for (int e = tid; e < 144; e += NT) {
      int r = e / 12, c = e - 12 * r;
      sm[L::SB + e] = (r == c) ? kTermQ * qdiag(r) : 0.0;
    }
    __syncthreads();
    int cur = 0;
    for (int t = N; t >= 1; --t) {
      const double* S = sm + L::SB + 144 * cur;
      // Y_{t-1} = S_t[:, 6:12] * Bd_{t-1}
      const double* bd = sm + L::BD + 36 * (t - 1);
      double* Y = sm + L::YY + 72 * (t - 1);
      for (int e = tid; e < 72; e += NT) {
        int r = e / 6, c = e - 6 * r;
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 6; ++q) acc += S[12 * r + 6 + q] * bd[6 * q + c];
        Y[e] = acc;
      }
      if (t > 1) {
        // S_{t-1} = W_{t-2} + Ad_{t-1}' S_t Ad_{t-1}
        const int ti = t - 1;
        const double cp = sm[L::CS + 2 * ti], sp = sm[L::CS + 2 * ti + 1];
        double* Sn = sm + L::SB + 144 * (cur ^ 1);
        for (int e = tid; e < 144; e += NT) {
          int r = e / 12, c = e - 12 * r;
          // column r of Ad = e_r + dt*A[:,r] has at most 3 nonzeros:
          // (r, 1), and (ra1, ca1), (ra2, ca2) with a zero coefficient when absent
          int ra1 = 0, ra2 = 0, rb1 = 0, rb2 = 0;
          double ca1 = 0.0, ca2 = 0.0, cb1 = 0.0, cb2 = 0.0;
          if (r >= 6 && r < 9) { ra1 = r - 6; ca1 = dt; }
          if (r == 9) { ra1 = 3; ca1 = cp * dt; ra2 = 4; ca2 = -sp * dt; }
          if (r == 10) { ra1 = 3; ca1 = sp * dt; ra2 = 4; ca2 = cp * dt; }
          if (r == 11) { ra1 = 5; ca1 = dt; }
          if (c >= 6 && c < 9) { rb1 = c - 6; cb1 = dt; }
          if (c == 9) { rb1 = 3; cb1 = cp * dt; rb2 = 4; cb2 = -sp * dt; }
          if (c == 10) { rb1 = 3; cb1 = sp * dt; rb2 = 4; cb2 = cp * dt; }
          if (c == 11) { rb1 = 5; cb1 = dt; }
          auto row = [&](int ra) {
            return S[12 * ra + c] + cb1 * S[12 * ra + rb1] + cb2 * S[12 * ra + rb2];
          };
          double acc = row(r) + ca1 * row(ra1) + ca2 * row(ra2);
          if (r == c) acc += qdiag(r);   // W_{t-2}, kf = 1 for t-2 < N-1
          Sn[e] = acc;
        }
        cur ^= 1;
      }
      __syncthreads();
    }
  }

  // ---------------- phase 4a: adjoint sweep (lanes 0..11) -------------------
  // a_N = W_{N-1}(xbar_N - r_{N-1}); a_t = W_{t-1}(xbar_t - r_{t-1}) + Ad_t' a_{t+1}
  {
    double av = 0.0;
    if (tid < 12)
      av = kTermQ * qdiag(tid) * (sm[L::XBAR + 12 * N + tid] - sm[L::XREF + 12 * (N - 1) + tid]);
    if (tid < 12) sm[L::ADJ + 12 * N + tid] = av;
    for (int t = N - 1; t >= 1; --t) {
      const double cp = sm[L::CS + 2 * t], sp = sm[L::CS + 2 * t + 1];
      const double s0 = __shfl(av, (tid + 58) & 63, 64);   // a[tid-6]
      const double a3 = __shfl(av, 3, 64), a4 = __shfl(av, 4, 64), a5 = __shfl(av, 5, 64);
      double at = av;
      if (tid >= 6 && tid < 9) at = av + dt * s0;
      else if (tid == 9) at = av + ((cp * dt) * a3 + (-sp * dt) * a4);
      else if (tid == 10) at = av + ((sp * dt) * a3 + (cp * dt) * a4);
      else if (tid == 11) at = av + dt * a5;
      if (tid < 12) at += qdiag(tid) * (sm[L::XBAR + 12 * t + tid] - sm[L::XREF + 12 * (t - 1) + tid]);
      av = at;
      if (tid < 12) sm[L::ADJ + 12 * t + tid] = av;
    }
  }
  __syncthreads();

  // ---------------- phase 4b: condensed Hessian rows + gradient -------------
  const int vj = tid / 6, vc = tid - 6 * (tid / 6);   // stage / component of my variable
  const bool active_lane = tid < NV;
  const double ubar_z_alias = (sm[L::CC + N - 1] != 0.0) ? 2.0 * a.m * a.g : 0.0;
  auto is_fixed = [&](int k, int c) -> bool {   // swing f = 0 (:134-136), 2f fy = 0 (2f :129)
    return (c < 3 && sm[L::CC + k] == 0.0) || (VAR == 2 && c == 1);
  };
  const bool my_fixed = active_lane && is_fixed(vj, vc);

  double Jr[NV];   // row `tid` of H, then L, then J
  double hv = 0.0;
  {
    double Z[12];
#pragma unroll
    for (int r = 0; r < 12; ++r) Z[r] = 0.0;
    sfor<0, N>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = N - 1 - decltype(ic)::value;
      if (i < N - 1) {   // Z <- Ad_{i+1}' Z for lanes with j > i
        const double cp = sm[L::CS + 2 * (i + 1)], sp = sm[L::CS + 2 * (i + 1) + 1];
        double Zn[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) Zn[r] = Z[r];
#pragma unroll
        for (int r = 6; r < 9; ++r) Zn[r] = Z[r] + dt * Z[r - 6];
        Zn[9] = Z[9] + ((cp * dt) * Z[3] + (-sp * dt) * Z[4]);
        Zn[10] = Z[10] + ((sp * dt) * Z[3] + (cp * dt) * Z[4]);
        Zn[11] = Z[11] + dt * Z[5];
        const bool upd = vj > i;
#pragma unroll
        for (int r = 0; r < 12; ++r) Z[r] = upd ? Zn[r] : Z[r];
      }
      {
        const int oz = opaque_zero();
        const bool ld = (vj == i) && active_lane;
        const double* Y = sm + L::YY + 72 * i + oz;
        const int cc = active_lane ? vc : 0;
        double yv[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) yv[r] = Y[6 * r + cc];   // unconditional gather
        pin_row(yv);
#pragma unroll
        for (int r = 0; r < 12; ++r) Z[r] = ld ? yv[r] : Z[r];
      }
      const int oz2 = opaque_zero();
      const double* bd = sm + L::BD + 36 * i + oz2;
      const bool row_ok = active_lane && vj >= i && !my_fixed;
      sfor<0, 6>([&](auto cc2) __attribute__((always_inline)) {
        constexpr int c2 = decltype(cc2)::value;
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 6; ++q) acc += bd[6 * q + c2] * Z[6 + q];
        acc *= 2.0;
        if (vj == i && vc == c2) acc += (i == N - 1) ? 0.0 : 2.0 * kRdiag;
        const bool colfix = is_fixed(i, c2);
        double val = (row_ok && !colfix) ? acc : 0.0;
        if (my_fixed && vj == i && vc == c2) val = 1.0;
        Jr[6 * i + c2] = val;
        pin(Jr[6 * i + c2]);
      });
      pin_row(Z);
    });
    // gradient h_v = 2 Bd_j' a_{j+1} - 2 V_j ubar_j
    if (active_lane && !my_fixed) {
      const double* bd = sm + L::BD + 36 * vj;
      const double* ad = sm + L::ADJ + 12 * (vj + 1);
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < 6; ++q) acc += bd[6 * q + vc] * ad[6 + q];
      double ub = 0.0;
      if (vc == 2) ub = a.uref_aliased ? ubar_z_alias : ((sm[L::CC + vj] != 0.0) ? 2.0 * a.m * a.g : 0.0);
      const double Vj = (vj == N - 1) ? 0.0 : kRdiag;
      hv = 2.0 * acc - 2.0 * Vj * ub;
    }
  }
  __syncthreads();   // union A (XLIN/XREF/PF/S/Y/ADJ) is dead from here on

  int status = ST_SOLVED;

  // ---------------- phase 5: Cholesky (right-looking, one column per step) --
  {
    double* Lp = sm + L::LP;
    double* invd = sm + L::INVD;
    sfor<0, NV>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      double* col = sm + L::COL + (k & 1) * NT;
      col[tid] = Jr[k];
      __syncthreads();
      col += opaque_zero();
      const double piv = col[k];
      const double sq = sqrt(piv > 0.0 ? piv : 1.0);
      if (!(piv > 0.0)) status = ST_NUMERICAL;
      const double rs = 1.0 / sq;
      const double tk = Jr[k] * (rs * rs);
      row_axpy<k + 1, NV, 8>(Jr, -tk, col);
      const double lik = Jr[k] * rs;
      Jr[k] = lik;
      const bool wr = tid >= k && tid < NV;
      Lp[wr ? loff(tid) + k : L::LPS - NT + tid] = lik;   // branch-free (pad slots)
      if (tid == k) invd[k] = rs;
      pin_row(Jr);
    });
    __syncthreads();
  }

  // ---------------- phase 7 (first): v0 = -L^-T L^-1 h -----------------------
  double v = 0.0;
  {
    const double* Lp = sm + L::LP;
    const double* invd = sm + L::INVD;
    double acc = hv, yv = 0.0;
    for (int s = 0; s < NV; ++s) {
      const double ys = B::bcast(acc, s, red) * invd[s];
      const int cidx = tid > s ? tid : s;   // keep the address inside the array
      const double lis = Lp[loff(cidx < NV ? cidx : NV - 1) + s];
      if (tid > s) acc = fma(-lis, ys, acc);
      if (tid == s) yv = ys;
    }
    acc = yv;
    for (int s = NV - 1; s >= 0; --s) {
      const double vs = B::bcast(acc, s, red) * invd[s];
      const double lsi = Lp[loff(s) + (tid < s ? tid : 0)];
      if (tid < s) acc = fma(-lsi, vs, acc);
      if (tid == s) v = -vs;
    }
  }

  // ---------------- phase 6: J = L^-T, row `tid` of J in registers ----------
  {
    const double* Lp = sm + L::LP;
    const double* invd = sm + L::INVD;
    sfor<0, NV>([&](auto rc) __attribute__((always_inline)) {
      constexpr int r = decltype(rc)::value;
      double acc0 = (tid == r) ? 1.0 : 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
      const double* Lr = Lp + loff(r) + opaque_zero();
      sfor<0, r / 4>([&](auto sc) __attribute__((always_inline)) {
        constexpr int s = 4 * decltype(sc)::value;
        if constexpr ((s % 8) == 0) {
          Lr += opaque_zero();
          pin(acc0); pin(acc1); pin(acc2); pin(acc3);
        }
        acc0 = fma(-Lr[s], Jr[s], acc0);
        acc1 = fma(-Lr[s + 1], Jr[s + 1], acc1);
        acc2 = fma(-Lr[s + 2], Jr[s + 2], acc2);
        acc3 = fma(-Lr[s + 3], Jr[s + 3], acc3);
      });
      sfor<(r / 4) * 4, r>([&](auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        acc0 = fma(-Lr[s], Jr[s], acc0);
      });
      Jr[r] = ((acc0 + acc1) + (acc2 + acc3)) * invd[r];
      pin(Jr[r]);
    });
  }
  __syncthreads();   // L is dead: its LDS becomes R

  // ---------------- phase 8: Goldfarb-Idnani dual active set ----------------
  // Constraints owned by lane v (id = 4 v + slot), all as n'v >= b:
  //   c in 3..5 : slot0  v >= -lim,  slot1 -v >= -lim          (:123-128)
  //   c == 3    : slot2  z_k >= 0.1, k = stage, 2 <= k <= N-1  (:129)
  //   c == 2    : slot0  fz >= 0,    slot1 -fz >= -206          (:145-146)
  //   c in 0..1 : slot0 -f + mu fz >= 0, slot1 f + mu fz >= 0   (:141-144)
  //   (stance only for c <= 2; 2f has no fy rows)
  int iters = 0;
  const double zmin_gap_k0 = sm[L::XIN + 2] - kZmin;       // z_0 row: constant
  const double zmin_gap_k1 = sm[L::XBAR + 12 + 2] - kZmin;  // z_1 row: constant
  if (zmin_gap_k0 < -kTol || zmin_gap_k1 < -kTol) status = ST_INFEAS;

  // my constraint slots: number, and the z-row norm for lanes (k,3)
  const bool stance_me = active_lane && vc <= 2 && sm[L::CC + vj] != 0.0;
  int nslots = 0;
  if (active_lane) {
    if (vc >= 3) nslots = (vc == 3 && vj >= 2) ? 3 : 2;
    else if (stance_me && !(VAR == 2 && vc == 1)) nslots = 2;
  }
  double znorm = 0.0;
  if (active_lane && vc == 3 && vj >= 2) {
    double s2 = 0.0;
    for (int j = 0; j <= vj - 2; ++j) {
      if (sm[L::CC + j] != 0.0) {
        double cz = dt * sm[L::BD + 36 * j + 2 * 6 + 2] * (double)(vj - 1 - j);
        s2 += cz * cz;
      }
    }
    znorm = sqrt(s2);
  }
  const double fric_norm = sqrt(1.0 + mu * mu);
  int actmask = 0;

  double* Rm = sm + L::LP;   // packed upper, column k at loff(k)
  double* ua = sm + L::UA;
  double* rv = sm + L::RV;
  int* act = reinterpret_cast<int*>(sm + L::ACT);
  double* dz = sm + L::DZ;
  double* xs = sm + L::XS;
  double* slot = sm + L::SLOT;
  double* sdg = sm + L::SD;
  int q = 0;
  const int max_iter = 4 * NV + 50;

  // coefficient of lane `i`'s variable in constraint `id`, and its rhs
  auto coef_of = [&](int id, int i) -> double {
    const int o = id >> 2, sl = id & 3, oj = o / 6, oc = o - 6 * oj;
    if (i >= NV) return 0.0;
    if (oc >= 3) {
      if (sl == 0) return i == o ? 1.0 : 0.0;
      if (sl == 1) return i == o ? -1.0 : 0.0;
      // z-row of stage oj over fz_j, j <= oj-2
      const int ij = i / 6, ic = i - 6 * ij;
      if (ic != 2 || ij > oj - 2 || sm[L::CC + ij] == 0.0) return 0.0;
      return dt * sm[L::BD + 36 * ij + 2 * 6 + 2] * (double)(oj - 1 - ij);
    }
    if (oc == 2) return i == o ? (sl == 0 ? 1.0 : -1.0) : 0.0;
    if (i == o) return sl == 0 ? -1.0 : 1.0;
    if (i == 6 * oj + 2) return mu;
    return 0.0;
  };
  auto rhs_of = [&](int id) -> double {
    const int o = id >> 2, sl = id & 3, oj = o / 6, oc = o - 6 * oj;
    if (oc >= 3) {
      if (sl < 2) return -tau_lim(oc);
      return kZmin - sm[L::XBAR + 12 * oj + 2];
    }
    if (oc == 2) return sl == 0 ? 0.0 : -kFzMax;
    return 0.0;
  };

  bool done = status != ST_SOLVED;
  while (!done) {
    // ---- slacks of my constraints; pick the most violated ----
    xs[tid] = v;
    __syncthreads();
    double best = INFINITY;
    int bid = 0x7fffffff;
    for (int sl = 0; sl < nslots; ++sl) {
      if (actmask & (1 << sl)) continue;
      double s, nrm;
      if (vc >= 3) {
        if (sl < 2) {
          s = (sl == 0 ? v : -v) + tau_lim(vc);
          nrm = 1.0;
        } else {
          double z = sm[L::XBAR + 12 * vj + 2];
          for (int j = 0; j <= vj - 2; ++j)
            if (sm[L::CC + j] != 0.0)
              z += dt * sm[L::BD + 36 * j + 14] * (double)(vj - 1 - j) * xs[6 * j + 2];
          s = z - kZmin;
          nrm = znorm;
        }
      } else if (vc == 2) {
        s = sl == 0 ? v : kFzMax - v;
        nrm = 1.0;
      } else {
        const double fz = xs[6 * vj + 2];
        s = (sl == 0 ? -v : v) + mu * fz;
        nrm = fric_norm;
      }
      double sc;
      if (nrm > 0.0) sc = s / nrm;
      else sc = (s < -kTol) ? -INFINITY : INFINITY;
      argmin_combine(best, bid, sc, 4 * tid + sl);
    }
    B::argmin(best, bid, red);
    if (!(best < -kTol)) break;   // primal feasible: optimal
    const int p = bid;
    const double bp = rhs_of(p);
    const double np_me = coef_of(p, tid);
    double u_plus = 0.0;

    // ---- inner loop: step towards satisfying constraint p ----
    while (true) {
      if (++iters > max_iter) { status = ST_MAXIT; done = true; break; }
      // d = J' n_p  (lane j gets d_j) through NSLOT row slots
      int rk, cnt;
      const bool nzf = np_me != 0.0;
      B::rank(nzf, rk, cnt, red);
      double dj = 0.0;
      for (int base = 0; base < cnt; base += L::NSLOT) {
        {
          // branch-free: lanes without a slot write into the pad row
          const bool mine = nzf && rk >= base && rk < base + L::NSLOT;
          double* sr = slot + (mine ? (rk - base) * NV : L::NSLOT * NV);
          sfor<0, NV>([&](auto jc) __attribute__((always_inline)) {
            constexpr int j = decltype(jc)::value;
            double prod = np_me * Jr[j];
            pin(prod);
            sr[j] = prod;
          });
        }
        __syncthreads();
        const int ns = (cnt - base) < L::NSLOT ? (cnt - base) : L::NSLOT;
        if (tid < NV)
          for (int s = 0; s < ns; ++s) dj += slot[s * NV + tid];
        __syncthreads();
      }
      // z = J_2 d_2, |d_2|^2
      const bool in2 = tid >= q && tid < NV;
      dz[tid] = in2 ? dj : 0.0;
      const double zn = B::sum(in2 ? dj * dj : 0.0, red);
      __syncthreads();
      double zi = 0.0;
      {
        zi = row_dot<0, NV, 8>(Jr, dz);
      }
      // r = R^-1 d_1 (lanes l < q), back substitution
      double rcur = tid < q ? dj : 0.0, rmine = 0.0;
      for (int l = q - 1; l >= 0; --l) {
        const double rl = B::bcast(rcur, l, red) / Rm[loff(l) + l];
        if (tid == l) rmine = rl;
        if (tid < l) rcur = fma(-Rm[loff(l) + tid], rl, rcur);
      }
      // partial step length t1 (drop candidate)
      double t1 = INFINITY;
      int kdrop = 0x7fffffff;
      if (tid < q && rmine > 0.0) { t1 = ua[tid] / rmine; kdrop = tid; }
      B::argmin(t1, kdrop, red);
      // full step length t2
      const double sp_ = B::sum(np_me * v, red) - bp;
      const bool has_z = zn > 1e-30;
      const double t2 = has_z ? -sp_ / zn : INFINITY;
      const double t = t1 < t2 ? t1 : t2;
      if (!(t < INFINITY)) { status = ST_INFEAS; done = true; break; }
      if (has_z) v = fma(t, zi, v);
      if (tid < q) ua[tid] -= t * rmine;
      u_plus += t;
      __syncthreads();
      if (has_z && t == t2) {
        // ---- add p: Householder reflection on d_2 ----
        const double dq = B::bcast(dj, q, red);
        const double nrm = sqrt(zn);
        const double alpha = dq > 0.0 ? -nrm : nrm;
        const double ww = (zn - dq * dq) + (dq - alpha) * (dq - alpha);
        dz[tid] = in2 ? (tid == q ? dj - alpha : dj) : 0.0;
        if (tid < q) Rm[loff(q) + tid] = dj;
        if (tid == q) Rm[loff(q) + q] = alpha;
        if (tid == 0) { act[q] = p; ua[q] = u_plus; }
        if (tid == (p >> 2)) actmask |= 1 << (p & 3);
        __syncthreads();
        if (ww > 0.0) {
          const double f = row_dot<0, NV, 8>(Jr, dz) * (2.0 / ww);
          row_axpy<0, NV, 8>(Jr, -f, dz);
        }
        ++q;
        __syncthreads();
        break;
      }
      // ---- drop active constraint kdrop ----
      {
        const int k = kdrop;
        const int idk = act[k];
        if (tid == (idk >> 2)) actmask &= ~(1 << (idk & 3));
        // shift R columns k+1..q-1 left; remember the subdiagonals
        for (int m = k; m + 1 < q; ++m) {
          double val = 0.0;
          if (tid <= m + 1) val = Rm[loff(m + 1) + tid];
          __syncthreads();
          if (tid <= m) Rm[loff(m) + tid] = val;
          if (tid == m + 1) sdg[m] = val;
          __syncthreads();
        }
        // shift the active list and multipliers
        {
          int an = 0;
          double un = 0.0;
          if (tid >= k && tid + 1 < q) { an = act[tid + 1]; un = ua[tid + 1]; }
          __syncthreads();
          if (tid >= k && tid + 1 < q) { act[tid] = an; ua[tid] = un; }
          __syncthreads();
        }
        // Givens to restore the triangle: rows (l, l+1), l = k..q-2
        for (int l = k; l + 1 < q; ++l) {
          const double aa = Rm[loff(l) + l], bb = sdg[l];
          const double hh = sqrt(aa * aa + bb * bb);
          const double cg = aa / hh, sg = bb / hh;
          __syncthreads();
          if (tid == l) Rm[loff(l) + l] = hh;
          const int mcol = tid;   // columns m > l hold rows l, l+1
          if (mcol > l && mcol + 1 < q) {
            const double rl = Rm[loff(mcol) + l], rl1 = Rm[loff(mcol) + l + 1];
            Rm[loff(mcol) + l] = cg * rl + sg * rl1;
            Rm[loff(mcol) + l + 1] = -sg * rl + cg * rl1;
          }
          sfor<0, NV - 1>([&](auto jc) __attribute__((always_inline)) {
            constexpr int jj = decltype(jc)::value;
            if (jj == l) {
              const double x0 = Jr[jj], x1 = Jr[jj + 1];
              Jr[jj] = cg * x0 + sg * x1;
              Jr[jj + 1] = -sg * x0 + cg * x1;
            }
          });
          pin_row(Jr);
          __syncthreads();
        }
        --q;
        __syncthreads();
      }
    }
  }

  // ---------------- phase 9: outputs ----------------------------------------
  if (active_lane) a.u[b * NV + tid] = v;
  xs[tid] = v;
  __syncthreads();
  {
    double* xo = sm + L::XOUT;
    double xv = tid < 12 ? sm[L::XIN + tid] : 0.0;
    if (tid < 12) xo[tid] = xv;
    double objp = 0.0;
    const double* xr = a.x_ref + b * 12 * N;
    for (int k = 0; k < N; ++k) {
      const double cp = sm[L::CS + 2 * k], sp = sm[L::CS + 2 * k + 1];
      const double vsrc = __shfl(xv, (tid + 6) & 63, 64);
      const double w0 = __shfl(xv, 9, 64), w1 = __shfl(xv, 10, 64), w2 = __shfl(xv, 11, 64);
      double nx = xv;
      if (tid < 3) nx = xv + dt * vsrc;
      else if (tid == 3) nx = xv + ((cp * dt) * w0 + (sp * dt) * w1);
      else if (tid == 4) nx = xv + ((-sp * dt) * w0 + (cp * dt) * w1);
      else if (tid == 5) nx = xv + dt * w2;
      else if (tid >= 6 && tid < 12) {
        const double* bd = sm + L::BD + 36 * k + 6 * (tid - 6);
        double bu = 0.0;
#pragma unroll
        for (int c = 0; c < 6; ++c) bu += bd[c] * xs[6 * k + c];
        nx = xv + bu;
        if (tid == 8) nx += -a.g * dt;
      }
      xv = nx;
      if (tid < 12) {
        xo[12 * (k + 1) + tid] = xv;
        const double e = xv - xr[12 * k + tid];
        objp += (k == N - 1 ? kTermQ : 1.0) * qdiag(tid) * e * e;
      }
      if (tid < 6 && k < N - 1) {
        double ub = 0.0;
        if (tid == 2) ub = a.uref_aliased ? ubar_z_alias : ((sm[L::CC + k] != 0.0) ? 2.0 * a.m * a.g : 0.0);
        const double du = xs[6 * k + tid] - ub;
        objp += kRdiag * du * du;
      }
    }
    const double objv = B::sum(objp, red);
    __syncthreads();
    if (a.x)
      for (int i = tid; i < 12 * (N + 1); i += NT) a.x[b * 12 * (N + 1) + i] = xo[i];
    if (tid == 0) {
      if (a.obj) a.obj[b] = objv;
      a.status[b] = status;
      if (a.iters) a.iters[b] = iters;
    }
  }
}

// ----------------------------------------------------------------------------
// per-horizon launcher.  This file is compiled once per horizon with
// -DHMPC_INST_N=<N> (see build.sh) so the instantiations build in parallel;
// hmpc_dispatch.cpp maps (variant, N) onto these entry points.
// ----------------------------------------------------------------------------
#ifndef HMPC_INST_N
#error "compile with -DHMPC_INST_N=<horizon>"
#endif
#define HMPC_CAT2(a, b) a##b
#define HMPC_CAT(a, b) HMPC_CAT2(a, b)

bool HMPC_CAT(launch_solve_n, HMPC_INST_N)(int variant, const SolveArgs& a, hipStream_t s) {
  constexpr int N = HMPC_INST_N;
  constexpr int NT = Lay<N>::NT;
  if (a.B <= 0) return true;
  if (variant == 3) {
    hipLaunchKernelGGL((solve_kernel<3, N>), dim3((unsigned)a.B), dim3(NT), 0, s, a);
    return true;
  }
  if (variant == 2) {
    hipLaunchKernelGGL((solve_kernel<2, N>), dim3((unsigned)a.B), dim3(NT), 0, s, a);
    return true;
  }
  return false;
}

}  // namespace hmpc
