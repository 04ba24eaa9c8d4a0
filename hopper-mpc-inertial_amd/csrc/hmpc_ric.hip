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
// R lives in LDS with a capacity ric_qcap(N) (hmpc_internal.h); an instance whose active set
// outgrows it is handed to the overflow pass (capacity 6N, R in global
// memory) instead of failing.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "hmpc_internal.h"
#include "hmpc_model.h"

namespace hmpc {

namespace {

constexpr int RT = 64;   // one wavefront per workgroup
// MRHS (speculative candidate columns) in every main-pass
// kernel, their four columns in LDS, the single-RHS sweeps through the same
// body; 16 candidate cache slots per workgroup (<= 64; 32 measured no better)
constexpr int kNSC = 16;
constexpr int kMRK = 4;                         // right-hand sides per sweep pair (DPP rows)

// LDS layout (in doubles) for a runtime horizon N and active-set capacity cap
// (R in LDS only when r_lds).
struct RicLay {
  int XIN, CC, CS, BW, ZB, ZN, ZD, MISC, VV, SV, NB, ZV, MU, UA, ACT, CB, SD, RM, U0, total;
  // fac: the factorisation kernel's layout (stage data, then the union)
  __host__ __device__ RicLay(int N, int cap, bool r_lds, bool fac = false) {
    const int NV = 6 * N;
    auto up2 = [](int x) { return (x + 1) & ~1; };   // 16-B alignment of every array
    int o = 0;
    XIN = o; o += 12;
    CC = o; o = up2(o + N);
    CS = o; o += 2 * N;
    BW = o; o += 18 * N;
    if (fac) {
      ZB = ZN = ZD = MISC = VV = SV = NB = ZV = MU = UA = ACT = CB = SD = U0 = RM = o;
      total = o + (568 > 12 * N ? 568 : 12 * N);
      return;
    }
    ZB = o; o = up2(o + N + 1);   // free-response heights z_k, k = 0..N
    ZN = o; o = up2(o + N);       // |n| of the z row of stage k
    ZD = o; o = up2(o + N);       // z-row dots of s = H^-1 n_p
    MISC = o; o += 8;
    VV = o; o += NV;              // primal iterate
    SV = o; o += NV;              // s = H^-1 n_p
    NB = o; o += NV;              // right-hand side of H^-1 (n_p, n_p - N_A r)
    ZV = o; o += NV;              // z = H^-1 (n_p - N_A r); with MU: d_t (12 N) in phase 1
    MU = o; o += NV;              // sweep scratch (mu, then G^-1 mu)
    UA = o; o = up2(o + cap);     // active multipliers
    ACT = o; o = up2(o + cap);    // active ids (int)
    CB = o; o = up2(o + cap);     // r of the dual step (z builder), then the
    SD = CB;                      // subdiagonal of a drop (not live together)
    U0 = o; o += 568;             // Riccati scratch | x_ref (12 N, phases 0-1 and 5,
    RM = o; if (r_lds) o = up2(o + cap * (cap + 1) / 2);   // over R too); packed upper R
    total = o > U0 + 12 * N ? o : U0 + 12 * N;
  }
};

// Riccati scratch inside the union (P_{k+1} and P_k in turn, P B, B'P A, G,
// Dinv, K_k)
constexpr int PS_OFF = 0, P2_OFF = 144, TS_OFF = 288, FS_OFF = 360, GS_OFF = 432, DL_OFF = 468,
              KL_OFF = 490;

// Global workspace of one workgroup (doubles): K_k [6][12] and Dinv_k (packed
// lower; G_k^-1 = Dinv_k' Dinv_k) of every stage -- written by the
// factorisation, read by every sweep
__host__ __device__ inline int64_t ric_kws_doubles(int N) { return ((93 * (int64_t)N) + 15) & ~(int64_t)15; }
// the factorisation kernel's per-instance output (ric_kinst_stride): K / Dinv
// of every stage, then a flag (nonzero: a non-positive pivot)
__host__ __device__ inline int64_t ric_kinst_doubles(int N) { return ((93 * (int64_t)N + 1) + 15) & ~(int64_t)15; }

__device__ __forceinline__ int loff(int r) { return (r * (r + 1)) >> 1; }

// maximum over the wave of x in [0, 63] (uniform result), by six ballots
__device__ __forceinline__ int wave_imax63(int x) {
  int hi = 0;
#pragma unroll
  for (int bit = 5; bit >= 0; --bit) {
    const int cand = hi | (1 << bit);
    if (__ballot(x >= cand)) hi = cand;
  }
  return hi;
}

// Ordering point between lanes of the one wavefront of a workgroup: LDS
// instructions of a wave execute in order, so only the compiler must be kept
// from reordering them.  Global-memory hand-offs between lanes (the K / Dinv
// workspace, the overflow pass's R) use gsync() = a workgroup barrier.
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }
__device__ __forceinline__ void gsync() { __syncthreads(); }

// Diagnostic build only (-DHMPC_STAMPS, tools/ric_stamps.py): s_memtime
// cycles per phase, accumulated, written over the instance's x* row.
#ifdef HMPC_STAMPS
#define RS_T(v) const long long v = __builtin_amdgcn_s_memtime()
#define RS_ACC(slot, v) (rst_[slot] += __builtin_amdgcn_s_memtime() - (v))
// event counts (stamped builds): slots 11-14 time the factorisation's parts
// where the kernel factorises, else they count s sweep pairs, MRHS cache
// hits, z fallback sweeps and right-hand sides per sweep pair
#define RS_CNT(slot, n) (rst_[slot] += (n))
#else
#define RS_T(v) ((void)0)
#define RS_ACC(slot, v) ((void)0)
#define RS_CNT(slot, n) ((void)0)
#endif

// inclusive prefix sum over the wave (lane order): Hillis-Steele inside each
// row of 16 lanes by DPP row shifts, then the row broadcasts of lanes 15 and
// 31 into the rows above (VALU modifiers, no LDS round trip)
template <int CTRL, int RM>
__device__ __forceinline__ double dpp0(double x) {   // 0 where the source is out of range / masked
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, RM, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, RM, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double wave_scan(double x) {
  x += dpp0<0x111, 0xf>(x);   // row_shr:1
  x += dpp0<0x112, 0xf>(x);   // row_shr:2
  x += dpp0<0x114, 0xf>(x);   // row_shr:4
  x += dpp0<0x118, 0xf>(x);   // row_shr:8
  x += dpp0<0x142, 0xa>(x);   // row_bcast:15 into rows 1, 3
  x += dpp0<0x143, 0xc>(x);   // row_bcast:31 into rows 2, 3
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

constexpr double kZcRel = 1e-3;   // the z-fallback threshold
// ZC: z = H^-1 (n_p - N_A r) as s - sum_a r_a S_a from the cached columns
// S_a = H^-1 n_a of the active rows (scw: cap x NV, kept in active order),
// instead of a third pair of sweeps per iteration
// NC, CAPC > 0: the horizon and the R capacity as compile-time constants
// (every LDS offset and loop bound folds; the runtime-N instantiation serves
// any other horizon)
// PART: 0 the whole solve; 1 phases 0 and 2 only (the
// factorisation kernel: K / Dinv and the pivot flag to kw); 2 every phase but
// the factorisation, whose K / Dinv and flag kw already holds
template <int VAR, int ENT, int RING, bool ZC, int NC = 0, int CAPC = 0, int PART = 0>
__device__ void ric_solve(const SolveArgs& a, const int N_, const int64_t b, double* sm, double* Rm,
                          const int cap_, double* kw, double* scw) {
  // lane and N through volatile asm: made afresh for every instance, so the
  // compiler cannot hoist lane- and N-derived values (masks, offsets) out of
  // the persistent instance loop and hold them -- spilled -- for the kernel's
  // whole life
  int lane, N;
  asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"((int)threadIdx.x));
  if constexpr (NC > 0) N = NC;
  else asm volatile("s_mov_b32 %0, %1" : "=s"(N) : "s"(N_));
  const int cap = CAPC > 0 ? CAPC : cap_;
  const RicLay L(N, cap, false, PART == 1);
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
  double* km = kw;            // K_k (global workspace)
  double* gi = kw + 72 * N;   // Dinv_k, G_k^-1 = Dinv'Dinv (global workspace, packed lower 21)
  double* ua = sm + L.UA;
  int* act = reinterpret_cast<int*>(sm + L.ACT);
  double* cbv = sm + L.CB;
  double* sdg = sm + L.SD;
  double* un = sm + L.U0;
  constexpr bool kMR = ENT == 1 && ZC;
  // ... with its four columns in LDS (SV, ZV, MU and the union's 568-double
  // Riccati scratch, all dead during the s sweep pair; 6N <= 568 for N <= 64)
  constexpr bool kMRL = kMR;
  static_assert(6 * kRicNmax <= 568, "an MRHS column must fit the union's Riccati scratch");
  // MRHS candidate columns: after the cached active columns S (cap x NV)
  [[maybe_unused]] double* gcache = kMR && scw ? scw + (int64_t)cap * NV : nullptr;   // (none in the factorisation kernel)

#ifdef HMPC_STAMPS
  long long rst_[16] = {0};
#endif
  RS_T(t_all);
  RS_T(t_p0);
  // ---------------- phase 0: loads + gen_dt_dynamics (lane k < N) ----------
  // x_ref / pf / C may be strided views of a resident plan (path_plan_grab,
  // src/robotrunner.py:228-230); x_lin rows per shift_mode (3f :50-62)
  const double* xrf = a.x_ref + b * a.xref_bs;
  const double mu = a.mu ? a.mu[b] : a.mu_default;
  // x_ref (12 N) into the union; with a compile-time horizon every load of
  // the lane is issued before its first store (round 6: the loop's load ->
  // store pairs were 12 serial round trips at N = 60)
  auto stage_xref = [&]() __attribute__((always_inline)) {
    if constexpr (NC > 0 && RING == 3) {   // (the one-wave kernels: registers to spare)
      constexpr int XE = (12 * NC + RT - 1) / RT;
      double xv[XE];
#pragma unroll
      for (int e = 0; e < XE; ++e) {
        const int i = lane + RT * e < 12 * NC ? lane + RT * e : 0, r = i / 12, c = i - 12 * r;
        xv[e] = xrf[(int64_t)r * a.xref_rs + c];
      }
#pragma unroll
      for (int e = 0; e < XE; ++e)
        if (lane + RT * e < 12 * NC) un[lane + RT * e] = xv[e];
    } else {
      for (int i = lane; i < 12 * N; i += RT) {
        const int r = i / 12, c = i - 12 * r;
        un[i] = xrf[(int64_t)r * a.xref_rs + c];
      }
    }
  };
  if (lane < 12) xin[lane] = a.x_in[b * 12 + lane];
  stage_xref();
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

  RS_ACC(0, t_p0);
  RS_T(t_p1);
  // ---------------- phase 1: free response, d_t, adjoint, gradient ----------
  // lane r < 12 holds component r.  d_t = kf Q (xbar_t - r_{t-1}) goes to
  // ZV..MU (12 N, free until phase 3), x_ref is staged in the union; the gradient h = 2 Gamma' W (xbar - r) - 2 V ubar goes to
  // NB as -h (the right-hand side of the unconstrained optimum).
  if constexpr (PART != 1) {
    double* dd = zv;
    double xr = lane < 12 ? xin[lane] : 0.0;
    const double qr = qdiag(lane);
    if (lane == 2) zb[0] = xr;
    const double ubar_alias = (cc[N - 1] != 0.0) ? 2.0 * a.m * a.g : 0.0;
    if constexpr (ENT == 1) {
      // both recursions load each stage's data one iteration ahead (x_ref,
      // cos / sin, Bd rows, C, d_t do not depend on the carried state): the
      // loads of the next iteration are in flight while this one's chain
      // runs, instead of a round trip in series at the head of every
      // iteration.  (Main kernels only: in the overflow kernel this form
      // put an AGPR copy before an EXEC restore, tests/test_exec_lint.py.)
      const int l12 = lane < 12 ? lane : 0;
      double cpn = cs[0], spn = cs[1], unn = un[l12];
      for (int k = 0; k < N; ++k) {
        const double cpk = cpn, spk = spn, uk = unn;
        const int k1 = k + 1 < N ? k + 1 : k;
        cpn = cs[2 * k1];
        spn = cs[2 * k1 + 1];
        unn = un[12 * k1 + l12];
        xr = ad_lane(xr, dt, cpk, spk, lane) + ((lane == 8) ? -a.g * dt : 0.0);
        const double kf = (k == N - 1) ? kTermQ : 1.0;
        if (lane < 12) dd[12 * k + lane] = kf * qr * (xr - uk);
        if (lane == 2) zb[k + 1] = xr;
      }
      wsync();
      double ar = lane < 12 ? dd[12 * (N - 1) + lane] : 0.0;   // a_N = d_N
      const int c6 = lane < 6 ? lane : 0;
      struct StageB { double cp, sp, b0, b1, b2, st, d; };
      auto load_stage = [&](int i, StageB& s) __attribute__((always_inline)) {
        s.cp = cs[2 * i];
        s.sp = cs[2 * i + 1];
        s.b0 = bw[18 * i + c6];
        s.b1 = bw[18 * i + 6 + c6];
        s.b2 = bw[18 * i + 12 + c6];
        s.st = cc[i];
        s.d = dd[12 * (i >= 1 ? i - 1 : 0) + l12];   // d_{t-1} of the a update (t >= 2)
      };
      StageB nx;
      load_stage(N - 1, nx);
      for (int t = N; t >= 1; --t) {
        const int i = t - 1;
        const StageB cur = nx;
        load_stage(i >= 1 ? i - 1 : 0, nx);
        const double a6 = rdlane(ar, 6), a7 = rdlane(ar, 7), a8 = rdlane(ar, 8);
        const double a9 = rdlane(ar, 9), a10 = rdlane(ar, 10), a11 = rdlane(ar, 11);
        {   // lanes c < 6 (branch-free; the others compute a copy of input 0)
          const int c = c6;
          const double cp = cur.cp, sp = cur.sp;
          double acc = cur.b0 * a9 + cur.b1 * a10 + cur.b2 * a11;
          const double af = bv<VAR>(0, c, dtm, cp, sp) * a6 + bv<VAR>(1, c, dtm, cp, sp) * a7 +
                            bv<VAR>(2, c, dtm, cp, sp) * a8;
          acc = c < 3 ? acc + af : acc;
          const bool stance = cur.st != 0.0;
          const bool fr = c >= 3 || (stance && !(VAR == 2 && c == 1));
          const double ub = a.uref_aliased ? ubar_alias : (stance ? 2.0 * a.m * a.g : 0.0);
          const double hz = 2.0 * acc - 2.0 * kRdiag * ub;
          const double h = fr ? ((c == 2 && i < N - 1) ? hz : 2.0 * acc) : 0.0;
          if (lane < 6) nb[6 * i + c] = -h;
        }
        if (t >= 2) ar = adt_lane(ar, dt, cur.cp, cur.sp, lane) + (lane < 12 ? cur.d : 0.0);
      }
    } else {
      for (int k = 0; k < N; ++k) {
        xr = ad_lane(xr, dt, cs[2 * k], cs[2 * k + 1], lane) + ((lane == 8) ? -a.g * dt : 0.0);
        const double kf = (k == N - 1) ? kTermQ : 1.0;
        if (lane < 12) dd[12 * k + lane] = kf * qr * (xr - un[12 * k + lane]);
        if (lane == 2) zb[k + 1] = xr;
      }
      wsync();
      double ar = lane < 12 ? dd[12 * (N - 1) + lane] : 0.0;   // a_N = d_N
      for (int t = N; t >= 1; --t) {
        const int i = t - 1;
        const double a6 = rdlane(ar, 6), a7 = rdlane(ar, 7), a8 = rdlane(ar, 8);
        const double a9 = rdlane(ar, 9), a10 = rdlane(ar, 10), a11 = rdlane(ar, 11);
        {   // lanes c < 6 (branch-free; the others compute a copy of input 0)
          const int c = lane < 6 ? lane : 0;
          const double cp = cs[2 * i], sp = cs[2 * i + 1];
          const double* bwi = bw + 18 * i;
          double acc = bwi[c] * a9 + bwi[6 + c] * a10 + bwi[12 + c] * a11;
          const double af = bv<VAR>(0, c, dtm, cp, sp) * a6 + bv<VAR>(1, c, dtm, cp, sp) * a7 +
                            bv<VAR>(2, c, dtm, cp, sp) * a8;
          acc = c < 3 ? acc + af : acc;
          const bool stance = cc[i] != 0.0;
          const bool fr = c >= 3 || (stance && !(VAR == 2 && c == 1));
          const double ub = a.uref_aliased ? ubar_alias : (stance ? 2.0 * a.m * a.g : 0.0);
          const double hz = 2.0 * acc - 2.0 * kRdiag * ub;
          const double h = fr ? ((c == 2 && i < N - 1) ? hz : 2.0 * acc) : 0.0;
          if (lane < 6) nb[6 * i + c] = -h;
        }
        if (t >= 2) {
          ar = adt_lane(ar, dt, cs[2 * i], cs[2 * i + 1], lane) + (lane < 12 ? dd[12 * (t - 2) + lane] : 0.0);
        }
      }
    }
  }
  wsync();

  RS_ACC(1, t_p1);
  RS_T(t_p2);
  // ---------------- phase 2: Riccati factorisation -------------------------
  // P_N = 2 (100 Q); per stage k = N-1..0, with A_k = I + dt E_k (column j of
  // A_k: 1 at row j plus at most two more rows, arow/acoef below):
  //   (a) T = P B                      (12 x 6; fixed columns 0)
  //   (b) G = 2 V + B'T, F = T'A       (identity rows/cols for fixed variables)
  //   (c) G = D D' (reciprocal pivots), K = G^-1 F, Dinv
  //   (d) G^-1 = Dinv'Dinv, P_k = 2 Q + A'P A - F'K straight from P_{k+1}
  //       (no P A product: every entry of A'P A is <= 9 entries of P)
  // Work items are laid over the 64 lanes with a second item per lane for
  // the overhang, both in one unrolled body (their LDS latencies overlap).
  int status = ST_SOLVED;
  if constexpr (PART == 2) {   // factorised by the factorisation kernel
    if (kw[93 * N] != 0.0) status = ST_NUMERICAL;
  } else {
    double* Pc = un + PS_OFF;   // P_{k+1}, 12 x 12 full
    double* Pn = un + P2_OFF;   // P_k
    double* T = un + TS_OFF;    // P B, 12 x 6
    double* F = un + FS_OFF;    // (B'P A)' by rows: F[6 j + c] = (B'P A)[c][j], j >= 6
    double* G = un + GS_OFF;    // 6 x 6
    // column j of B'P A as a contiguous 6-vector: T's row j for j < 6 (A's
    // first six columns are e_j), F's row j otherwise; read as 3 b128 loads
    typedef double dbl2 __attribute__((ext_vector_type(2)));
    auto col6 = [&](int j, double (&v)[6]) __attribute__((always_inline)) {
      const dbl2* p = reinterpret_cast<const dbl2*>((j < 6 ? T : F) + 6 * j);
      const dbl2 v0 = p[0], v1 = p[1], v2 = p[2];
      v[0] = v0.x; v[1] = v0.y; v[2] = v1.x; v[3] = v1.y; v[4] = v2.x; v[5] = v2.y;
    };
    double* Kl = un + KL_OFF;   // K_k by columns (Kl[6 j + c] = K[c][j]; the P update reads it)
    for (int e = lane; e < 144; e += RT) {
      const int i = e / 12, j = e - 12 * i;
      Pc[e] = (i == j) ? 2.0 * kTermQ * kQ[i] : 0.0;
    }
    // lane constants: P-update items (i, j), j <= i (78 = 64 + 14), the G^-1
    // item (c, d) of lanes < 21
    auto tri = [](int e, int& i, int& j) {
      i = 0;
      while (loff(i + 1) <= e) ++i;
      j = e - loff(i);
    };
    int pi0, pj0, pi1, pj1, gc, gd;   // (gc, gd): lane's G item, lanes 36..56
    tri(lane, pi0, pj0);
    tri(lane + 64 < 78 ? lane + 64 : 0, pi1, pj1);
    tri(lane >= 36 && lane < 57 ? lane - 36 : 0, gc, gd);
    const bool p1 = lane + 64 < 78;
    // column j of A: extra rows ar1, ar2 with coefficients dt * (x1 + y1 cos
    // + z1 sin), dt * (y2 cos + z2 sin)
    struct ACol {
      int r1, r2;
      double x1, y1, z1, y2, z2;
    };
    // branch-free: j is a per-lane value, and an if/else chain here compiled
    // to divergent branches that reloaded spilled SGPRs on every path
    auto acol = [&](int j) -> ACol {
      const bool v = j >= 6 && j < 9, w9 = j == 9, w10 = j == 10, w11 = j == 11, w = w9 || w10;
      ACol c;
      c.r1 = v ? j - 6 : (w ? 3 : (w11 ? 5 : j));
      c.r2 = w ? 4 : j;
      c.x1 = (v || w11) ? dt : 0.0;
      c.y1 = w9 ? dt : 0.0;
      c.z1 = w10 ? dt : 0.0;
      c.y2 = w10 ? dt : 0.0;
      c.z2 = w9 ? -dt : 0.0;
      return c;
    };
    wsync();
    double nbad = 0.0;
    for (int k = N - 1; k >= 0; --k) {
      const double cp = cs[2 * k], sp = cs[2 * k + 1];
      const bool stance = cc[k] != 0.0;
      const double* bwk = bw + 18 * k;
      auto freec = [&](int c) { return c >= 3 || (stance && !(VAR == 2 && c == 1)); };
      // B[6 + r][c], r < 3 (the force map; 3f: dtm I, 2f: dtm Rz')
      auto bforce = [&](int r, int c) -> double { return c < 3 ? bv<VAR>(r, c, dtm, cp, sp) : 0.0; };
      RS_T(t_fa);
      // (a) T[i][c] = sum_r P[i][6 + r] B[6 + r][c] + P[i][9 + r] BW[r][c]
      {
        auto titem = [&](int e) -> double {
          const int i = e / 6, c = e - 6 * i;
          const double* pr = Pc + 12 * i;
          double acc = pr[9] * bwk[c];
          acc = fma(pr[10], bwk[6 + c], acc);
          acc = fma(pr[11], bwk[12 + c], acc);
          if (c < 3) {
            acc = fma(pr[6], bforce(0, c), acc);
            acc = fma(pr[7], bforce(1, c), acc);
            acc = fma(pr[8], bforce(2, c), acc);
          }
          return freec(c) ? acc : 0.0;
        };
        const double t0 = titem(lane);
        const double t1 = titem(lane < 8 ? lane + 64 : 0);
        T[lane] = t0;
        if (lane < 8) T[lane + 64] = t1;
      }
      wsync();
      RS_ACC(11, t_fa);
      RS_T(t_fb);
      // (b) in one pass: F[c][j] = (T'A)[c][j] for the columns j >= 6 (lanes
      // < 36; the columns j < 6 of A are unit vectors, so F[c][j] = T[j][c]
      // there and is read from T), and the lower triangle of G = 2V + B'T
      // (lanes 36..56; identity rows/columns for fixed variables)
      {
        if (lane < 36) {
          const int c = lane / 6, j = 6 + lane - 6 * c;
          const ACol aj = acol(j);
          double f = T[6 * j + c];
          f = fma(aj.x1 + aj.y1 * cp + aj.z1 * sp, T[6 * aj.r1 + c], f);
          f = fma(aj.y2 * cp + aj.z2 * sp, T[6 * aj.r2 + c], f);
          F[6 * j + c] = f;
        } else if (lane < 57) {
          const int c = gc, d = gd;
          double acc = bwk[c] * T[54 + d];
          acc = fma(bwk[6 + c], T[60 + d], acc);
          acc = fma(bwk[12 + c], T[66 + d], acc);
          if (c < 3) {
            acc = fma(bforce(0, c), T[36 + d], acc);
            acc = fma(bforce(1, c), T[42 + d], acc);
            acc = fma(bforce(2, c), T[48 + d], acc);
          }
          if (!freec(c)) acc = c == d ? 1.0 : 0.0;
          else if (c == d) acc += (k < N - 1) ? 2.0 * kRdiag : 0.0;
          G[6 * c + d] = acc;
        }
      }
      wsync();
      RS_ACC(12, t_fb);
      RS_T(t_fc);
      // (c) G = D D' (every lane, redundantly) with reciprocal pivots (no
      // fp64 divide or sqrt sequences), Dinv = D^-1; K = Dinv'(Dinv F) (lanes
      // j < 12, one column each); Dinv to LDS for G^-1 = Dinv'Dinv (lanes < 21)
      double D[21], Di[21], dinv[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
#pragma unroll
        for (int d = 0; d <= c; ++d) {
          double s = G[6 * c + d];
#pragma unroll
          for (int m = 0; m < d; ++m) s = fma(-D[loff(c) + m], D[loff(d) + m], s);
          if (d == c) {
            nbad += (s > 0.0) ? 0.0 : 1.0;
            dinv[c] = rsq_nr(s > 0.0 ? s : 1.0);
          } else {
            D[loff(c) + d] = s * dinv[d];
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) {   // column c of Dinv: forward substitution of e_c
        Di[loff(c) + c] = dinv[c];
#pragma unroll
        for (int r = c + 1; r < 6; ++r) {
          double s = 0.0;
#pragma unroll
          for (int m = c; m < r; ++m) s = fma(D[loff(r) + m], Di[loff(m) + c], s);
          Di[loff(r) + c] = -s * dinv[r];
        }
      }
      // Dinv (packed lower) for the sweeps, which apply G^-1 = Dinv'Dinv as
      // two triangular products: every lane holds all 21 entries, lane 0
      // stores them (no per-lane select chain)
      if (lane == 0) {
        double* g = gi + 21 * k;
#pragma unroll
        for (int e = 0; e < 21; ++e) g[e] = Di[e];
      }
      if (lane < 12) {
        const int j = lane;
        double y[6], fj[6];
        col6(j, fj);
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double s = 0.0;
#pragma unroll
          for (int m = 0; m <= c; ++m) s = fma(Di[loff(c) + m], fj[m], s);
          y[c] = s;
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double s = 0.0;
#pragma unroll
          for (int m = c; m < 6; ++m) s = fma(Di[loff(m) + c], y[m], s);
          km[72 * k + 12 * c + j] = s;
          Kl[6 * j + c] = s;
        }
      }
      wsync();
      RS_ACC(13, t_fc);
      RS_T(t_fd);
      // (d) P_k (i, j), j <= i, mirrored
      if (k == 0) break;
      {
        auto pitem = [&](int i, int j) -> double {
          const ACol ai = acol(i), aj = acol(j);
          const double q = (i == j) ? 2.0 * qdiag(i) : 0.0;
          const double ca1 = ai.x1 + ai.y1 * cp + ai.z1 * sp, ca2 = ai.y2 * cp + ai.z2 * sp;
          const double cb1 = aj.x1 + aj.y1 * cp + aj.z1 * sp, cb2 = aj.y2 * cp + aj.z2 * sp;
          const double* r0 = Pc + 12 * i;
          const double* r1 = Pc + 12 * ai.r1;
          const double* r2 = Pc + 12 * ai.r2;
          const double s0 = fma(cb2, r0[aj.r2], fma(cb1, r0[aj.r1], r0[j]));
          const double s1 = fma(cb2, r1[aj.r2], fma(cb1, r1[aj.r1], r1[j]));
          const double s2 = fma(cb2, r2[aj.r2], fma(cb1, r2[aj.r1], r2[j]));
          double pn = fma(ca2, s2, fma(ca1, s1, s0)) + q;
          double fi[6], kj[6];
          col6(i, fi);
          {
            const dbl2* kp = reinterpret_cast<const dbl2*>(Kl + 6 * j);
            const dbl2 k0 = kp[0], k1 = kp[1], k2 = kp[2];
            kj[0] = k0.x; kj[1] = k0.y; kj[2] = k1.x; kj[3] = k1.y; kj[4] = k2.x; kj[5] = k2.y;
          }
#pragma unroll
          for (int c = 0; c < 6; ++c) pn = fma(-fi[c], kj[c], pn);
          return pn;
        };
        const double v0 = pitem(pi0, pj0);
        const double v1 = pitem(pi1, pj1);   // (lanes >= 14: a duplicate of item 0, not stored)
        Pn[12 * pi0 + pj0] = v0;
        Pn[12 * pj0 + pi0] = v0;
        if (p1) {
          Pn[12 * pi1 + pj1] = v1;
          Pn[12 * pj1 + pi1] = v1;
        }
      }
      wsync();
      double* tmp = Pc; Pc = Pn; Pn = tmp;
      RS_ACC(14, t_fd);
    }
    if (nbad != 0.0) status = ST_NUMERICAL;
  }
  if constexpr (PART == 1) {   // the factorisation kernel: the pivot flag, then done
    if (lane == 0) kw[93 * N] = status == ST_SOLVED ? 0.0 : 1.0;
    return;
  }
  gsync();   // K, Dinv (global) visible to every lane of the workgroup

  // ---------------- H^-1 by two sweeps ----------------------------------------
  // dst = H^-1 NB (NB kept; MU scratch).  Lanes 0..11 hold the 12 state
  // (forward) / adjoint (backward) components; the cross-component terms of A
  // come from DPP row shifts, the 6 inputs from lanes 0..5 by readlane.
  //   backward: mu_j[c] = n_j[c] - B_j[:,c]'lam    (lane c < 6; lam[6..11] in SGPRs)
  //             lam_j[i] = (A_j'lam)[i] + K_j[:,i]'mu_j   (lane i < 12)
  //   per stage: w_j = G_j^-1 mu_j                (lane j)
  //   forward:  u_k[r] = w_k[r] - K_k[r,:] x       (lane r < 6; x in SGPRs)
  //             x_{k+1}[i] = (A_k x)[i] + B_k[i,:] u_k    (lane i < 12)
  // Every step's data (K_k from the global workspace, B_k / w_k from LDS) is
  // loaded two steps ahead (a three-deep register ring).
  // acc += x[lane n of the row] * k as ONE instruction: gfx950's 64-bit DPP
  // (row_newbcast only) broadcasts lane n of each 16-lane row, and every
  // consumer here is in row 0 (lanes < 12) -- no readlane -> SGPR -> FMA
  // round trip.  Each block starts with s_nop 4: the compiler does not see
  // DPP inside asm, so the block covers the worst hazard in front of it
  // itself -- an SALU write of EXEC (the lane < 6 stores) followed by a DPP
  // op needs 5 wait states (a VALU write of x, 2).
// The overflow pass (ENT > 1) keeps the readlane form.
#define HMPC_DPPF(acc, x, k, n) "v_fmac_f64_dpp %" #acc ", %" #x ", %" #k " row_newbcast:" #n " row_mask:0xf bank_mask:0xf\n\t"
#define HMPC_DPPFN(acc, x, k, n) "v_fmac_f64_dpp %" #acc ", %" #x ", -%" #k " row_newbcast:" #n " row_mask:0xf bank_mask:0xf\n\t"
  struct BwdL {
    double cp, sp, st, b0, b1, b2, n, kc[6];
  };
  struct FwdL {
    double cp, sp, w, kr[12], br[6];
  };
  // jt (uniform): the last stage where the right-hand side NB is nonzero --
  // the backward sweep starts there (lam_{jt+1} = 0, mu_j = 0 beyond it)
  // hinv_g(MR, ...): MR = std::false_type: dst = H^-1 NB as described above.
  // MR = std::true_type (speculative candidate columns, MRHS; c0..c3 = the
  // rows' columns): up to 4
  // right-hand sides at once, one per 16-lane DPP row -- every broadcast and
  // row shift of the sweeps acts within a row, so row r runs the same
  // recursion on its own vector for free.  Row r's right-hand side, its mu
  // scratch and its result all live in one global column (colb: this lane's
  // row's column; the backward sweep overwrites n_j with mu_j after reading
  // it, the forward sweep w_k with u_k), rows >= nr idle (rowok false).
  auto hinv_g = [&](auto MRt, double* dst, int jt, double* colb, bool rowok, int nr, double* c0, double* c1,
                    double* c2, double* c3) __attribute__((always_inline)) {
    constexpr bool MR = decltype(MRt)::value;
    const int lr = MR ? (lane & 15) : lane;   // lane within its row
    // (lane constants made here, per call: not live across the active set)
    // per-lane constants of the A maps (see the shift comments below)
    const double gA = (lr >= 6 && lr <= 8) || lr == 11 ? dt : 0.0;   // bwd s6, fixed
    const double gB = (lr == 9 || lr == 10) ? dt : 0.0;                // bwd s6, * cos
    const double gC = lr == 9 ? -dt : 0.0;                               // bwd s5, * sin
    const double gD = lr == 10 ? dt : 0.0;                               // bwd s7, * sin
    const double fA = lr < 3 || lr == 5 ? dt : 0.0;                    // fwd s6, fixed
    const double fB = (lr == 3 || lr == 4) ? dt : 0.0;                 // fwd s6, * cos
    const double fC = lr == 3 ? dt : 0.0;                                // fwd s7, * sin
    const double fD = lr == 4 ? -dt : 0.0;                               // fwd s5, * sin
    const int c6 = lr < 6 ? lr : 0;
    // force map rows 6..8 of B_k = dtm (3f: I; 2f: Rz(psi)') as per-lane
    // coefficients P + Q cos + S sin, branch-free:
    //   k*[r] (backward, lane c < 6):  B[6+r][c]
    //   r*[c] (forward, lane 6+r):     B[6+r][c]
    double kP[3], kQ_[3], kS[3], rP[3], rQ[3], rS[3];
  #pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double on_b = lr == r ? dtm : 0.0, on_f = lr == 6 + r ? dtm : 0.0;
      if constexpr (VAR == 3) {
        kP[r] = on_b; kQ_[r] = 0.0; kS[r] = 0.0;
        rP[r] = on_f; rQ[r] = 0.0; rS[r] = 0.0;
      } else {   // Rz' = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
        kP[r] = r == 2 ? on_b : 0.0;
        kQ_[r] = r < 2 ? on_b : 0.0;
        kS[r] = r == 0 ? (lr == 1 ? -dtm : 0.0) : (r == 1 ? (lr == 0 ? dtm : 0.0) : 0.0);
        rP[r] = r == 2 ? (lr == 8 ? dtm : 0.0) : 0.0;
        rQ[r] = r < 2 ? on_f : 0.0;   // column r of row r: cos
        rS[r] = r == 0 ? (lr == 7 ? dtm : 0.0) : (r == 1 ? (lr == 6 ? -dtm : 0.0) : 0.0);
      }
    }
    const double m911 = (lr >= 9 && lr < 12) ? 1.0 : 0.0;
    auto load_b = [&](int j, BwdL& d) __attribute__((always_inline)) {
      d.cp = cs[2 * j];
      d.sp = cs[2 * j + 1];
      d.st = cc[j];
      d.b0 = bw[18 * j + c6];
      d.b1 = bw[18 * j + 6 + c6];
      d.b2 = bw[18 * j + 12 + c6];
      if constexpr (MR) d.n = colb[6 * j + c6];
      else d.n = nb[6 * j + c6];
      const double* kcol = km + 72 * j + (lr < 12 ? lr : 0);
  #pragma unroll
      for (int c = 0; c < 6; ++c) d.kc[c] = kcol[12 * c];
      asm volatile("" ::: "memory");   // issue here, two steps ahead of the use
    };
    auto load_f = [&](int k, FwdL& d) __attribute__((always_inline)) {
      d.cp = cs[2 * k];
      d.sp = cs[2 * k + 1];
      if constexpr (MR) d.w = colb[6 * k + c6];
      else d.w = mu_[6 * k + c6];
      const double* krow = km + 72 * k + 12 * c6;
  #pragma unroll
      for (int c = 0; c < 12; ++c) d.kr[c] = krow[c];
      const int rr = (lr >= 9 && lr < 12) ? lr - 9 : 0;
  #pragma unroll
      for (int c = 0; c < 6; ++c) d.br[c] = bw[18 * k + 6 * rr + c];
      asm volatile("" ::: "memory");   // issue here, two steps ahead of the use
    };
    // ---- backward sweep
    {
      double li = 0.0;                                  // lam_{j+1}[lane]
      auto bstep = [&](int j, const BwdL& d) __attribute__((always_inline)) {
        double k6, k7, k8;
        if constexpr (VAR == 3) {
          k6 = kP[0]; k7 = kP[1]; k8 = kP[2];
        } else {
          k6 = fma(kQ_[0], d.cp, kS[0] * d.sp);
          k7 = fma(kQ_[1], d.cp, kS[1] * d.sp);
          k8 = kP[2];
        }
        // B_j'lam over lam[6..11] (lanes 6..11 of li)
        double bc;
        if constexpr (ENT == 1) {
          double bc0 = 0.0, bc1 = 0.0;
          asm("s_nop 4\n\t" HMPC_DPPF(0, 2, 3, 6) HMPC_DPPF(1, 2, 4, 7) HMPC_DPPF(0, 2, 5, 8)
              HMPC_DPPF(1, 2, 6, 9) HMPC_DPPF(0, 2, 7, 10) HMPC_DPPF(1, 2, 8, 11)
              : "+v"(bc0), "+v"(bc1)
              : "v"(li), "v"(k6), "v"(k7), "v"(k8), "v"(d.b0), "v"(d.b1), "v"(d.b2));
          bc = bc0 + bc1;
        } else {
          bc = fma(k6, rdlane(li, 6), fma(k7, rdlane(li, 7), k8 * rdlane(li, 8))) +
               fma(d.b0, rdlane(li, 9), fma(d.b1, rdlane(li, 10), d.b2 * rdlane(li, 11)));
        }
        const bool fr = lr >= 3 || (d.st != 0.0 && !(VAR == 2 && lr == 1));
        const double m = fr ? d.n - bc : d.n;
        if constexpr (MR) {
          if (lr < 6 && rowok) colb[6 * j + lr] = m;
        } else {
          if (lane < 6) mu_[6 * j + lane] = m;
        }
        if (j == 0) return;
        // (A'lam)[i]: lanes 6..8 += dt lam[i-6]; 9 += dt (c lam3 - s lam4);
        // 10 += dt (s lam3 + c lam4); 11 += dt lam5
        const double s6 = row_shift<-6>(li), s5 = row_shift<-5>(li), s7 = row_shift<-7>(li);
        double a0 = fma(fma(gB, d.cp, gA), s6, li), a1 = (gC * d.sp) * s5, a2 = (gD * d.sp) * s7;
        // + K_j[:, i]'mu_j, mu_j in lanes 0..5 of m
        if constexpr (ENT == 1) {
          asm("s_nop 4\n\t" HMPC_DPPF(0, 3, 4, 0) HMPC_DPPF(1, 3, 5, 1) HMPC_DPPF(2, 3, 6, 2)
              HMPC_DPPF(0, 3, 7, 3) HMPC_DPPF(1, 3, 8, 4) HMPC_DPPF(2, 3, 9, 5)
              : "+v"(a0), "+v"(a1), "+v"(a2)
              : "v"(m), "v"(d.kc[0]), "v"(d.kc[1]), "v"(d.kc[2]), "v"(d.kc[3]), "v"(d.kc[4]), "v"(d.kc[5]));
        } else {
          a0 = fma(d.kc[0], rdlane(m, 0), a0);
          a1 = fma(d.kc[1], rdlane(m, 1), a1);
          a2 = fma(d.kc[2], rdlane(m, 2), a2);
          a0 = fma(d.kc[3], rdlane(m, 3), a0);
          a1 = fma(d.kc[4], rdlane(m, 4), a1);
          a2 = fma(d.kc[5], rdlane(m, 5), a2);
        }
        li = lr < 12 ? (a0 + a1) + a2 : 0.0;
      };
      // (loads are unconditional -- out-of-range steps reload stage 0 -- so
      // that the vmcnt/lgkmcnt waits stay counted, not drained)
      static_assert(RING == 2 || RING == 3, "ring depth");
      if constexpr (RING == 3) {
        BwdL R0, R1, R2;
        load_b(jt, R0);
        load_b(jt >= 1 ? jt - 1 : 0, R1);
        for (int j = jt; j >= 0; j -= 3) {
          load_b(j >= 2 ? j - 2 : 0, R2);
          bstep(j, R0);
          if (j < 1) break;
          load_b(j >= 3 ? j - 3 : 0, R0);
          bstep(j - 1, R1);
          if (j < 2) break;
          load_b(j >= 4 ? j - 4 : 0, R1);
          bstep(j - 2, R2);
        }
      } else {   // two-deep (register budget of 2 waves / SIMD)
        BwdL R0, R1;
        load_b(jt, R0);
        for (int j = jt; j >= 0; j -= 2) {
          load_b(j >= 1 ? j - 1 : 0, R1);
          bstep(j, R0);
          if (j < 1) break;
          load_b(j >= 2 ? j - 2 : 0, R0);
          bstep(j - 1, R1);
        }
      }
    }
    if constexpr (MR) {
      gsync();   // every row's mu_j (global) visible to the lanes of the stage step
    } else {
      for (int i = 6 * (jt + 1) + lane; i < NV; i += RT) mu_[i] = 0.0;
      wsync();
    }
    // ---- w_j = G_j^-1 mu_j = Dinv'(Dinv mu_j) (lane-per-stage; 0 beyond jt)
    // lane j holds stage j (jt < kRicNmax = 64): its Dinv is loaded once,
    // one round trip, for every row (round 6: one item per (row, stage)
    // reloaded Dinv per row, up to four serial round trips at N = 60)
    const int nrows = MR ? nr : 1;
    for (int j = lane; j <= jt; j += RT) {
      double g[21];
      const double* gj = gi + 21 * j;
#pragma unroll
      for (int e = 0; e < 21; ++e) g[e] = gj[e];
      for (int r_ = 0; r_ < nrows; ++r_) {
        double* mcol = mu_;
        if constexpr (MR) mcol = r_ == 0 ? c0 : r_ == 1 ? c1 : r_ == 2 ? c2 : c3;
        double mv[6], y[6], w[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) mv[c] = mcol[6 * j + c];
#pragma unroll
        for (int c = 0; c < 6; ++c) {   // y = Dinv mu (lower)
          double s = 0.0;
#pragma unroll
          for (int d = 0; d <= c; ++d) s = fma(g[loff(c) + d], mv[d], s);
          y[c] = s;
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) {   // w = Dinv' y
          double s = 0.0;
#pragma unroll
          for (int d = c; d < 6; ++d) s = fma(g[loff(d) + c], y[d], s);
          w[c] = s;
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) mcol[6 * j + c] = w[c];
      }
    }
    if constexpr (MR) gsync();
    else wsync();
    // ---- forward sweep
    {
      double xi = 0.0;   // x_k[lane]
      auto fstep = [&](int k, const FwdL& d) __attribute__((always_inline)) {
        // u = w - K_k x (x in lanes 0..11 of xi)
        double a0 = d.w, a1 = 0.0;
        if constexpr (ENT == 1) {
          asm("s_nop 4\n\t" HMPC_DPPFN(0, 2, 3, 0) HMPC_DPPFN(1, 2, 4, 1) HMPC_DPPFN(0, 2, 5, 2)
              HMPC_DPPFN(1, 2, 6, 3) HMPC_DPPFN(0, 2, 7, 4) HMPC_DPPFN(1, 2, 8, 5)
              HMPC_DPPFN(0, 2, 9, 6) HMPC_DPPFN(1, 2, 10, 7) HMPC_DPPFN(0, 2, 11, 8)
              HMPC_DPPFN(1, 2, 12, 9) HMPC_DPPFN(0, 2, 13, 10) HMPC_DPPFN(1, 2, 14, 11)
              : "+v"(a0), "+v"(a1)
              : "v"(xi), "v"(d.kr[0]), "v"(d.kr[1]), "v"(d.kr[2]), "v"(d.kr[3]), "v"(d.kr[4]), "v"(d.kr[5]),
                "v"(d.kr[6]), "v"(d.kr[7]), "v"(d.kr[8]), "v"(d.kr[9]), "v"(d.kr[10]), "v"(d.kr[11]));
        } else {
#pragma unroll
          for (int c = 0; c < 12; c += 2) {
            a0 = fma(-d.kr[c], rdlane(xi, c), a0);
            a1 = fma(-d.kr[c + 1], rdlane(xi, c + 1), a1);
          }
        }
        const double u = a0 + a1;
        if constexpr (MR) {
          if (lr < 6 && rowok) colb[6 * k + lr] = u;
        } else {
          if (lane < 6) dst[6 * k + lane] = u;
        }
        // (A x)[i]: lanes 0..2 += dt x[i+6]; 3 += dt (c x9 + s x10);
        // 4 += dt (c x10 - s x9); 5 += dt x11
        const double s6 = row_shift<6>(xi), s5 = row_shift<5>(xi), s7 = row_shift<7>(xi);
        // B rows: 6..8 the force map, 9..11 the stored rows of B_k
        double r0, r1, r2;
        if constexpr (VAR == 3) {
          r0 = rP[0]; r1 = rP[1]; r2 = rP[2];
        } else {
          r0 = fma(rQ[0], d.cp, rS[0] * d.sp);
          r1 = fma(rQ[1], d.cp, rS[1] * d.sp);
          r2 = rP[2];
        }
        r0 = fma(m911, d.br[0], r0);
        r1 = fma(m911, d.br[1], r1);
        r2 = fma(m911, d.br[2], r2);
        const double r3 = m911 * d.br[3], r4 = m911 * d.br[4], r5 = m911 * d.br[5];
        double b0 = fma(fma(fB, d.cp, fA), s6, xi), b1 = (fC * d.sp) * s7, b2 = (fD * d.sp) * s5;
        // + B_k u_k, u_k in lanes 0..5 of u
        if constexpr (ENT == 1) {
          asm("s_nop 4\n\t" HMPC_DPPF(0, 3, 4, 0) HMPC_DPPF(1, 3, 5, 1) HMPC_DPPF(2, 3, 6, 2)
              HMPC_DPPF(0, 3, 7, 3) HMPC_DPPF(1, 3, 8, 4) HMPC_DPPF(2, 3, 9, 5)
              : "+v"(b0), "+v"(b1), "+v"(b2)
              : "v"(u), "v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(r4), "v"(r5));
        } else {
          b0 = fma(r0, rdlane(u, 0), b0);
          b1 = fma(r1, rdlane(u, 1), b1);
          b2 = fma(r2, rdlane(u, 2), b2);
          b0 = fma(r3, rdlane(u, 3), b0);
          b1 = fma(r4, rdlane(u, 4), b1);
          b2 = fma(r5, rdlane(u, 5), b2);
        }
        xi = lr < 12 ? (b0 + b1) + b2 : 0.0;
      };
      if constexpr (RING == 3) {
        FwdL R0, R1, R2;
        load_f(0, R0);
        load_f(N >= 2 ? 1 : 0, R1);
        for (int k = 0; k < N; k += 3) {
          load_f(k + 2 < N ? k + 2 : N - 1, R2);
          fstep(k, R0);
          if (k + 1 >= N) break;
          load_f(k + 3 < N ? k + 3 : N - 1, R0);
          fstep(k + 1, R1);
          if (k + 2 >= N) break;
          load_f(k + 4 < N ? k + 4 : N - 1, R1);
          fstep(k + 2, R2);
        }
      } else {
        FwdL R0, R1;
        load_f(0, R0);
        for (int k = 0; k < N; k += 2) {
          load_f(k + 1 < N ? k + 1 : N - 1, R1);
          fstep(k, R0);
          if (k + 1 >= N) break;
          load_f(k + 2 < N ? k + 2 : N - 1, R0);
          fstep(k + 1, R1);
        }
      }
    }
    if constexpr (MR) gsync();
    else wsync();
  };
  auto hinv = [&](double* dst, int jt) __attribute__((always_inline)) {
    if constexpr (ENT == 1 && ZC) {
      // one sweep body in the kernel: the MRHS form with a single row, its
      // column the destination (NB copied in first; dst is SV, ZV or VV)
      for (int i = lane; i < NV; i += RT) dst[i] = nb[i];
      wsync();
      double* const c1 = dst == zv ? sv : zv;   // rows >= 1 idle: any other LDS vector
      hinv_g(std::true_type{}, dst, jt, (lane >> 4) == 0 ? dst : c1, (lane >> 4) == 0, 1, dst, c1, c1, c1);
    } else {
      hinv_g(std::false_type{}, dst, jt, nullptr, false, 1, nullptr, nullptr, nullptr, nullptr);
    }
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
  // lane k: sum_{j <= k-2} zc (k-1-j) C_j X[fz_j] (the z-row of stage k over
  // X) = zc * (exclusive scan of the exclusive scan of C_j X[fz_j])
  // (the lane's stance flag once, not an LDS load ahead of X's in every call)
  const bool zst = lane < N && cc[lane < N ? lane : 0] != 0.0;
  auto zdot = [&](const double* X) -> double {
    const double xz = X[6 * (lane < N ? lane : 0) + 2];
    const double aj = zst ? xz : 0.0;
    const double e1 = wave_scan(aj) - aj;
    return zc * (wave_scan(e1) - e1);
  };

  RS_ACC(2, t_p2);
  RS_T(t_p3);
  // ---------------- phase 3: unconstrained optimum v0 = -H^-1 h --------------
  hinv(vv, N - 1);
  // |n| of the z rows (lane k): zc sqrt(sum_{j <= k-2, stance} (k-1-j)^2)
  {
    // the stance stages as one wave-uniform mask (N <= 64): the loop reads no
    // LDS, where one dependent load per stage cost a round trip each
    const uint64_t stm = __ballot(lane < N && cc[lane < N ? lane : 0] != 0.0);
    if (lane < N) {
      double s2 = 0.0;
      for (int j = 0; j + 2 <= lane; ++j) {
        const double cz = (double)(lane - 1 - j);
        if ((stm >> j) & 1) s2 = fma(cz, cz, s2);
      }
      znrm[lane] = zc * sqrt(s2);
    }
  }
  wsync();

  RS_ACC(3, t_p3);
  // ---------------- phase 4: dual active set --------------------------------
  // R lives in LDS (main pass) or global memory (overflow pass, ENT > 1)
  auto rsync = [&]() __attribute__((always_inline)) {
    if constexpr (ENT > 1) gsync();
    else wsync();
  };
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
  // last stage a constraint row touches: its own stage k, or k - 2 for the
  // z row of stage k (fz_j, j <= k - 2)
  auto stage_top = [](int id) -> int {
    const int v = id >> 2, k = v / 6, c = v - 6 * k;
    return (c >= 3 && (id & 3) >= 2) ? k - 2 : k;
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

  // MRHS candidate cache (global, after the active columns): lane t < kNSC
  // holds the id whose s = H^-1 n_id sits in slot t (-1: empty)
  [[maybe_unused]] int cid = -1;
  [[maybe_unused]] int cnext = 0;
  bool done = status != ST_SOLVED;
  while (!done) {
    RS_T(t_scan);
    // ---- slacks of my stage's constraints; the most violated ----
    const double vz = zdot(vv);
    double best = INFINITY;
    int bid = 0x7fffffff;
    // the main-pass kernels combine by selects, not exec-masked branches
    // (round 5: N = 60 +3 %, configs[3] +1.7 %, less scratch at the 2-wave
    // cap); the overflow pass (ENT > 1) keeps the branch form
    constexpr bool kSel = ENT == 1;
    auto comb = [&](bool c, double v, int i) __attribute__((always_inline)) {
      if constexpr (kSel) argmin_combine_sel(best, bid, c ? v : INFINITY, c ? i : 0x7fffffff);
      else if (c) argmin_combine(best, bid, v, i);
    };
    if (lane < N) {
      const int k = lane;
      double u[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) u[c] = vv[6 * k + c];
#pragma unroll
      for (int c = 3; c < 6; ++c) {
        const double lim = tau_lim(c);
        const int v = 6 * k + c;
        comb(!(amask & (1 << (4 * c))), u[c] + lim, 4 * v);
        comb(!(amask & (1 << (4 * c + 1))), lim - u[c], 4 * v + 1);
      }
      if (k >= 2) {
        const double zrow = (zb[k] - kZmin) + vz;
        const double zn = znrm[k];
        const double s2 = zn > 0.0 ? zrow / zn : ((zrow < -kTol) ? -INFINITY : INFINITY);
        comb(!(amask & (1 << 14)), s2, 4 * (6 * k + 3) + 2);
      }
      if (stance_me) {
        const int v = 6 * k + 2;
        comb(!(amask & (1 << 8)), u[2], 4 * v);
        comb(!(amask & (1 << 9)), kFzMax - u[2], 4 * v + 1);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          if (VAR == 2 && c == 1) continue;
          const int vc = 6 * k + c;
          comb(!(amask & (1 << (4 * c))), (mu * u[2] - u[c]) * inv01, 4 * vc);
          comb(!(amask & (1 << (4 * c + 1))), (mu * u[2] + u[c]) * inv01, 4 * vc + 1);
        }
      }
    }
    [[maybe_unused]] const double lbest = best;   // this stage's most violated (MRHS candidates)
    [[maybe_unused]] const int lbid = bid;
    wave_argmin<kSel>(best, bid);
    RS_ACC(4, t_scan);
    if (!(best < -kTol)) break;   // primal feasible: optimal
    RS_T(t_s);
    const int p = uni(bid);
    const double bp = rhs_of(p);
    // n_p -> NB
    for (int j = lane; j < N; j += RT) {
      double acc[6] = {0, 0, 0, 0, 0, 0};
      add_coef(p, j, 1.0, acc);
#pragma unroll
      for (int c = 0; c < 6; ++c) nb[6 * j + c] = acc[c];
    }
    rsync();
    if constexpr (kMR) {
      // s = H^-1 n_p from the candidate cache, or by one multi-RHS sweep pair
      // that also fills the cache for the next most violated constraints of
      // other stages (MRHS)
      const uint64_t hit = __ballot(lane < kNSC && cid == p);
      if (hit) {
        if constexpr (PART == 2) RS_CNT(12, 1);
        const double* col = gcache + (int64_t)__builtin_ctzll(hit) * NV;
        if constexpr (NC > 0) {
          // every load of the column in flight before the first store (round
          // 6: the loop's load -> store pairs were serial round trips)
          constexpr int CE = (6 * NC + RT - 1) / RT;
          double cv[CE];
#pragma unroll
          for (int e = 0; e < CE; ++e) cv[e] = col[lane + RT * e < NV ? lane + RT * e : 0];
#pragma unroll
          for (int e = 0; e < CE; ++e)
            if (lane + RT * e < NV) sv[lane + RT * e] = cv[e];
        } else {
          for (int i = lane; i < NV; i += RT) sv[i] = col[i];
        }
        wsync();
      } else {
        // candidates: each stage's most violated constraint (lanes < N), not
        // p, not cached already; the most violated of those first
        bool cached = false;
        for (int t = 0; t < kNSC; ++t) cached = cached || (__builtin_amdgcn_readlane(cid, t) == lbid);
        double bl = (lane < N && lbest < -kTol && lbid != p && !cached) ? lbest : INFINITY;
        int ids[kMRK], sl[kMRK];
        ids[0] = p;
        int nr = 1, jt = stage_top(p);
#pragma unroll
        for (int r = 1; r < kMRK; ++r) {
          double b2 = bl;
          int i2 = lbid;
          wave_argmin<ENT == 1>(b2, i2);
          if (!(b2 < -kTol)) break;
          const int q2 = uni(i2);
          if (lbid == q2) bl = INFINITY;
          ids[r] = q2;
          jt = max(jt, stage_top(q2));
          nr = r + 1;
        }
        for (int r = 0; r < kMRK; ++r) {   // cache slots, round robin
          if (r < nr) {
            sl[r] = cnext;
            if (lane == cnext) cid = ids[r];
            cnext = cnext + 1 == kNSC ? 0 : cnext + 1;
          } else {
            sl[r] = sl[0];
          }
        }
        const int row = lane >> 4;
        if constexpr (PART == 2) { RS_CNT(11, 1); RS_CNT(14, nr); }
        if constexpr (kMRL) {
          // the four columns in LDS vectors that are dead during this sweep
          // pair: SV (row 0, so s lands in place), ZV, MU and the union's
          // Riccati scratch (568 >= 6N doubles); then to their cache slots
          auto colr = [&](int r) -> double* { return r == 0 ? sv : r == 1 ? zv : r == 2 ? mu_ : un; };
          for (int r = 0; r < nr; ++r) {
            double* col = colr(r);
            for (int j = lane; j < N; j += RT) {
              double acc[6] = {0, 0, 0, 0, 0, 0};
              add_coef(ids[r], j, 1.0, acc);
#pragma unroll
              for (int c = 0; c < 6; ++c) col[6 * j + c] = acc[c];
            }
          }
          wsync();
          hinv_g(std::true_type{}, sv, jt, colr(row), row < nr, nr, sv, zv, mu_, un);
          for (int r = 0; r < nr; ++r) {
            const double* col = colr(r);
            double* gc = gcache + (int64_t)sl[r] * NV;
            for (int i = lane; i < NV; i += RT) gc[i] = col[i];
          }
          gsync();
        } else {
          // right-hand sides n_q into their cache columns (global)
          for (int r = 0; r < nr; ++r) {
            double* col = gcache + (int64_t)sl[r] * NV;
            for (int j = lane; j < N; j += RT) {
              double acc[6] = {0, 0, 0, 0, 0, 0};
              add_coef(ids[r], j, 1.0, acc);
#pragma unroll
              for (int c = 0; c < 6; ++c) col[6 * j + c] = acc[c];
            }
          }
          gsync();
          const int myslot = row == 0 ? sl[0] : row == 1 ? sl[1] : row == 2 ? sl[2] : sl[3];
          hinv_g(std::true_type{}, gcache, jt, gcache + (int64_t)myslot * NV, row < nr, nr,
                 gcache + (int64_t)sl[0] * NV, gcache + (int64_t)sl[1] * NV, gcache + (int64_t)sl[2] * NV,
                 gcache + (int64_t)sl[3] * NV);
          const double* col = gcache + (int64_t)sl[0] * NV;
          for (int i = lane; i < NV; i += RT) sv[i] = col[i];
          wsync();
        }
      }
    } else {
      hinv(sv, stage_top(p));       // s = H^-1 n_p
    }
    const double sn = vdot(nb, sv);
    const double szd = zdot(sv);
    if (lane < N) zd[lane] = szd;
    rsync();
    RS_ACC(5, t_s);
    double uplus = 0.0;
    // ---- inner loop: step towards satisfying constraint p ----
    while (true) {
      if (++iters > max_iter) { status = ST_MAXIT; done = true; break; }
      RS_T(t_c);
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
      // the reciprocals of R's diagonal first (one division per lane), so the
      // substitutions' chains are readlane -> mul -> fma (round 5)
      double rinv[ENT];
#pragma unroll
      for (int e = 0; e < ENT; ++e) {
        const int m = 64 * e + lane < q ? 64 * e + lane : 0;
        rinv[e] = 1.0 / Rm[loff(m) + m];
      }
      constexpr bool kSelU = ENT == 1;   // (selects in the main-pass kernels, as the scan)
      for (int l = 0; l < q; ++l) {   // forward substitution with R'
        const double yl = vget(yv, l) * vget(rinv, l);
        vset(yv, l, yl);
#pragma unroll
        for (int e = 0; e < ENT; ++e) {
          const int m = 64 * e + lane;
          if constexpr (kSelU) {
            const bool up = m > l && m < q;
            const double rv_ = Rm[loff(up ? m : l) + l];
            yv[e] = up ? fma(-rv_, yl, yv[e]) : yv[e];
          } else if (m > l && m < q) {
            yv[e] = fma(-Rm[loff(m) + l], yl, yv[e]);
          }
        }
      }
#pragma unroll
      for (int e = 0; e < ENT; ++e) rv[e] = yv[e];
      for (int l = q - 1; l >= 0; --l) {   // back substitution with R
        const double rl = vget(rv, l) * vget(rinv, l);
        vset(rv, l, rl);
#pragma unroll
        for (int e = 0; e < ENT; ++e) {
          const int m = 64 * e + lane;
          if constexpr (kSelU) {
            const double r_ = Rm[loff(l) + (m < l ? m : 0)];
            rv[e] = m < l ? fma(-r_, rl, rv[e]) : rv[e];
          } else if (m < l) {
            rv[e] = fma(-Rm[loff(l) + m], rl, rv[e]);
          }
        }
      }
      // z = H^-1 (n_p - N_A r), n_z' z
      RS_ACC(6, t_c);
      RS_T(t_z);
      const double* zsrc = sv;
      double zn = sn;
      if (q > 0) {
        // r to LDS first: the per-stage loop below runs on lanes < N only,
        // and a readlane from a lane outside it would read a stale register
#pragma unroll
        for (int e = 0; e < ENT; ++e) {
          const int ai = 64 * e + lane;
          if (ai < q) cbv[ai] = rv[e];
        }
        rsync();
        // n_z = n_p - N_A r is formed only for the sweep fallback below: the
        // step's n_z'z equals n_p'z (N_A'z = c - R'R r = 0), the classic
        // Goldfarb-Idnani denominator, so NB keeps n_p (round 6: the
        // per-stage loop over every active row cost ~20 % of this phase at
        // N = 60, where the fallback runs 0.006 times per instance)
        auto nz_to_nb = [&]() __attribute__((always_inline)) {
          for (int j = lane; j < N; j += RT) {
            double acc[6] = {0, 0, 0, 0, 0, 0};
            add_coef(p, j, 1.0, acc);
            for (int ai = 0; ai < q; ++ai) add_coef(act[ai], j, -cbv[ai], acc);
#pragma unroll
            for (int c = 0; c < 6; ++c) nb[6 * j + c] = acc[c];
          }
          rsync();
        };
        bool sweep = !ZC;
        // the batched form: the one-wave kernels, and (round 6) the 3f
        // two-wave ones -- configs[3] 13.45 -> 13.71 M at 12 -> 20 B/lane of
        // scratch; in the 2f two-wave kernels it spilled 32 B/lane
        if constexpr (ZC && (RING != 2 || VAR == 3)) {   // 
          // z = s - S r streamed column by column, each lane's ZE entries
          // i = i0 + lane + 64 e side by side: 4 x ZE independent loads in flight
          // per lane per batch of 4 columns (the latency of the L2/MALL-resident
          // columns, not the FMAs, bounds this phase)
          constexpr int ZE = NC > 0 ? (6 * NC + RT - 1) / RT : (RING == 2 ? 2 : 6);
          for (int i0 = 0; i0 < NV; i0 += RT * ZE) {
            double za[ZE], zb2[ZE];
            const double* sc[ZE];
#pragma unroll
            for (int e = 0; e < ZE; ++e) {
              const int i = i0 + lane + RT * e, ic = i < NV ? i : 0;
              sc[e] = scw + ic;
              za[e] = sv[ic];
              zb2[e] = 0.0;
            }
            // whole batches of KB columns, the last one padded by a repeated
            // column with coefficient 0: one memory round trip per batch
            // (round 6: the one-column tail loop waited for up to 3 serial
            // round trips per iteration; N = 60 B = 4096: the z phase 218 k ->
            // 67 k cycles per instance, 1.83 -> 1.96 M solves/s; 4-column
            // padded batches 1.94 M.  In the two-wave kernels 4-column
            // batches of both entries per lane, ZE = 2: configs[3] +1.9 %)
            constexpr int KB = RING == 2 ? 4 : 8;
            for (int a0 = 0; a0 < q; a0 += KB) {
              double rr[KB], c[ZE][KB];
#pragma unroll
              for (int t = 0; t < KB; ++t) {
                const int a = a0 + t < q ? a0 + t : q - 1;
                rr[t] = a0 + t < q ? cbv[a] : 0.0;
#pragma unroll
                for (int e = 0; e < ZE; ++e) c[e][t] = sc[e][(int64_t)a * NV];
              }
#pragma unroll
              for (int e = 0; e < ZE; ++e) {
#pragma unroll
                for (int t = 0; t < KB; t += 2) {
                  za[e] = fma(-rr[t], c[e][t], za[e]);
                  zb2[e] = fma(-rr[t + 1], c[e][t + 1], zb2[e]);
                }
              }
            }
#pragma unroll
            for (int e = 0; e < ZE; ++e) {
              const int i = i0 + lane + RT * e;
              if (i < NV) zv[i] = za[e] + zb2[e];
            }
          }
          rsync();
          zn = vdot(nb, zv);
          sweep = !(zn > kZcRel * sn);
        } else if constexpr (ZC) {
          for (int i = lane; i < NV; i += RT) {
            const double* sc = scw + i;
            double z0 = sv[i], z1 = 0.0;
            int a0 = 0;
            for (; a0 + 4 <= q; a0 += 4) {
              const double c0 = sc[(int64_t)a0 * NV], c1 = sc[(int64_t)(a0 + 1) * NV];
              const double c2 = sc[(int64_t)(a0 + 2) * NV], c3 = sc[(int64_t)(a0 + 3) * NV];
              z0 = fma(-cbv[a0], c0, z0);
              z1 = fma(-cbv[a0 + 1], c1, z1);
              z0 = fma(-cbv[a0 + 2], c2, z0);
              z1 = fma(-cbv[a0 + 3], c3, z1);
            }
            for (; a0 < q; ++a0) z0 = fma(-cbv[a0], sc[(int64_t)a0 * NV], z0);
            zv[i] = z0 + z1;
          }
          rsync();
          // the cached form cancels in H^-1 space: when n_z'z is small against
          // n_p'H^-1 n_p the result is recomputed by the sweeps
          zn = vdot(nb, zv);
          sweep = !(zn > kZcRel * sn);
        }
        if (sweep) {
          int tz = stage_top(p);   // n_p - N_A r: the last stage of p and the active rows
#pragma unroll
          for (int e = 0; e < ENT; ++e) {
            const int ai = 64 * e + lane;
            if (ai < q) tz = max(tz, stage_top(act[ai]));
          }
          if constexpr (PART == 2) RS_CNT(13, 1);
          nz_to_nb();
          hinv(zv, wave_imax63(tz));
          zn = vdot(nb, zv);
          // NB back to n_p for the next pass of the inner loop
          for (int j = lane; j < N; j += RT) {
            double acc[6] = {0, 0, 0, 0, 0, 0};
            add_coef(p, j, 1.0, acc);
#pragma unroll
            for (int c = 0; c < 6; ++c) nb[6 * j + c] = acc[c];
          }
          rsync();
        }
        zsrc = zv;
      }
      RS_ACC(7, t_z);
      RS_T(t_u);
      // partial step t1 (drop candidate) over r > 0
      double t1 = INFINITY;
      int kdrop = 0x7fffffff;
#pragma unroll
      for (int e = 0; e < ENT; ++e) {
        const int ai = 64 * e + lane;
        if constexpr (ENT == 1) {
          const bool c = ai < q && rv[e] > 0.0;
          argmin_combine_sel(t1, kdrop, c ? ua[ai < q ? ai : 0] / rv[e] : INFINITY, c ? ai : 0x7fffffff);
        } else if (ai < q && rv[e] > 0.0) {
          argmin_combine(t1, kdrop, ua[ai] / rv[e], ai);
        }
      }
      wave_argmin<ENT == 1>(t1, kdrop);
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
      rsync();
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
        if constexpr (ZC)   // cache S_q = H^-1 n_p (each lane its own entries)
          for (int i = lane; i < NV; i += RT) scw[(int64_t)q * NV + i] = sv[i];
        ++q;
        rsync();
        RS_ACC(8, t_u);
        break;
      }
      // ---- drop kdrop: delete its column of R, restore the triangle ----
      {
        const int k = uni(kdrop);
        const int idk = act[k];
        RS_CNT(15, (1LL << 32) + (q - k - 1));   // (stamped builds: drops, cached columns shifted)
        if (lane == (idk >> 2) / 6) amask &= ~(1 << (4 * ((idk >> 2) % 6) + (idk & 3)));
        if constexpr (ZC)   // the cached columns follow the active order
          for (int m = k; m + 1 < q; ++m)
            for (int i = lane; i < NV; i += RT) scw[(int64_t)m * NV + i] = scw[(int64_t)(m + 1) * NV + i];
        for (int m = k; m + 1 < q; ++m) {   // shift columns m+1 -> m, keep subdiagonals
          for (int i0 = 0; i0 <= m + 1; i0 += RT) {
            const int i = i0 + lane;
            const double val = i <= m + 1 ? Rm[loff(m + 1) + i] : 0.0;
            rsync();
            if (i <= m) Rm[loff(m) + i] = val;
            if (i == m + 1) sdg[m] = val;
            rsync();
          }
        }
        for (int i0 = k; i0 + 1 < q; i0 += RT) {   // shift the active list
          const int i = i0 + lane;
          int an = 0;
          double un_ = 0.0;
          if (i + 1 < q) { an = act[i + 1]; un_ = ua[i + 1]; }
          rsync();
          if (i + 1 < q) { act[i] = an; ua[i] = un_; }
          rsync();
        }
        for (int l = k; l + 1 < q; ++l) {   // Givens on rows (l, l+1)
          const double aa = Rm[loff(l) + l], bb = sdg[l];
          const double hh = sqrt(aa * aa + bb * bb);
          const double cg = hh != 0.0 ? aa / hh : 1.0, sg = hh != 0.0 ? bb / hh : 0.0;
          rsync();
          if (lane == 0) Rm[loff(l) + l] = hh;
          for (int i0 = 0; i0 < q; i0 += RT) {
            const int mcol = i0 + lane;   // columns m > l hold rows l, l+1
            if (mcol > l && mcol + 1 < q) {
              const double rl = Rm[loff(mcol) + l], rl1 = Rm[loff(mcol) + l + 1];
              Rm[loff(mcol) + l] = cg * rl + sg * rl1;
              Rm[loff(mcol) + l + 1] = -sg * rl + cg * rl1;
            }
          }
          rsync();
        }
        q = q - 1;
        rsync();
        RS_ACC(8, t_u);
      }
    }
  }

  RS_T(t_p5);
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
  // x_ref into the union again (over the dead R), x* staged over SV..
  stage_xref();
  for (int i = lane; i < NV; i += RT) {
    const int j = i / 6, c = i - 6 * j;
    const bool fr = c >= 3 || (cc[j] != 0.0 && !(VAR == 2 && c == 1));
    const double u = (status == ST_SOLVED && fr) ? vv[i] : 0.0;
    vv[i] = u;
    a.u[b * NV + i] = u;
  }
  wsync();
  double* xo = sv;   // 12 (N+1) <= 4 NV doubles (SV, NB, ZV, MU)
  {
    double xr = lane < 12 ? xin[lane] : 0.0;
    if (lane < 12) xo[lane] = xr;
    const double qr = qdiag(lane);
    const double ub_alias = (cc[N - 1] != 0.0) ? 2.0 * a.m * a.g : 0.0;
    double objl = 0.0;
    // the one-wave kernels: every lane loads its stage inputs (no divergent
    // loads): lanes 9-11 their row of the omega block, lanes < 12 their x_ref
    // entry, lanes < 6 their input; stage k+1's loads are issued before stage
    // k's x store, which the compiler cannot move them across (one LDS round
    // trip per stage on the rollout's chain otherwise).  The two-wave kernels,
    // at their register cap, keep the plain loop (56 vs 24 B/lane of scratch).
    if constexpr (RING == 3) {
      const int rw = (lane >= 9 && lane < 12) ? lane - 9 : 0;
      const int l12 = lane < 12 ? lane : 0, l6 = lane < 6 ? lane : 0;
      struct Stage { double cp, sp, u[6], bwr[6], xr, ul, cck; };
      auto load_stage = [&](int k, Stage& s) __attribute__((always_inline)) {
        s.cp = cs[2 * k];
        s.sp = cs[2 * k + 1];
#pragma unroll
        for (int c = 0; c < 6; ++c) s.u[c] = vv[6 * k + c];
#pragma unroll
        for (int c = 0; c < 6; ++c) s.bwr[c] = bw[18 * k + 6 * rw + c];
        s.xr = un[12 * k + l12];
        s.ul = vv[6 * k + l6];
        s.cck = cc[k];
      };
      Stage cur, nxt;
      load_stage(0, cur);
      for (int k = 0; k < N; ++k) {
        load_stage(k + 1 < N ? k + 1 : k, nxt);
        const double cp = cur.cp, sp = cur.sp;
        const double u0 = cur.u[0], u1 = cur.u[1], u2 = cur.u[2], u3 = cur.u[3], u4 = cur.u[4], u5 = cur.u[5];
        double nx = ad_lane(xr, dt, cp, sp, lane) + ((lane == 8) ? -a.g * dt : 0.0);
        if (lane >= 6 && lane < 9) {
          const int r = lane - 6;
          nx += bv<VAR>(r, 0, dtm, cp, sp) * u0 + bv<VAR>(r, 1, dtm, cp, sp) * u1 + bv<VAR>(r, 2, dtm, cp, sp) * u2;
        } else if (lane >= 9 && lane < 12) {
          const double* bwr = cur.bwr;
          nx += ((bwr[0] * u0 + bwr[1] * u1) + (bwr[2] * u2 + bwr[3] * u3)) + (bwr[4] * u4 + bwr[5] * u5);
        }
        xr = lane < 12 ? nx : 0.0;
        const double kf = (k == N - 1) ? kTermQ : 1.0;
        const double e = lane < 12 ? xr - cur.xr : 0.0;
        objl = fma(kf * qr * e, e, objl);
        if (k < N - 1 && lane < 6) {
          const double ub = a.uref_aliased ? ub_alias : ((cur.cck != 0.0) ? 2.0 * a.m * a.g : 0.0);
          const double du = cur.ul - (lane == 2 ? ub : 0.0);
          objl = fma(kRdiag * du, du, objl);
        }
        if (lane < 12) xo[12 * (k + 1) + lane] = xr;
        cur = nxt;
      }
    } else {
      for (int k = 0; k < N; ++k) {
        const double cp = cs[2 * k], sp = cs[2 * k + 1];
        const double* uk = vv + 6 * k;
        const double u0 = uk[0], u1 = uk[1], u2 = uk[2], u3 = uk[3], u4 = uk[4], u5 = uk[5];
        double nx = ad_lane(xr, dt, cp, sp, lane) + ((lane == 8) ? -a.g * dt : 0.0);
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
    }
    const double objv = wave_sum(objl);
    wsync();
#ifdef HMPC_STAMPS
    RS_ACC(9, t_p5);
    RS_ACC(10, t_all);
    if (a.x && lane == 0)
      for (int i = 0; i < 16; ++i) reinterpret_cast<long long*>(a.x)[b * 12 * (N + 1) + i] = rst_[i];
#else
    if (a.x)
      for (int i = lane; i < 12 * (N + 1); i += RT) a.x[b * 12 * (N + 1) + i] = xo[i];
#endif
    if (lane == 0) {
      if (a.obj) a.obj[b] = objv;
      a.status[b] = status;
      if (a.iters) a.iters[b] = iters;
      if (a.active) a.active[b] = q;
    }
  }
}

// Persistent: a.ric_groups workgroups, each with its slot of the K / Dinv
// workspace, take instances off an atomic counter (a.work, zeroed with the
// overflow count before the launch) until the batch is done.
// OCC = waves per SIMD the register allocation is held to (2: <= 256 VGPRs +
// AGPRs; 1: up to 512)
// sweep prefetch depth (ring slots) at 1 wave/SIMD
constexpr int kRing1Wave = 3;   // (4-6 slots measured slower)
// ... and at 2 waves/SIMD (register budget 256)
constexpr int kRing2Wave = 2;
// PART 2: the factorisation kernel has run, K / Dinv per
// instance in a.kinst; the workgroup's slot keeps only the cached columns.
template <int VAR, int OCC, int NC = 0, int CAPC = 0, int PART = 0>
__global__ void __launch_bounds__(RT) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) ric_kernel(SolveArgs a, int N, int cap) {
  extern __shared__ __attribute__((aligned(16))) double ric_sm[];
  if constexpr (NC > 0) { N = NC; cap = CAPC; }
  const RicLay L(N, cap, true);
  double* kw = a.kws + (int64_t)blockIdx.x * a.kws_stride;
  while (true) {
    int b = 0;
    if constexpr (OCC == 1) {
      if (threadIdx.x == 0) b = atomicAdd(a.work, 1);
      // longest-first queue: ticket b in the stance buckets, highest first;
      // the bucket counts load beside the ticket, one per lane (round 6:
      // lane 0 walked them one serial round trip per bucket; the 2-wave
      // kernels keep that form, whose registers sit at the 256 cap)
      const int bc = a.list && (int)threadIdx.x < a.split_nbkt ? a.list_count[threadIdx.x] : 0;
      // (a.work_bound: the tickets of a list shorter than the batch -- the
      // N = 60 second-tier pass over the main pass's overflow list)
      const int bound = a.work_bound ? *a.work_bound : (int)a.B;
      b = __builtin_amdgcn_readfirstlane(b);
      if (b >= bound) break;
      if (a.list) {
        int s = a.split_nbkt - 1;
        for (; s > 0; --s) {
          const int c = __builtin_amdgcn_readlane(bc, s);
          if (b < c) break;
          b -= c;
        }
        b = a.list[(int64_t)s * a.B + b];
      }
    } else {
      if (threadIdx.x == 0) {
        b = atomicAdd(a.work, 1);
        if (a.list && b < a.B) {   // longest-first queue: ticket b in the stance buckets, highest first
          int s = a.split_nbkt - 1;
          for (; s > 0; --s) {
            const int c = a.list_count[s];
            if (b < c) break;
            b -= c;
          }
          b = a.list[(int64_t)s * a.B + b];
        }
      }
      b = __builtin_amdgcn_readfirstlane(b);
    }
    if (b >= a.B) break;
    double* kwi = PART == 2 ? a.kinst + (int64_t)b * a.kinst_stride : kw;
    ric_solve<VAR, 1, OCC == 2 ? kRing2Wave : kRing1Wave, true, NC, CAPC, PART>(a, N, (int64_t)b, ric_sm, ric_sm + L.RM,
                                                                               cap, kwi, kw + ric_kws_doubles(N));
    __syncthreads();
  }
}

// The factorisation kernel (ric_kinst_stride): one workgroup per instance,
// phases 0 and 2 of ric_solve into the instance's K / Dinv block of a.kinst.
// Few registers and 21 N + max(568, 12 N) doubles of LDS, so several waves
// per SIMD share the factorisation's dependent chains, which the
// one-instance-per-wave solve kernel leaves latency-bound.
// 3 waves / SIMD: 162 VGPRs, no spill (4: 128 B/lane of spill, -10 % at
// configs[3])
template <int VAR, int NC = 0, int CAPC = 0>
__global__ void __launch_bounds__(RT) __attribute__((amdgpu_waves_per_eu(3)))
ric_factor_kernel(SolveArgs a, int N, int cap) {
  extern __shared__ __attribute__((aligned(16))) double ric_sm[];
  if constexpr (NC > 0) { N = NC; cap = CAPC; }
  const int64_t b = blockIdx.x;
  ric_solve<VAR, 1, kRing2Wave, true, NC, CAPC, 1>(a, N, b, ric_sm, nullptr, cap, a.kinst + b * a.kinst_stride, nullptr);
}

// the overflow pass: instances listed in a.ovf_list, capacity 6N, R and the
// K / Dinv workspace in the global block of the workgroup (rws_stride doubles)
template <int VAR>
__global__ void __launch_bounds__(RT) ric_overflow_kernel(SolveArgs a, int N) {
  extern __shared__ __attribute__((aligned(16))) double ric_sm[];
  const int n = *a.ovf_count;
  // the header holding the split counts: the first one when the fp64 dense
  // fallback pass ran in between (a.ovf_hdr1, HMPC_PREC_F32_REFINED), whose
  // instances the running total counts (this pass re-solves a subset of them)
  int32_t* const h1 = a.ovf_hdr1 ? a.ovf_hdr1 : a.ovf_count;
  if (n == 0) {
    // nothing to re-solve (the usual case): no block depends on the counters
    // any more, so block 0 zeroes them at once, without the done counter's
    // one serialised atomic per workgroup
    if (blockIdx.x == 0) {
      // (thread 0 reads the first count before it zeroes it itself)
      if (a.ovf_hdr1 && threadIdx.x == 0 && a.ovf_total) atomicAdd(a.ovf_total, (unsigned long long)h1[0]);
      if ((int)threadIdx.x < 3) a.ovf_count[threadIdx.x] = 0;
      if ((int)threadIdx.x < 3 + a.split_nbkt) h1[threadIdx.x] = 0;
    }
    return;
  }
  double* Rm = a.rws + (int64_t)blockIdx.x * a.rws_stride;
  double* kw = Rm + (a.rws_stride - ric_kws_doubles(N));
  SolveArgs a2 = a;
  a2.ovf_count = nullptr;   // no further overflow: capacity is 6N
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int64_t b = a.ovf_list[i];
    ric_solve<VAR, (6 * kRicNmax + 63) / 64, 3, false>(a2, N, b, ric_sm, Rm, 6 * N, kw, nullptr);
    __syncthreads();
  }
  // the last workgroup out zeroes [overflow count | instance counter | its
  // own done counter | the dense split's counts] for the next solve on this stream (every group read
  // the count above before it counts itself done): no memset per solve
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(a.ovf_count + 2, 1) == (int)gridDim.x - 1) {
      if (a.ovf_total) atomicAdd(a.ovf_total, (unsigned long long)(a.ovf_hdr1 ? h1[0] : n));
      atomicExch(a.ovf_count, 0);
      atomicExch(a.ovf_count + 1, 0);
      atomicExch(a.ovf_count + 2, 0);
      if (a.ovf_hdr1)
        for (int i = 0; i < 3; ++i) atomicExch(h1 + i, 0);
      for (int i = 0; i < a.split_nbkt; ++i) atomicExch(h1 + 3 + i, 0);   // the dense split's counts
    }
  }
}

// The longest-first work queue (a.lpt: a few instances per workgroup, where
// the queue's last round is the tail): every instance's stance stages are
// counted and the instance is appended to bucket nst / W (W stages per
// bucket, nb <= kLptMax buckets at split_list[bucket * B ..], lengths in
// split_count[bucket], zero at the launch; the overflow pass zeroes them).
// The kernel then serves the buckets from the most stance stages down.
// Each wave counts its 64 instances row by row: lane j < N reads C[i][j], one
// coalesced row per load and a ballot (round 5; one thread per instance
// walking its own row was 64 uncoalesced loads per instruction and 50 us per
// N = 60 step at B = 4096).  All 64 row loads are issued before
// the first ballot, and a workgroup is one wave (B = 4096: 64 CUs, 64 atomics
// per bucket counter): 9.3 us at N = 60 B = 4096, of which probe builds put
// ~3.7 us on the C reads, ~1.6 us on the counters and ~4 us on the launch
// itself (1024-thread groups: 78 us -- the per-CU load rate).  Run beside
// the factorisation kernel on a second stream it saved nothing at N = 60
// B = 4096 (1.597 vs 1.603 M, the fork / join costs what it hides).
constexpr int kLptT = 64;
constexpr int kLptMax = 13;
static_assert(kRicNmax <= 64, "a C row per wave load");   // bucket counters in the overflow header (hmpc_capi.cpp)
__global__ void __launch_bounds__(kLptT) ric_buckets_kernel(SolveArgs a, int N, int W) {
  __shared__ int wc[kLptT / 64][kLptMax];
  __shared__ int base[kLptMax];
  const int nb = a.split_nbkt;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * kLptT + 64 * w;   // this wave's 64 instances
  const int64_t i = i0 + lane;
  const bool in = i < a.B;
  int nst = 0;
  const int64_t last = a.B - 1;
  const int col = lane < N ? lane : 0;
  double cv[64];
#pragma unroll
  for (int u = 0; u < 64; ++u) {
    const int64_t ir = i0 + u;
    cv[u] = a.C[(ir < last ? ir : last) * a.C_bs + col];
  }
#pragma unroll
  for (int u = 0; u < 64; ++u) {
    const bool ok = i0 + u <= last && lane < N;
    const int cnt = __builtin_popcountll(__ballot(ok && cv[u] != 0.0));
    nst = lane == u ? cnt : nst;
  }
  const int k = in ? min(nst / W, nb - 1) : 0;
  uint64_t mine = 0;
  for (int s = 0; s < nb; ++s) {
    const uint64_t m = __ballot(in && k == s);
    mine = (in && k == s) ? m : mine;
    if (lane == 0) wc[w][s] = __builtin_popcountll(m);
  }
  __syncthreads();
  if (threadIdx.x < nb) {   // thread s: exclusive scan of bucket s over the waves, one atomic
    const int s = threadIdx.x;
    int t = 0;
    for (int v = 0; v < kLptT / 64; ++v) {
      const int c = wc[v][s];
      wc[v][s] = t;
      t += c;
    }
    base[s] = t ? atomicAdd(a.split_count + s, t) : 0;
  }
  __syncthreads();
  if (in)
    a.split_list[(int64_t)k * a.B + base[k] + wc[w][k] + __builtin_popcountll(mine & ((1ull << lane) - 1))] =
        (int32_t)i;
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

namespace {
constexpr size_t kLdsPerCU = 160 * 1024;
struct RicCfg {
  int cap, occ;
};
RicCfg ric_config(int N) {
  const int nv = 6 * N, cmax = nv < 64 ? nv : 64, cmin = nv < 32 ? nv : 32;
  for (int occ = 2; occ >= 1; --occ) {
    const size_t budget = kLdsPerCU / (4 * occ);
    for (int c = cmax; c >= cmin; --c)
      if (ric_lds_bytes(N, c) <= budget) return {c, occ};
  }
  return {cmin, 1};
}
}  // namespace

int ric_qcap(int N) { return ric_config(N).cap; }
int ric_occ(int N) { return ric_config(N).occ; }
int ric_static_n(int N) {
  const RicCfg c = ric_config(N);
  if (N == 60 && c.occ == 1 && c.cap == 47) return 60;
  if (N == 20 && c.occ == 2 && c.cap == 38) return 20;
  return 0;
}

// The Runner's horizon at small batches (round 6): the solve kernel with R's
// capacity 64 (48.8 KB of LDS, 3 workgroups per CU) when every instance
// gets its own workgroup at that occupancy anyway.  The Runner's own
// trajectory (the reference's configs[0] run) has calls with 48-59 active
// rows, which capacity 47 handed to the generic capacity-6N overflow pass at
// ~7 ms each: 41 of the single robot's 108 ms per run.
constexpr int kSmallCap60 = 64;

int ric_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  return cus;
}
int ric_qcap_batch(int N, int64_t B) {
  if (ric_static_n(N) == 60 && B <= 3 * (int64_t)ric_cus() && ric_kinst_stride(N, B) > 0) return kSmallCap60;
  return ric_qcap(N);
}

// K / Dinv of every stage, then the cached columns H^-1 n_a (capacity x NV),
// then the MRHS candidate columns (kNSC x NV)
int64_t ric_kws_stride(int N) {
  const int cap = ric_static_n(N) == 60 ? kSmallCap60 : ric_qcap(N);
  return ric_kws_doubles(N) + (((((int64_t)cap + kNSC) * 6 * N) + 15) & ~(int64_t)15);
}

int64_t ric_rws_stride(int N) {
  const int64_t nv = 6 * (int64_t)N;
  return (((nv * (nv + 1) / 2) + 15) & ~(int64_t)15) + ric_kws_doubles(N);
}

namespace {
template <typename K>
bool ric_launch_k(K kern, int N, int cap, const SolveArgs& a, hipStream_t s, int* per) {
  const size_t lds = ric_lds_bytes(N, cap);
  if (!set_lds(kern, lds)) return false;
  if (per) return hipOccupancyMaxActiveBlocksPerMultiprocessor(per, kern, RT, lds) == hipSuccess;
  const unsigned g = (unsigned)(a.B < a.ric_groups ? a.B : a.ric_groups);
  hipLaunchKernelGGL(kern, dim3(g), dim3(RT), lds, s, a, N, cap);
  return true;
}
// the Runner's horizon N = 60 and configs[3]'s N = 20 have compile-time
// instantiations, used when the host-side configuration matches the one they
// were built for: +7 % at N = 60 (B = 4096), +1.4 % at N = 20 (B = 262144;
// 12 B/lane of scratch at the 2-wave 256-VGPR cap since the round-2 register
// savings -- it lost 6 % when it spilled more)
// the factorisation kernel, one workgroup per instance
template <typename K>
bool ric_launch_fac(K kern, int N, int cap, const SolveArgs& a, hipStream_t s) {
  const size_t lds = (size_t)RicLay(N, cap, false, true).total * sizeof(double);
  if (!set_lds(kern, lds)) return false;
  hipLaunchKernelGGL(kern, dim3((unsigned)a.B), dim3(RT), lds, s, a, N, cap);
  return true;
}
// the N = 60 second-tier pass: the capacity-64 solve kernel over a list
// (a.list, count *a.work_bound), persistent workgroups that take its entries
// off their own counter (a.work)
template <int VAR>
bool ric_launch_tier2(int N, const SolveArgs& a, hipStream_t s) {
  if (ric_static_n(N) != 60 || !a.kinst || !a.list || !a.work_bound) return false;
  auto kern = ric_kernel<VAR, 1, 60, kSmallCap60, 2>;
  const size_t lds = ric_lds_bytes(N, kSmallCap60);
  if (!set_lds(kern, lds)) return false;
  // every workgroup resident at once (3 per CU): the list is usually empty
  // (each group reads the bound and exits), but when many instances share a
  // hard call -- the Runner's robots in step -- it is most of the batch
  const int64_t g3 = 3 * (int64_t)(ric_cus() > 0 ? ric_cus() : 256);
  const int64_t g = a.B < g3 ? a.B : g3;
  hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(RT), lds, s, a, N, kSmallCap60);
  return true;
}
template <int VAR, int OCC>
bool ric_launch(int N, const SolveArgs& a, hipStream_t s, int* per) {
  const int cap = ric_qcap(N);
  if (a.kinst && !per) {   // factorisation kernel, then the solve kernel without phase 2
    if constexpr (OCC == 1) {
      if (ric_static_n(N) == 60 && ric_qcap_batch(N, a.B) == kSmallCap60)   // small batches: capacity 64
        return ric_launch_fac(ric_factor_kernel<VAR, 60, 47>, N, cap, a, s) &&
               ric_launch_k(ric_kernel<VAR, OCC, 60, kSmallCap60, 2>, N, kSmallCap60, a, s, per);
      if (ric_static_n(N) == 60)
        return ric_launch_fac(ric_factor_kernel<VAR, 60, 47>, N, cap, a, s) &&
               ric_launch_k(ric_kernel<VAR, OCC, 60, 47, 2>, N, cap, a, s, per);
    } else {
      if (ric_static_n(N) == 20)
        return ric_launch_fac(ric_factor_kernel<VAR, 20, 38>, N, cap, a, s) &&
               ric_launch_k(ric_kernel<VAR, OCC, 20, 38, 2>, N, cap, a, s, per);
    }
    return ric_launch_fac(ric_factor_kernel<VAR>, N, cap, a, s) &&
           ric_launch_k(ric_kernel<VAR, OCC, 0, 0, 2>, N, cap, a, s, per);
  }
  if constexpr (OCC == 1) {
    if (ric_static_n(N) == 60) return ric_launch_k(ric_kernel<VAR, OCC, 60, 47>, N, cap, a, s, per);
  } else {
    if (ric_static_n(N) == 20) return ric_launch_k(ric_kernel<VAR, OCC, 20, 38>, N, cap, a, s, per);
  }
  return ric_launch_k(ric_kernel<VAR, OCC>, N, cap, a, s, per);
}
bool ric_launch_any(int variant, int N, const SolveArgs& a, hipStream_t s, int* per) {
  const bool o2 = ric_occ(N) == 2;
  if (variant == 3) return o2 ? ric_launch<3, 2>(N, a, s, per) : ric_launch<3, 1>(N, a, s, per);
  return o2 ? ric_launch<2, 2>(N, a, s, per) : ric_launch<2, 1>(N, a, s, per);
}
}  // namespace

int ric_groups(int variant, int N) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  SolveArgs none{};
  if (!ric_launch_any(variant, N, none, nullptr, &per) || per < 1) per = 1;
  return cus * per;
}

// The separate factorisation kernel pays where the solve kernel runs one
// wave per SIMD (LDS-bound horizons, N > 24): there the factorisation's
// chains otherwise run alone on their SIMD.  Interleaved A/B
// (profiles/r04_ab.json r04l): N = 60 B = 4096 1.475 -> 1.552 M solves/s;
// at 2 waves / SIMD it gains 1.3 % at configs[3] for a 3.9 GB buffer and
// loses 7.7 % at B = 16384, so N <= 24 keeps the fused kernel.  Bounded to
// kKinstBytes of per-instance blocks.
constexpr int64_t kKinstBytes = (int64_t)4 << 30;
int64_t ric_kinst_stride(int N, int64_t B) {
  if (ric_occ(N) != 1) return 0;
  const int64_t s = ric_kinst_doubles(N);
  return B * s * (int64_t)sizeof(double) <= kKinstBytes ? s : 0;
}

int ric_lpt_buckets(int N) {
  if (N < 1) return 0;
  return N + 1 < kLptMax ? N + 1 : kLptMax;
}

bool launch_solve_ric(int variant, int N, const SolveArgs& a, hipStream_t s) {
  if (N < 1 || N > kRicNmax || (variant != 2 && variant != 3)) return false;
  if (a.B <= 0) return true;
  if (!a.work || !a.kws || a.ric_groups < 1) return false;
  const int nb = ric_lpt_buckets(N);
  if (a.lpt && nb > 0 && a.split_list && a.split_count && a.split_nbkt == nb) {
    const int W = (N + nb) / nb;   // ceil((N + 1) / nb) stance counts per bucket
    hipLaunchKernelGGL(ric_buckets_kernel, dim3((unsigned)((a.B + kLptT - 1) / kLptT)), dim3(kLptT), 0, s, a, N, W);
    SolveArgs al = a;
    al.list = a.split_list;
    al.list_count = a.split_count;
    return ric_launch_any(variant, N, al, s, nullptr);
  }
  SolveArgs a0 = a;
  a0.list = nullptr;
  return ric_launch_any(variant, N, a0, s, nullptr);
}

bool ric_has_tier2(int N, int64_t B) { return ric_static_n(N) == 60 && ric_qcap_batch(N, B) < kSmallCap60; }
bool launch_solve_ric_tier2(int variant, int N, const SolveArgs& a, hipStream_t s) {
  if (a.B <= 0) return true;
  return variant == 3 ? ric_launch_tier2<3>(N, a, s) : variant == 2 ? ric_launch_tier2<2>(N, a, s) : false;
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
