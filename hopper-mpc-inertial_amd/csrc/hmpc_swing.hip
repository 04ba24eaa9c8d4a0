// hmpc_swing.hip -- the dense split's third class: the all-swing windows,
// TWO QP instances per wavefront (round 5).
//
// An all-swing window (every stage of the contact schedule C is 0) fixes
// every force to zero (src/mpc_cvx_euler_3f.py:134-136; 2f :129-136), so its
// QP has only the 3N torques as free variables, a dense 3N x 3N condensed
// Hessian (torques reach the orientation through the angular rates) and only
// box rows on them (:123-128).  Its friction and fz rows vanish, and its
// z >= 0.1 rows (:129) have zero normals: they are constants of the free
// response, checked once.  The rest of the kernel is the dense kernel's
// algorithm (hmpc_kernels.hip 4.1): condensed Hessian rows, a right-looking
// Cholesky with the trailing row in registers, range-space Goldfarb-Idnani.
//
// At N = 10 the 30 variables fit half a wave: lanes 0..31 solve one
// instance and lanes 32..63 another, each half with its own LDS image.  Every
// cross-lane step is half-local:
//   * a broadcast of lane s within each 16-lane row is one 64-bit DPP move
//     (row_newbcast); a half of 32 lanes is two rows, so the triangular
//     sweeps run block by block (rows 0..15, then 16..29) with the other
//     row's share of each block deferred to one permlane16_swap and a DPP
//     pass;
//   * a broadcast of lane s over the whole half (the Cholesky pivots) is a
//     row broadcast plus a permlane16_swap;
//   * sums and argmins are a DPP butterfly inside each row plus the swap.
// Nothing is wave-uniform any more: per-instance scalars live in VGPRs
// (equal across their half), and the two halves diverge only in the active
// set, where SIMT masking runs each half's own path.
//
// The kernel does not depend on the variant: with every force fixed, 3f and
// 2f pose the same torque QP (Bd's torque block J_w_inv Rz' dt is the same
// in both, 3f :89, 2f :89), so one kernel serves both.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <utility>

#include "hmpc_internal.h"
#include "hmpc_model.h"

namespace hmpc {
namespace {

template <int Begin, typename F, int... Is>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Begin + Is>{}), ...);
}
template <int Begin, int End, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (End > Begin) sfor_impl<Begin>(std::make_integer_sequence<int, End - Begin>{}, f);
}
// f(l) for l = L, L+1, ... while l < n (n per lane, equal over a half)
template <int L, int LMAX, typename F>
__device__ __forceinline__ void ladder(int n, F&& f) {
  if constexpr (L < LMAX) {
    if (L < n) {
      f(std::integral_constant<int, L>{});
      ladder<L + 1, LMAX>(n, f);
    }
  }
}

__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}
// per-lane select on a compile-time 64-bit lane mask (v_cndmask on an SGPR
// pair holding the constant)
__device__ __forceinline__ unsigned msel(uint64_t m, unsigned t, unsigned f) {
  unsigned r;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}
__device__ __forceinline__ double msel(uint64_t m, double t, double f) {
  const unsigned long long bt = __double_as_longlong(t), bf = __double_as_longlong(f);
  const unsigned lo = msel(m, (unsigned)bt, (unsigned)bf), hi = msel(m, (unsigned)(bt >> 32), (unsigned)(bf >> 32));
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
// a 32-bit lane pattern in both halves
constexpr uint64_t rep(uint32_t m) { return (uint64_t)m | ((uint64_t)m << 32); }
// rep(M) materialised where it is used (a volatile s_mov): the sweeps' step
// masks are loop-invariant inside the active set, and machine LICM hoisted
// all of them out of it -- ~90 SGPR pairs live across the loop, 196 SGPR
// spills into VGPR lanes and a readlane per reload
template <uint32_t M>
__device__ __forceinline__ uint64_t kmask() {
  uint32_t v;
  asm volatile("s_mov_b32 %0, %1" : "=s"(v) : "i"(M));
  return ((uint64_t)v << 32) | v;
}
constexpr uint32_t lo_bits(int n) { return n >= 32 ? 0xffffffffu : ((1u << n) - 1u); }

typedef __attribute__((address_space(3))) double lds_double;
typedef double double2_ __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned lds_addr(const void* p) { return (unsigned)(uintptr_t)p; }
// LDS loads the scheduler cannot move (valid after the matching lds_wait)
template <int OFF>
__device__ __forceinline__ void lds_ld2(double2_& v, unsigned base) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ void lds_ld1o(double& v, unsigned base) {
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF) : "memory");
}
__device__ __forceinline__ void lds_ld1(double& v, unsigned addr) {
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(addr) : "memory");
}
template <int CNT>
__device__ __forceinline__ void lds_wait(double2_& a, double2_& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(CNT));
}
template <int CNT>
__device__ __forceinline__ void lds_wait(double& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(CNT));
}
// LDS ordering point (one wave: the compiler must not reorder LDS accesses)
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

// ---------------------------------------------------------------------------
// half-wave cross-lane primitives
// ---------------------------------------------------------------------------
// lane S of each 16-lane row (gfx950 64-bit DPP, row_newbcast: one move)
template <int S>
__device__ __forceinline__ double rbc(double x) {
  static_assert(S >= 0 && S < 16, "row lane");
  return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + S, 0xf, 0xf, true);
}
// permlane16_swap of x with itself: .first holds rows (0, 0, 2, 2), .second
// rows (1, 1, 3, 3) -- i.e. every row gets the even / odd row of its half
struct RowPair {
  double even, odd;
};
__device__ __forceinline__ RowPair row_pair(double x) {
  const long long b = __double_as_longlong(x);
  const unsigned lo = (unsigned)b, hi = (unsigned)((unsigned long long)b >> 32);
  const auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  RowPair r;
  r.even = __longlong_as_double(((long long)(unsigned)ph[0] << 32) | (unsigned)pl[0]);
  r.odd = __longlong_as_double(((long long)(unsigned)ph[1] << 32) | (unsigned)pl[1]);
  return r;
}
__device__ __forceinline__ void int_pair(int x, int& even, int& odd) {
  const auto p = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
  even = (int)p[0];
  odd = (int)p[1];
}
// lane S of each 32-lane half, over the whole half
template <int S>
__device__ __forceinline__ double hbc(double x) {
  const RowPair p = row_pair(rbc<(S & 15)>(x));
  return S < 16 ? p.even : p.odd;
}
// lane l (runtime, equal over the half) of each half: a bpermute
__device__ __forceinline__ double hbc_rt(double x, int l, int hbase) {
  const long long b = __double_as_longlong(x);
  const int a = (hbase + l) << 2;
  const int lo = __builtin_amdgcn_ds_bpermute(a, (int)b);
  const int hi = __builtin_amdgcn_ds_bpermute(a, (int)((unsigned long long)b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// sum over each half, in every lane of it (bit-identical across the half:
// each butterfly step adds the same two values in either order)
__device__ __forceinline__ double half_sum(double x) {
  x += dpp<kDppXor1>(x);
  x += dpp<kDppXor2>(x);
  x += dpp<kDppHalfMirror>(x);
  x += dpp<kDppMirror>(x);
  const RowPair p = row_pair(x);
  return p.even + p.odd;
}
// lexicographic (v, i) minimum over each half, in every lane of it
__device__ __forceinline__ void half_argmin(double& v, int& i) {
  argmin_combine(v, i, dpp<kDppXor1>(v), dpp<kDppXor1>(i));
  argmin_combine(v, i, dpp<kDppXor2>(v), dpp<kDppXor2>(i));
  argmin_combine(v, i, dpp<kDppHalfMirror>(v), dpp<kDppHalfMirror>(i));
  argmin_combine(v, i, dpp<kDppMirror>(v), dpp<kDppMirror>(i));
  const RowPair p = row_pair(v);
  int ie, io;
  int_pair(i, ie, io);
  v = p.even;
  i = ie;
  argmin_combine(v, i, p.odd, io);
}
// any lane of my half
__device__ __forceinline__ bool half_any(bool f, int h) {
  const uint64_t m = __ballot(f);
  return ((m >> (32 * h)) & 0xffffffffull) != 0;
}

// x <- Ad x and g <- Ad' g lane-parallel (lane r < 12 of each half holds
// component r; hmpc_model.h ad_lane / adt_lane with half-local broadcasts:
// every consumer sits in row 0 of its half)
__device__ __forceinline__ double ad_lane_h(double x, double dt, double cp, double sp, int r) {
  const double xv = row_shift<6>(x);
  const double w0 = rbc<9>(x), w1 = rbc<10>(x);
  const double k1 = (r == 3 || r == 4) ? 1.0 : 0.0;
  const double k0 = (r < 6 && r != 3 && r != 4) ? 1.0 : 0.0;
  const double s1 = (r == 3) ? 1.0 : 0.0, s0 = (r == 4) ? -1.0 : 0.0;
  const double d = fma(fma(k1, cp, k0), xv, sp * fma(s1, w1, s0 * w0));
  return fma(dt, d, x);
}
__device__ __forceinline__ double adt_lane_h(double g, double dt, double cp, double sp, int r) {
  const double gv = row_shift<-6>(g);
  const double g3 = rbc<3>(g), g4 = rbc<4>(g);
  const double k1 = (r == 9 || r == 10) ? 1.0 : 0.0;
  const double k0 = (r >= 6 && r < 12 && r != 9 && r != 10) ? 1.0 : 0.0;
  const double s3 = (r == 10) ? 1.0 : 0.0, s4 = (r == 9) ? -1.0 : 0.0;
  const double d = fma(fma(k1, cp, k0), gv, sp * fma(s3, g3, s4 * g4));
  return fma(dt, d, g);
}

// ---------------------------------------------------------------------------
// LDS layout of one instance (doubles); the wave holds two of these
// ---------------------------------------------------------------------------
template <int N, int QM>
struct SwLay {
  static constexpr int NV = 3 * N;   // the torques (every force is fixed)
  static_assert(NV <= 32, "one instance per half wave");
  static constexpr int e2(int n) { return (n + 1) & ~1; }
  static constexpr int XIN = 0;                  // [12]
  static constexpr int CS = 12;                  // [N][2] cos, sin of the linearisation yaw
  static constexpr int BW = CS + 2 * N;          // [N][3][3] Bd_k rows 9..11, torque columns
  static constexpr int ZR = BW + e2(9 * N);      // [2] a 0.0 for masked loads
  // active-set state (phase 6); the Cholesky's column buffers overlay it
  static constexpr int G0 = ZR + 2;
  static_assert((G0 & 1) == 0, "column buffers must be 16-B aligned");
  static constexpr int UA = G0;                  // [QM] active multipliers
  static constexpr int ACT = UA + QM;            // [QM] active ids (int)
  static constexpr int CB = ACT + QM;            // [QM] c = Qw' w
  static constexpr int GV = CB + QM;             // [QM][2] Givens of a drop
  static constexpr int SD = GV + 2 * QM;         // [QM] subdiagonal scratch
  static constexpr int RM = SD + QM;             // packed upper R, col l at l(l+1)/2
  static constexpr int GEND = RM + e2(QM * (QM + 1) / 2);
  static constexpr int CBS = 40;                 // column buffer stride (>= 32, 16-B multiple)
  static constexpr int COLB = G0;                // [2][CBS] (phase 4 only)
  static constexpr int U0 = GEND > COLB + 2 * CBS ? GEND : COLB + 2 * CBS;
  // union A (phases 0-3)
  static constexpr int XREF = U0;                // [N][12]
  static constexpr int SS = XREF + 12 * N;       // [N][9] S_{t+1}: tw ww M00 M01 M10 M11 Q00 Q01 Q11
  static constexpr int AJ = SS + 9 * N;          // [N][3] adjoint a_{t+1}, rows 9..11
  static constexpr int ENDA = AJ + 3 * N;
  // union B (phases 4-7)
  static constexpr int LC = U0;                  // M = L diag(L)^-1, column-major packed, 1/L_kk on the diagonal
  static constexpr int XS = U0;                  // phase 7: u by variable [32], then x* [N+1][12]
  static constexpr int XO = XS + 32;
  static constexpr int ENDB = LC + e2(NV * (NV + 1) / 2);
  static_assert(XO + 12 * (N + 1) <= ENDB, "x* staging does not fit");
  static constexpr int TOTAL = e2(ENDA > ENDB ? ENDA : ENDB);
  static_assert((TOTAL & 1) == 0, "16-B aligned halves");
  // start of column k of L (rows k..NV-1)
  __host__ __device__ static constexpr int cb(int k) { return k * NV - ((k * (k - 1)) >> 1); }
};

__device__ __forceinline__ int loff(int r) { return (r * (r + 1)) >> 1; }

// ---------------------------------------------------------------------------
// triangular sweeps on M (unit lower, column-major packed; 1/L_kk in the
// diagonal slot), per half.  Variables 0..15 sit in row 0 of the half, 16..NV-1
// in row 1.  A step's broadcast (the just-final entry) is a row_newbcast, so
// it reaches its own row only: the other row's share of a block waits for
// the block to end and then runs as one pass over the row-swapped vector.
// Each step's M entries come through a ring of hand-counted LDS loads
// (kRing steps ahead); lanes without an entry in a step read the 0.0 at ZR.
// ---------------------------------------------------------------------------
constexpr int kRing = 4;

// one load of the ring: lane mask (lanes that read M), byte offset from the
// lane's base, which base (0: the forward base, 1: the backward base)
struct Step {
  uint32_t mask;   // lanes of each half (replicated by kmask)
  int off;
};

// y = L^-1 b (lane v holds b_v)
template <class L>
__device__ __forceinline__ double tri_fwd(double acc, unsigned fbase, unsigned zaddr, double dinv) {
  constexpr int NV = L::NV;
  constexpr int NA = NV < 16 ? NV : 16;          // block A: columns 0..NA-1 (row 0)
  constexpr int NB = NV - NA;                    // block B: columns 16..NV-1 (row 1)
  constexpr int SA = NA - 1;                     // block A steps s = 0..NA-2 (column NA-1 has no row-0 entries below)
  constexpr int SX = NB > 0 ? NA : 0;            // cross steps t = 0..NA-1 (row 1 takes column t)
  constexpr int SB = NB > 0 ? NB - 1 : 0;        // block B steps s = 16..NV-2
  constexpr int NS = SA + SX + SB;
  constexpr uint32_t kLive = lo_bits(NV);
  // step j of the sequence A, X, B
  constexpr auto step = [](int j) constexpr -> Step {
    if (j < SA) {   // column s = j, lanes s < i < 16
      const int s = j;
      return Step{lo_bits(NA) & ~lo_bits(s + 1), 8 * (L::cb(s) - s)};
    }
    if (j < SA + SX) {   // column t, lanes 16 <= i < NV
      const int t = j - SA;
      return Step{kLive & ~lo_bits(16), 8 * (L::cb(t) - t)};
    }
    const int s = 16 + (j - SA - SX);   // column s, lanes s < i < NV
    return Step{kLive & ~lo_bits(s + 1), 8 * (L::cb(s) - s)};
  };
  auto addr = [&](auto jc) -> unsigned {
    constexpr int j = decltype(jc)::value;
    if constexpr (j >= NS) {
      return zaddr;
    } else {
      constexpr Step st = step(j);
      return msel(kmask<st.mask>(), fbase + (unsigned)st.off, zaddr);
    }
  };
  static_assert(NS >= kRing, "the ring is primed with real steps");
  double ring[kRing];
  sfor<0, kRing>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    lds_ld1(ring[j], addr(jc));
  });
  double ysw = 0.0;
  sfor<0, NS>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    if constexpr (NB > 0 && j == SA) ysw = row_pair(acc).even;   // row 1 gets row 0's final y
    double src;
    if constexpr (j < SA) src = rbc<j>(acc);
    else if constexpr (j < SA + SX) src = rbc<j - SA>(ysw);
    else src = rbc<j - SA - SX>(acc);
    // (loads younger than step j's: the ring's, fewer at the tail -- no
    // dummy loads past the last step: an asynchronous write into a register
    // the compiler already considers dead would clobber its next owner)
    lds_wait<(kRing - 1 < NS - 1 - j ? kRing - 1 : NS - 1 - j)>(ring[j % kRing]);
    acc = fma(-ring[j % kRing], src, acc);
    if constexpr (j + kRing < NS) lds_ld1(ring[j % kRing], addr(std::integral_constant<int, j + kRing>{}));
  });
  return acc * dinv;
}

// z = L^-T b (lane v holds b_v)
template <class L>
__device__ __forceinline__ double tri_bwd(double acc, unsigned bbase, unsigned zaddr, double dinv) {
  constexpr int NV = L::NV;
  constexpr int NA = NV < 16 ? NV : 16;
  constexpr int NB = NV - NA;
  constexpr int SB = NB > 0 ? NB - 1 : 0;        // block B steps s = NV-1 .. 17 (lanes 16 <= i < s)
  constexpr int SX = NB;                         // cross steps s = NV-1 .. 16 (lanes i < 16)
  constexpr int SA = NA - 1;                     // block A steps s = NA-1 .. 1 (lanes i < s)
  constexpr int NS = SB + SX + SA;
  acc *= dinv;
  // M[s][i] (row s, column i < s) sits at LC + cb(i) + s - i: the lane's base
  // (LC + cb(i) - i) plus 8 s
  constexpr auto step = [](int j) constexpr -> Step {
    if (j < SB) {
      const int s = NV - 1 - j;
      return Step{lo_bits(s) & ~lo_bits(16), 8 * s};
    }
    if (j < SB + SX) {
      const int s = NV - 1 - (j - SB);
      return Step{lo_bits(16), 8 * s};
    }
    const int s = NA - 1 - (j - SB - SX);
    return Step{lo_bits(s), 8 * s};
  };
  auto addr = [&](auto jc) -> unsigned {
    constexpr int j = decltype(jc)::value;
    if constexpr (j >= NS) {
      return zaddr;
    } else {
      constexpr Step st = step(j);
      return msel(kmask<st.mask>(), bbase + (unsigned)st.off, zaddr);
    }
  };
  static_assert(NS >= kRing, "the ring is primed with real steps");
  double ring[kRing];
  sfor<0, kRing>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    lds_ld1(ring[j], addr(jc));
  });
  double zsw = 0.0;
  sfor<0, NS>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    if constexpr (NB > 0 && j == SB) zsw = row_pair(acc).odd;   // row 0 gets row 1's final z
    double src;
    if constexpr (j < SB) src = rbc<NV - 1 - j - 16>(acc);
    else if constexpr (j < SB + SX) src = rbc<NV - 1 - (j - SB) - 16>(zsw);
    else src = rbc<NA - 1 - (j - SB - SX)>(acc);
    lds_wait<(kRing - 1 < NS - 1 - j ? kRing - 1 : NS - 1 - j)>(ring[j % kRing]);
    acc = fma(-ring[j % kRing], src, acc);
    if constexpr (j + kRing < NS) lds_ld1(ring[j % kRing], addr(std::integral_constant<int, j + kRing>{}));
  });
  return acc;
}

constexpr int kPrioSwing = 1;

// Diagnostic build only (-DHMPC_STAMPS, tools/phase_stamps.py): s_memtime at
// the dense kernel's phase boundaries (slots 0..8; 1 == 2, the dynamics run
// with the loads) and its accumulated active-set sub-phases (9..14), written
// over each instance's x* row.  One wave runs both halves, so a pair shares
// its stamps.
#ifdef HMPC_STAMPS
#define SW_STAMP(i) (stamp_[i] = __builtin_amdgcn_s_memtime())
#define SW_TIC(v) const long long v = __builtin_amdgcn_s_memtime()
#define SW_TOC(slot, v) (stamp_[slot] += __builtin_amdgcn_s_memtime() - (v))
#else
#define SW_STAMP(i) ((void)0)
#define SW_TIC(v) ((void)0)
#define SW_TOC(slot, v) ((void)0)
#endif

// ---------------------------------------------------------------------------
// the kernel: block i solves instances 2i (lanes 0..31) and 2i + 1 (lanes
// 32..63) of its class list
// ---------------------------------------------------------------------------
template <int N, int QM>
__global__ void __launch_bounds__(64, HMPC_SWING_WAVES) swing_kernel(SolveArgs a) {
  using L = SwLay<N, QM>;
  constexpr int NV = L::NV;
  __shared__ __attribute__((aligned(16))) double smem[2 * L::TOTAL];
  const int lane = threadIdx.x;
  const int h = lane >> 5, hl = lane & 31;
  double* const sm = smem + h * L::TOTAL;   // my instance's LDS image

  const int cnt = *a.list_count;
  const int i0 = 2 * (int)blockIdx.x;
  if (i0 >= cnt) return;
  const bool valid = i0 + h < cnt;
  // an odd list's last block: the upper half repeats the lower half's
  // instance (identical control flow) and stores nothing
  const int64_t b = a.list[valid ? i0 + h : i0];
  const double dt = a.dt;
#ifdef HMPC_STAMPS
  long long stamp_[16] = {0};
#endif
  SW_STAMP(0);

  // ---------------- phase 0: loads ------------------------------------------
  {
    constexpr int NR = (12 * N + 31) / 32;
    const double* xrf = a.x_ref + b * a.xref_bs;
    const int mode = a.shift_mode;
    double vr[NR];
    const double vi = a.x_in[b * 12 + (hl < 12 ? hl : 0)];
    sfor<0, NR>([&](auto itc) __attribute__((always_inline)) {
      constexpr int it = decltype(itc)::value;
      const int i = hl + 32 * it, ic = i < 12 * N ? i : 0;
      const int r = ic / 12, c = ic - 12 * r;
      vr[it] = xrf[r * a.xref_rs + c];
    });
    // the linearisation yaw of stage k = hl (the only part of x_lin the
    // torque dynamics read, :86-89): given (mode 0), [x_in; x_ref] (mode 1,
    // :52-53) or the time shift of x_prev (mode 2, :59-62)
    const int k = hl < N ? hl : 0;
    const double* xp = a.x_lin + b * 12 * (N + 1);
    double psi;
    if (mode == 0) psi = xp[12 * k + 5];
    else if (mode == 1) psi = k == 0 ? a.x_in[b * 12 + 5] : xrf[(k - 1) * a.xref_rs + 5];
    else psi = k == 0 ? a.x_in[b * 12 + 5] : xp[12 * (k + 1 <= N ? k + 1 : N) + 5];
    if (hl < 12) sm[L::XIN + hl] = vi;
    sfor<0, NR>([&](auto itc) __attribute__((always_inline)) {
      constexpr int it = decltype(itc)::value;
      const int i = hl + 32 * it;
      if (i < 12 * N) sm[L::XREF + i] = vr[it];
    });
    if (hl == 0) sm[L::ZR] = 0.0;
    SW_STAMP(1);
    // ---------------- phase 1: gen_dt_dynamics, torque block (lane k < N)
    // (3f :71-94, 2f :70-94: B[9:12, 3:6] = J_w_inv Rz' dt, :86,89)
    if (hl < N) {
      double sp, cp;
      sincos(psi, &sp, &cp);
      const double Rz[3][3] = {{cp, sp, 0.0}, {-sp, cp, 0.0}, {0.0, 0.0, 1.0}};   // src/utils.py:46-51
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
      double* bw = sm + L::BW + 9 * k;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          bw[3 * i + j] = (Jw[i][0] * RzT[0][j] + Jw[i][1] * RzT[1][j] + Jw[i][2] * RzT[2][j]) * dt;
      sm[L::CS + 2 * k] = cp;
      sm[L::CS + 2 * k + 1] = sp;
    }
  }
  wsync();
  SW_STAMP(2);

  // ---------------- phase 2: free response, cost-to-go, adjoint --------------
  // (lane r < 12 of a half holds component r; the cost-to-go's rotational
  // blocks are computed on every lane, lane 0 of the half stores them)
  int status = ST_SOLVED, iters = 0;
  bool zpre, zrow;
  {
    double xr = hl < 12 ? sm[L::XIN + hl] : 0.0;
    const double qr = qdiag(hl);
    const double cpl = hl < N ? sm[L::CS + 2 * hl] : 0.0;
    const double spl = hl < N ? sm[L::CS + 2 * hl + 1] : 0.0;
    // z >= 0.1 (:129): the z_0 and z_1 rows are constants (no input reaches
    // them); with every force fixed so are the later ones.  The dense kernel
    // fails the first two before the active set and picks a violated later
    // one as its first (infinitely violated) constraint: the same here.
    bool zbad0 = hl == 2 && xr - kZmin < -kTol, zbad1 = false;
    // yaw block [tt, tw, ww] of S (x5, w_z): no yaw dependence
    double ya = kTermQ * kQ[5], yb = 0.0, yc = kTermQ * kQ[11];
    double s[10];   // P00 P01 P11 M00 M01 M10 M11 Q00 Q01 Q11 (roll/pitch block)
    s[0] = kTermQ * kQ[3]; s[1] = 0.0; s[2] = kTermQ * kQ[4];
    s[3] = s[4] = s[5] = s[6] = 0.0;
    s[7] = kTermQ * kQ[9]; s[8] = 0.0; s[9] = kTermQ * kQ[10];
    auto store_s = [&](int t) __attribute__((always_inline)) {
      if (hl == 0) {
        double* st = sm + L::SS + 9 * t;
        st[0] = yb; st[1] = yc;
#pragma unroll
        for (int e = 0; e < 7; ++e) st[2 + e] = s[3 + e];
      }
    };
    store_s(N - 1);
    double xrf[N], dgv[N];
    sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      xrf[k] = sm[L::XREF + 12 * k + (hl < 12 ? hl : 0)];
    });
    sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      xr = ad_lane_h(xr, dt, rbc<k>(cpl), rbc<k>(spl), hl) + ((hl == 8) ? -a.g * dt : 0.0);
      const double kf = (k == N - 1) ? kTermQ : 1.0;
      dgv[k] = kf * qr * (xr - xrf[k]);
      if constexpr (k == 0) zbad0 = zbad0 || (hl == 2 && xr - kZmin < -kTol);
      else if constexpr (k + 1 <= N - 1) zbad1 = zbad1 || (hl == 2 && xr - kZmin < -kTol);
      constexpr int t = N - 1 - k;
      if constexpr (t >= 1) {
        const double ct = rbc<t>(cpl), st = rbc<t>(spl);
        {
          const double aa = ya, bb = yb, cc = yc;
          yb = fma(dt, aa, bb);
          yc = cc + dt * (2.0 * bb + dt * aa);
          ya = aa + kQ[5];
          yc = yc + kQ[11];
        }
        const double D00 = ct * dt, D01 = st * dt, D10 = -st * dt, D11 = ct * dt;
        const double P00 = s[0], P01 = s[1], P11 = s[2];
        const double M00 = s[3], M01 = s[4], M10 = s[5], M11 = s[6];
        const double N00 = M00 + (P00 * D00 + P01 * D10), N01 = M01 + (P00 * D01 + P01 * D11);
        const double N10 = M10 + (P01 * D00 + P11 * D10), N11 = M11 + (P01 * D01 + P11 * D11);
        const double A00 = D00 * N00 + D10 * N10, A01 = D00 * N01 + D10 * N11;
        const double A11 = D01 * N01 + D11 * N11;
        const double B00 = M00 * D00 + M10 * D10, B01 = M00 * D01 + M10 * D11;
        const double B11 = M01 * D01 + M11 * D11;
        s[7] += A00 + B00;
        s[8] += A01 + B01;
        s[9] += A11 + B11;
        s[3] = N00; s[4] = N01; s[5] = N10; s[6] = N11;
        s[0] += kQ[3]; s[2] += kQ[4];
        s[7] += kQ[9]; s[9] += kQ[10];
        store_s(t - 1);
      }
    });
    // adjoint a_N = d_N, a_t = d_t + Ad_t' a_{t+1}; rows 9..11 (the torque
    // rows of Bd) are kept
    double ar = dgv[N - 1];
    if (hl >= 9 && hl < 12) sm[L::AJ + 3 * (N - 1) + hl - 9] = ar;
    sfor<1, N>([&](auto ic) __attribute__((always_inline)) {
      constexpr int t = N - decltype(ic)::value;   // N-1 .. 1
      ar = adt_lane_h(ar, dt, rbc<t>(cpl), rbc<t>(spl), hl) + dgv[t - 1];
      if (hl >= 9 && hl < 12) sm[L::AJ + 3 * (t - 1) + hl - 9] = ar;
    });
    zpre = half_any(zbad0, h);
    zrow = half_any(zbad1, h);
  }
  wsync();
  SW_STAMP(3);

  // ---------------- phase 3: Hessian row (lower part) + gradient -------------
  // lane v < NV owns torque c = v % 3 of stage i = v / 3; lanes NV..31 are
  // padding (zero rows, never stepped)
  const bool active_lane = hl < NV;
  double Rg[NV];
  double hv = 0.0;
  {
    const int ii = active_lane ? hl / 3 : 0;
    const int ci = active_lane ? hl - 3 * (hl / 3) : 0;
    const double rowm = active_lane ? 1.0 : 0.0;
    const double* bwi = sm + L::BW + 9 * ii;
    const double e9 = rowm * bwi[ci], e10 = rowm * bwi[3 + ci], e11 = rowm * bwi[6 + ci];
    const double* si = sm + L::SS + 9 * ii;   // S_{i+1}
    const double tw = si[0], ww = si[1], M00 = si[2], M01 = si[3], M10 = si[4], M11 = si[5];
    const double Q00 = si[6], Q01 = si[7], Q11 = si[8];
    // f = S_{i+1} b, b = Bd_i e_c (rows 9..11; hmpc_model.h s_times<true>)
    const double f3 = M00 * e9 + M01 * e10, f4 = M10 * e9 + M11 * e10, f5 = tw * e11;
    double g9 = Q00 * e9 + Q01 * e10, g10 = Q01 * e9 + Q11 * e10, g11 = ww * e11;
    // gradient h_v = 2 b' a_{i+1}
    const double* aj = sm + L::AJ + 3 * ii;
    double hacc = 0.0;
    hacc = fma(e9, aj[0], hacc);
    hacc = fma(e10, aj[1], hacc);
    hacc = fma(e11, aj[2], hacc);
    hv = 2.0 * hacc;
    // H[v, (j, c2)] = 2 Bd_j[:, c2]' g_j, g_i = f, g_j = Ad_{j+1}' g_{j+1}:
    // Ad' leaves the angle rows (f3, f4, f5) alone and adds dt Rz' of them to
    // the rate rows.  Entries right of the diagonal (j > i) keep the finite
    // values that fall out; only the lower triangle is read.
    double cp_up = 0.0, sp_up = 0.0;   // cos / sin of the stage above
    sfor<0, N>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = N - 1 - decltype(jc)::value;
      // stage j's torque block of Bd and cos / sin in one LDS round trip
      // (eleven loads, one wait) instead of one per product
      double bw[9], cj, sj;
      {
        const unsigned sb = lds_addr(sm + opaque_zero());
        sfor<0, 9>([&](auto ic) __attribute__((always_inline)) {
          constexpr int i = decltype(ic)::value;
          lds_ld1o<8 * (L::BW + 9 * j + i)>(bw[i], sb);
        });
        lds_ld1o<8 * (L::CS + 2 * j)>(cj, sb);
        lds_ld1o<8 * (L::CS + 2 * j + 1)>(sj, sb);
        sfor<0, 9>([&](auto ic) __attribute__((always_inline)) { lds_wait<0>(bw[decltype(ic)::value]); });
        lds_wait<0>(cj);
        lds_wait<0>(sj);
      }
      if constexpr (j < N - 1) {
        const double cp1 = cp_up, sp1 = sp_up;
        const double n9 = g9 + ((cp1 * dt) * f3 + (-sp1 * dt) * f4);
        const double n10 = g10 + ((sp1 * dt) * f3 + (cp1 * dt) * f4);
        const double n11 = fma(dt, f5, g11);
        g9 = (ii > j) ? n9 : g9;
        g10 = (ii > j) ? n10 : g10;
        g11 = (ii > j) ? n11 : g11;
      }
      cp_up = cj;
      sp_up = sj;
      sfor<0, 3>([&](auto cc) __attribute__((always_inline)) {
        constexpr int c2 = decltype(cc)::value;
        double acc = 0.0;
        acc = fma(bw[c2], g9, acc);
        acc = fma(bw[3 + c2], g10, acc);
        acc = fma(bw[6 + c2], g11, acc);
        Rg[3 * j + c2] = 2.0 * acc;
        pin(Rg[3 * j + c2]);
      });
    });
  }
  double wv = -hv;   // the forward sweep's accumulator (phase 4)
  wsync();           // union A (XREF / SS / AJ) is dead from here on
  SW_STAMP(4);
  __builtin_amdgcn_s_setprio(kPrioSwing);

  // ---------------- phase 4: Cholesky ---------------------------------------
  // hmpc_kernels.hip's one-wave right-looking factorisation per half: lane v
  // holds row v of the trailing matrix; step k publishes column k through
  // the half's LDS column buffer, the pivot reaches the half by a
  // broadcast, column k of M goes to LDS for the sweeps, the forward
  // substitution of phase 5 rides along.  Every step is compile-time.
  double dinv;
  {
    constexpr int CW = 4;
    // depth of the column-chunk ring (3 one chunk further ahead; 2 for the
    // 4-wave register budget)
    constexpr int kCR = HMPC_SWING_WAVES >= 4 ? 2 : 3;
    constexpr int CBS = L::CBS;
    constexpr uint32_t kLive = lo_bits(NV);
    auto nldc = [](int ja, int ch) constexpr {   // b128 loads of chunk ch of [ja, NV)
      return (NV - ja - CW * ch) >= CW ? CW / 2 : ((NV - ja - CW * ch) > 0 ? (NV - ja - CW * ch + 1) / 2 : 0);
    };
    // the diagonal not built in phase 3: 2 V_i (R, every stage but the last,
    // 3f :114,132,139), by step
    auto dx = [](int s) constexpr { return (s / 3 != N - 1) ? 2.0 * kRdiag : 0.0; };
    int nbad = 0;
    double2_ nb[CW / 2];
    double p_rs = 0.0, p_tk = 0.0;
    unsigned colb[2] = {lds_addr(sm + L::COLB), lds_addr(sm + L::COLB + CBS)};
    asm volatile("" : "+v"(colb[0]), "+v"(colb[1]));
    auto ahead = [&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      constexpr int JS = (s + 1) & ~1;
      double* col = sm + L::COLB + (s & 1) * CBS;
      const double mine = Rg[s];
      col[hl] = mine;
      wsync();
      const unsigned cb0 = colb[s & 1];
      sfor<0, nldc(JS, 0)>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        lds_ld2<8 * (JS + 2 * i)>(nb[i], cb0);
      });
      const double piv = hbc<s>(mine) + dx(s);
      nbad |= piv > 0.0 ? 0 : 1;
      const double pv = piv > 0.0 ? piv : 1.0;
      p_rs = rsq_nr(pv);
      p_tk = (mine * p_rs) * p_rs;
    };
    ahead(std::integral_constant<int, 0>{});
    const unsigned tb = lds_addr(sm + hl);
    sfor<0, NV>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      constexpr int JA = (k + 1) & ~1;
      constexpr int NCH = (NV - JA + CW - 1) / CW;
      constexpr int NAHEAD = (k + 1 < NV) ? 1 + nldc((k + 2) & ~1, 0) : 0;   // LDS ops of ahead()
      const double rs = p_rs, tk = p_tk;
      if constexpr (k == 0) lds_wait<0>(nb[0], nb[1]);
      const double nt = -tk;
      constexpr uint64_t m_eq = rep(1u << k);
      constexpr uint64_t m_ge = rep(kLive & ~lo_bits(k));
      constexpr uint64_t m_gt = m_ge & ~m_eq;
      {   // column k of M (other lanes: the column buffer of step k+1)
        constexpr int DOFF = 8 * (L::COLB + ((k + 1) & 1) * CBS);
        constexpr int LOFF = 8 * (L::LC + L::cb(k) - k);
        const unsigned ad = msel(m_ge, tb + (unsigned)(LOFF - DOFF), tb);
        *(lds_double*)(ad + DOFF) = msel(m_eq, rs, tk);
      }
      wv = fma(msel(m_gt, tk, 0.0), -hbc<k>(wv), wv);
      const unsigned cbase = colb[k & 1];
      double2_ buf[kCR][CW / 2];
      auto load = [&](auto chc) __attribute__((always_inline)) {
        constexpr int ch = decltype(chc)::value;
        if constexpr (ch >= 1 && ch < NCH) {
          sfor<0, nldc(JA, ch)>([&](auto ic) __attribute__((always_inline)) {
            constexpr int i = decltype(ic)::value;
            lds_ld2<8 * (JA + CW * ch + 2 * i)>(buf[ch % kCR][i], cbase);
          });
        }
      };
      auto nl = [](int ja, int ch) constexpr {
        return (ch >= 1 && ch < (NV - ja + CW - 1) / CW)
                   ? ((NV - ja - CW * ch) >= CW ? CW / 2 : (NV - ja - CW * ch + 1) / 2)
                   : 0;
      };
      auto update = [&](auto chc, const double2_ (&bf)[CW / 2]) __attribute__((always_inline)) {
        constexpr int ch = decltype(chc)::value;
        sfor<0, CW>([&](auto ic) __attribute__((always_inline)) {
          constexpr int i = decltype(ic)::value;
          constexpr int j = JA + CW * ch + i;
          if constexpr (j > k && j < NV) {
            const double cv = (i & 1) ? bf[i / 2].y : bf[i / 2].x;
            Rg[j] = fma(nt, cv, Rg[j]);
            pin(Rg[j]);
          }
        });
      };
      // chunks >= 1 through a kCR-deep ring: the prologue loads chunks
      // 1 .. kCR-1, then ahead(k+1) issues its LDS ops, and iteration ch
      // loads chunk ch + kCR - 1 before it waits for chunk ch
      sfor<1, kCR>([&](auto chc) __attribute__((always_inline)) { load(chc); });
      if constexpr (NCH > 0) update(std::integral_constant<int, 0>{}, nb);
      if constexpr (k + 1 < NV) ahead(std::integral_constant<int, k + 1>{});
      sfor<1, NCH>([&](auto chc) __attribute__((always_inline)) {
        constexpr int ch = decltype(chc)::value;
        load(std::integral_constant<int, ch + kCR - 1>{});
        // LDS ops issued after chunk ch's loads
        constexpr int younger = [&]() constexpr {
          int y = ch <= kCR - 1 ? NAHEAD : 0;
          for (int c = ch + 1; c <= ch + kCR - 1; ++c) y += nl(JA, c);
          return y;
        }();
        lds_wait<younger>(buf[ch % kCR][0], buf[ch % kCR][1]);
        update(chc, buf[ch % kCR]);
      });
      if constexpr (k + 1 < NV) lds_wait<0>(nb[0], nb[1]);
    });
    wsync();
    // (the dense kernel's order: a bad pivot, then the z_0 / z_1 rows before
    // the active set, then a later z row as its first pick)
    if (zpre) status = ST_INFEAS;
    else if (nbad) status = ST_NUMERICAL;
    else if (zrow) { status = ST_INFEAS; iters = 1; }
    dinv = active_lane ? sm[L::LC + L::cb(active_lane ? hl : 0)] : 1.0;   // 1 / L[v][v]
  }

  SW_STAMP(5);
  const unsigned zaddr = lds_addr(sm + L::ZR);
  const unsigned fbase = lds_addr(sm + L::LC + hl);                                   // + 8 (cb(s) - s)
  const unsigned bbase = lds_addr(sm + L::LC + (active_lane ? L::cb(hl) - hl : 0));   // + 8 s

  // ---------------- phase 5: v0 = -L^-T L^-1 h --------------------------------
  double v = tri_bwd<L>(wv * dinv, bbase, zaddr, dinv);
  SW_STAMP(6);
  // (padding lanes hold 0: zero rows and right-hand sides)

  // ---------------- phase 6: Goldfarb-Idnani, range-space form --------------
  // Constraints of lane v (id = 4 v + slot): slot 0  v >= -lim, slot 1
  // -v >= -lim (:123-128); lim = 7.78 for tau_x, tau_y, 4 for tau_z.
  const double lim = active_lane ? tau_lim(3 + hl - 3 * (hl / 3)) : 0.0;
  int actmask = 0;
  double* Rm = sm + L::RM;
  double* ua = sm + L::UA;
  int* act = reinterpret_cast<int*>(sm + L::ACT);
  double* cbv = sm + L::CB;
  double* gv = sm + L::GV;
  double* sdg = sm + L::SD;
  double Qw[QM];
#pragma unroll
  for (int l = 0; l < QM; ++l) Qw[l] = 0.0;
  int q = 0;
  const int max_iter = 4 * NV + 50;
  const int hbase = 32 * h;

  bool done = status != ST_SOLVED;
  while (!done) {
    // ---- slacks of my rows; the most violated over the half ----
    SW_TIC(t_scan);
    double best = INFINITY;
    int bid = 0x7fffffff;
    if (active_lane && !(actmask & 1)) argmin_combine(best, bid, v + lim, 4 * hl);
    if (active_lane && !(actmask & 2)) argmin_combine(best, bid, lim - v, 4 * hl + 1);
    half_argmin(best, bid);
    SW_TOC(9, t_scan);
    if (!(best < -kTol)) break;   // primal feasible: optimal
    const int p = bid;
    const int o = p >> 2;
    const double sgn = (p & 3) == 0 ? 1.0 : -1.0;
    const double bp = -tau_lim(3 + o - 3 * (o / 3));
    const double np_me = hl == o ? sgn : 0.0;
    double u_plus = 0.0;
    // w = L^-1 n_p
    SW_TIC(t_fwd);
    const double wfull = tri_fwd<L>(np_me, fbase, zaddr, dinv);
    const double wnorm2 = half_sum(wfull * wfull);
    SW_TOC(10, t_fwd);
    // ---- inner loop: step towards satisfying constraint p ----
    while (true) {
      if (++iters > max_iter) { status = ST_MAXIT; done = true; break; }
      const int qu = q;
      // w_perp = (I - Qw Qw') w and c = Qw' w (modified Gram-Schmidt, a
      // second pass when the first cancels more than half the norm)
      SW_TIC(t_gs);
      double wp = wfull, zn = wnorm2;
      for (int pass = 0; pass < 2 && qu > 0; ++pass) {
        ladder<0, QM>(qu, [&](auto lc) __attribute__((always_inline)) {
          constexpr int l = decltype(lc)::value;
          const double cl = half_sum(Qw[l] * wp);
          wp = fma(-cl, Qw[l], wp);
          if (hl == 0) cbv[l] = (pass == 0) ? cl : cbv[l] + cl;
        });
        const double n2 = half_sum(wp * wp);
        const bool enough = n2 > 0.25 * zn;
        zn = n2;
        if (enough) break;
      }
      wsync();
      SW_TOC(11, t_gs);
      // primal direction z = L^-T w_perp
      SW_TIC(t_bwd);
      const double zi = tri_bwd<L>(wp, bbase, zaddr, dinv);
      SW_TOC(12, t_bwd);
      SW_TIC(t_dual);
      // dual direction r = R^-1 c (lanes l < q), back substitution
      double rcur = hl < qu ? cbv[hl < qu ? hl : 0] : 0.0, rmine = 0.0;
      for (int l = qu - 1; l >= 0; --l) {
        const double rl = hbc_rt(rcur, l, hbase) / Rm[loff(l) + l];
        if (hl == l) rmine = rl;
        if (hl < l) rcur = fma(-Rm[loff(l) + (hl < l ? hl : 0)], rl, rcur);
      }
      // partial step length t1 (drop candidate)
      double t1 = INFINITY;
      int kdrop = 0x7fffffff;
      if (hl < qu && rmine > 0.0) { t1 = ua[hl] / rmine; kdrop = hl; }
      half_argmin(t1, kdrop);
      // full step length t2 (n_p' z = |w_perp|^2)
      const double sp_ = half_sum(np_me * v) - bp;
      const bool has_z = zn > 1e-24 * wnorm2;
      const double t2 = has_z ? -sp_ / zn : INFINITY;
      const double t = t1 < t2 ? t1 : t2;
      if (!(t < INFINITY)) { status = ST_INFEAS; done = true; break; }
      if (has_z) v = fma(t, zi, v);
      if (hl < qu) ua[hl] -= t * rmine;
      u_plus += t;
      wsync();
      SW_TOC(13, t_dual);
      SW_TIC(t_upd);
      if (has_z && t == t2) {
        // ---- add p: new basis column w_perp / |w_perp|, R column [c; rho] ----
        if (qu >= QM) { status = a.ovf_count ? ST_OVERFLOW : ST_NUMERICAL; done = true; break; }
        const double rho = sqrt(zn);
        const double qn = wp / rho;
#pragma unroll
        for (int l = 0; l < QM; ++l) Qw[l] = (l == qu) ? qn : Qw[l];
        if (hl < qu) Rm[loff(qu) + hl] = cbv[hl < qu ? hl : 0];
        if (hl == qu) Rm[loff(qu) + qu] = rho;
        if (hl == 0) { act[qu] = p; ua[qu] = u_plus; }
        if (hl == o) actmask |= 1 << (p & 3);
        q = qu + 1;
        wsync();
        SW_TOC(14, t_upd);
        break;
      }
      // ---- drop active constraint kdrop ----
      {
        const int k = kdrop;
        const int idk = act[k];
        if (hl == (idk >> 2)) actmask &= ~(1 << (idk & 3));
        for (int m = k; m + 1 < qu; ++m) {   // shift R columns k+1..q-1 left
          double val = 0.0;
          if (hl <= m + 1) val = Rm[loff(m + 1) + hl];
          wsync();
          if (hl <= m) Rm[loff(m) + hl] = val;
          if (hl == m + 1) sdg[m] = val;
          wsync();
        }
        {   // shift the active list and multipliers
          int an = 0;
          double un = 0.0;
          if (hl >= k && hl + 1 < qu) { an = act[hl + 1]; un = ua[hl + 1]; }
          wsync();
          if (hl >= k && hl + 1 < qu) { act[hl] = an; ua[hl] = un; }
          wsync();
        }
        for (int l = k; l + 1 < qu; ++l) {   // Givens on rows (l, l+1)
          const double aa = Rm[loff(l) + l], bb = sdg[l];
          const double hh = sqrt(aa * aa + bb * bb);
          const double cg = aa / hh, sg = bb / hh;
          wsync();
          if (hl == l) { Rm[loff(l) + l] = hh; gv[2 * l] = cg; gv[2 * l + 1] = sg; }
          const int mcol = hl;
          if (mcol > l && mcol + 1 < qu) {
            const double rl = Rm[loff(mcol) + l], rl1 = Rm[loff(mcol) + l + 1];
            Rm[loff(mcol) + l] = cg * rl + sg * rl1;
            Rm[loff(mcol) + l + 1] = -sg * rl + cg * rl1;
          }
          wsync();
        }
#pragma unroll
        for (int l = 0; l + 1 < QM; ++l) {   // the same rotations on the basis
          const bool rot = l >= k && l + 1 < qu;
          const int lg = rot ? l : 0;
          const double cg = gv[2 * lg], sg = gv[2 * lg + 1];
          const double x0 = Qw[l], x1 = Qw[l + 1];
          Qw[l] = rot ? cg * x0 + sg * x1 : x0;
          Qw[l + 1] = rot ? -sg * x0 + cg * x1 : x1;
        }
#pragma unroll
        for (int l = 0; l < QM; ++l) Qw[l] = (l == qu - 1) ? 0.0 : Qw[l];
        q = qu - 1;
        wsync();
        SW_TOC(14, t_upd);
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);
  SW_STAMP(7);

  // an overflowed instance writes nothing but its status and its place in
  // the overflow list (x_lin may be this solve's input, mpcontrol shift)
  if (status == ST_OVERFLOW) {
    if (hl == 0 && valid) {
      a.status[b] = ST_OVERFLOW;
      a.ovf_list[atomicAdd(a.ovf_count, 1)] = (int32_t)b;
    }
    return;
  }

  // ---------------- phase 7: outputs ----------------------------------------
  // x_ref again (its LDS copy is gone): every row's load issued up front
  const double* xrf7 = a.x_ref + b * a.xref_bs + (hl < 12 ? hl : 0);
  double xrg[N];
  sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    xrg[k] = xrf7[k * a.xref_rs];
  });
  double* xs = sm + L::XS;
  xs[hl] = active_lane ? v : 0.0;   // u by variable (L is dead)
  wsync();
  if (valid) {   // u* in full order: forces 0, torques from xs
    double* ub = a.u + b * 6 * N;
    for (int e = hl; e < 6 * N; e += 32) {
      const int k = e / 6, c = e - 6 * k;
      ub[e] = c >= 3 ? xs[3 * k + c - 3] : 0.0;
    }
  }
  {
    double* xo = sm + L::XO;
    double xr = hl < 12 ? sm[L::XIN + hl] : 0.0;
    if (hl < 12) xo[hl] = xr;
    const double qr = qdiag(hl);
    const int rw = (hl >= 9 && hl < 12) ? hl - 9 : 0;   // my row of Bd's omega block
    const double rdu = (hl >= 3 && hl < 6) ? kRdiag : 0.0;   // forces are 0 and u_ref is 0 here
    const int tu = (hl >= 3 && hl < 6) ? hl - 3 : 0;
    const double gdt = hl == 8 ? -a.g * dt : 0.0;
    const double isw = (hl >= 9 && hl < 12) ? 1.0 : 0.0;
    double objl = 0.0;
    // the rollout first, the objective after it: the x_ref loads land while
    // the rollout runs (as in the dense kernel's phase 7)
    double xk[N];
    sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      const double cp = sm[L::CS + 2 * k], sp = sm[L::CS + 2 * k + 1];
      const double* bwr = sm + L::BW + 9 * k + 3 * rw;
      const double* uk = xs + 3 * k;
      double bw_u = 0.0;
#pragma unroll
      for (int c = 0; c < 3; ++c) bw_u = fma(bwr[c], uk[c], bw_u);
      xr = ad_lane_h(xr, dt, cp, sp, hl) + isw * bw_u + gdt;
      xk[k] = xr;
      if constexpr (k < N - 1) {
        const double du = uk[tu];
        objl = fma(rdu * du, du, objl);
      }
      if (hl < 12) xo[12 * (k + 1) + hl] = xr;
    });
    sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      const double kf = (k == N - 1) ? kTermQ : 1.0;
      const double e = xk[k] - xrg[k];
      objl = fma(kf * qr * e, e, objl);
    });
    const double objv = half_sum(objl);
    wsync();
#ifdef HMPC_STAMPS
    SW_STAMP(8);
    if (hl < 16) xo[hl] = __longlong_as_double(stamp_[hl]);   // (lane-uniform stamps)
    wsync();
#endif
    if (valid) {
      if (a.x)
        for (int i = hl; i < 12 * (N + 1); i += 32) a.x[b * 12 * (N + 1) + i] = xo[i];
      if (hl == 0) {
        if (a.obj) a.obj[b] = objv;
        a.status[b] = status;
        if (a.iters) a.iters[b] = iters;
        if (a.active) a.active[b] = q;
      }
    }
  }
}

}  // namespace

// the launcher (hmpc_kernels.hip's split launch calls it for the all-swing
// list: a.list / a.list_count set by the caller; grid = ceil(B / 2))
#define HMPC_SW_CAT2(a, b) a##b
#define HMPC_SW_CAT(a, b) HMPC_SW_CAT2(a, b)
bool HMPC_SW_CAT(launch_swing_n, HMPC_INST_N)(const SolveArgs& a, hipStream_t s) {
  if (a.B <= 0) return true;
  hipLaunchKernelGGL((swing_kernel<HMPC_INST_N, HMPC_SWING_Q>), dim3((unsigned)((a.B + 1) / 2)), dim3(64), 0, s, a);
  return true;
}
int HMPC_SW_CAT(swing_qmax_n, HMPC_INST_N)() { return HMPC_SWING_Q; }

}  // namespace hmpc
