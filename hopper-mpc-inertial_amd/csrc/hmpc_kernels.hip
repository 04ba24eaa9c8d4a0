// hmpc_kernels.hip -- batched MPC/QP solve for MI355X (gfx950), fp64 (and
// an fp32 build of the same kernel for BASELINE configs[4]).
//
// One workgroup of W = ceil(6N/64) wavefronts solves ONE QP instance of the
// reference's Mpc.build_qp/solve_qp (src/mpc_cvx_euler_3f.py:96-160; 2f
// :96-158) to its exact optimum, on the CONDENSED problem (states eliminated
// through the dynamics; NV = 6N input variables).  Lane v owns variable
// v = 6*i + c (stage i, component c).  Phases (DESIGN.md "Kernel"):
//
//   0  coalesced load of the instance's inputs into LDS
//   1  per-stage linearisation = Mpc.gen_dt_dynamics (3f :71-94, 2f :70-94)
//   2  wave-uniform sweeps in registers (every lane computes the same values):
//      free response xbar, gradient terms d_t = W_{t-1}(xbar_t - r_{t-1}),
//      and the backward cost-to-go S_t = W_{t-1} + Ad_t' S_{t+1} Ad_t.
//      S_t is block-structured (Ad never mixes translation and rotation and
//      Q is diagonal): 3 x (p_a, v_a) 2x2 + (yaw, w_z) 2x2 + (roll, pitch,
//      w_x, w_y) 4x4 = 22 unique entries.
//   3  lane v builds row v of the condensed Hessian (lower triangle: all the
//      Cholesky reads) and its gradient entry: the impulse response
//      e_j = Phi(j+1,i+1) B_i e_c (gradient), the diagonal block from
//      S_{i+1} B_i e_c, and g_j = Phi(i+1,j+1)' S_{i+1} B_i e_c (j < i).
//   4  right-looking Cholesky H = L L' with the trailing row in registers.
//      Every step shifts the row by one register as it updates it, so step k
//      always reads register 0 and one loop body serves 8 consecutive k (a
//      runtime loop: the kernel stays small enough for the instruction
//      cache).  L goes to LDS column-major.
//   5  unconstrained optimum v0 = -H^-1 h (two triangular sweeps)
//   6  Goldfarb-Idnani dual active set in range-space form: instead of
//      J = L^-T Q it keeps an orthonormal basis Qw of L^-1 N_A (lane v holds
//      row v of Qw in registers) and the triangular R with L^-1 N_A = Qw R
//      (LDS).  Adding constraint p costs one forward sweep w = L^-1 n_p, a
//      Gram-Schmidt projection against Qw and one backward sweep
//      z = L^-T w_perp; dropping one costs Givens rotations on R and Qw.
//      Constraints: torque box (:123-128), fz box + friction pyramid
//      (:141-146), z >= 0.1 (:129, dense rows over fz through the dynamics);
//      swing / 2f fy equalities (:134-136, 2f :129) are eliminated as fixed
//      variables.
//   7  outputs: u* (coalesced), x* by forward simulation, objective incl.
//      its constant term evaluated on (x*, u*), status, iterations.
//
// No MFMA: every product is a tiny dense block or a rank-1 update.
//
// The arithmetic type `real` is fixed per object: double (the product path,
// launch_solve_n<N>) or, built with -DHMPC_REAL=float, float
// (launch_solve_n<N>_f32: inputs and outputs stay fp64 in HBM, every
// operation in between is fp32).  Everything but the launcher sits in an
// anonymous namespace, so the two builds never share a symbol.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <stdio.h>
#include <string>
#include <utility>

#include "hmpc_internal.h"
#include "hmpc_model.h"

#ifndef HMPC_REAL
#define HMPC_REAL double
#define HMPC_REAL_FP64 1   // (the default fp64 objects)
#endif

namespace hmpc {
namespace {

using real = HMPC_REAL;
constexpr bool kF32 = sizeof(real) == 4;
// fp32 solve + fp64 iterative refinement on its final active set
// (HMPC_PREC_F32_REFINED, configs[4]): the object is built with
// -DHMPC_F32_REFINE=1, the number of corrections is a.refine (run time)
#ifndef HMPC_F32_REFINE
#define HMPC_F32_REFINE 0
#endif
constexpr bool kRefine = kF32 && HMPC_F32_REFINE;
// the refinement's acceptance: scaled row violations and negative multipliers
// beyond this send the instance to the fp64 pass
constexpr double kRefineTol = 1e-9;
// and the largest last correction accepted as converged
constexpr double kRefineDu = 4e-6;
// ... and the early exit of the corrections
constexpr double kRefineStop = 4e-7;
// feasibility tolerance of the slack scan and the relative threshold on
// |w_perp|^2 for a usable primal direction, per precision
constexpr real kTolR = kF32 ? real(2e-4) : real(kTol);
constexpr real kZnRel = kF32 ? real(1e-10) : real(1e-24);

__device__ __forceinline__ void sincos_r(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ void sincos_r(float x, float* s, float* c) { sincosf(x, s, c); }

// compile-time loop: f(std::integral_constant<int, i>) for i in [Begin, End).
// Every index into a register-resident row goes through this (or the ladders
// below), so no row ever lands in scratch memory.
template <int Begin, typename F, int... Is>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Begin + Is>{}), ...);
}
template <int Begin, int End, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (End > Begin) sfor_impl<Begin>(std::make_integer_sequence<int, End - Begin>{}, f);
}
// f(l) for l = L, L+1, ... while l < n (n wave-uniform): nested, so the first
// failing test jumps past every remaining body.
template <int L, int LMAX, typename F>
__device__ __forceinline__ void ladder(int n, F&& f) {
  if constexpr (L < LMAX) {
    if (L < n) {
      f(std::integral_constant<int, L>{});
      ladder<L + 1, LMAX>(n, f);
    }
  }
}
// f(l) for the single l == n (n wave-uniform).
template <int L, int LMAX, typename F>
__device__ __forceinline__ void at_index(int n, F&& f) {
  if constexpr (L < LMAX) {
    if (L == n) f(std::integral_constant<int, L>{});
    else at_index<L + 1, LMAX>(n, f);
  }
}

// Empty asm that claims to read and write x: pins the value into a VGPR pair
// at this point, so the scheduler cannot sink a step's FMAs past the next
// step's loads (which would real the live set and spill the row).
__device__ __forceinline__ void pin(real& x) { asm volatile("" : "+v"(x)); }
// A wave-uniform 0 the compiler cannot see through.  Added to an LDS address
// it keeps the loads behind it from being hoisted above this point (the
// scheduler otherwise pulls every load of a long unrolled loop to the top
// and spills).
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}
// Per-lane select on a wave-uniform 64-bit lane mask (bit l set: lane l
// takes t).  With a compile-time mask this is one v_cndmask per 32 bits and
// an s_mov of the constant -- no v_cmp of the lane id against a step index.
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
__device__ __forceinline__ float msel(uint64_t m, float t, float f) {
  return __uint_as_float(msel(m, __float_as_uint(t), __float_as_uint(f)));
}
typedef __attribute__((address_space(3))) real lds_real;

// LDS loads the scheduler cannot move.  hipcc sinks prefetches next to their
// use and then waits with lgkmcnt(0); these are issued where they stand, and
// the value is valid only after the matching lds_wait (s_waitcnt lgkmcnt(n),
// n = LDS instructions issued after the load), which also ties the registers
// so nothing reads them earlier.
typedef real real2 __attribute__((ext_vector_type(2)));
constexpr int RB = (int)sizeof(real);   // bytes per element
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)p;   // low 32 bits of the flat address = LDS offset
}
// two consecutive elements (OFF in bytes); one element
template <int OFF>
__device__ __forceinline__ void lds_ld2(real2& v, unsigned base) {
  if constexpr (kF32) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF) : "memory");
  else asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF) : "memory");
}
__device__ __forceinline__ void lds_ld1(real& v, unsigned addr) {
  if constexpr (kF32) asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  else asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(addr) : "memory");
}
template <int CNT>
__device__ __forceinline__ void lds_wait(real2& a, real2& b, real2& c, real2& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "i"(CNT));
}
template <int CNT>
__device__ __forceinline__ void lds_wait(real2& a, real2& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(CNT));
}
template <int CNT>
__device__ __forceinline__ void lds_wait(real& a, real& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(CNT));
}
template <int CNT>
__device__ __forceinline__ void lds_wait(real& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(CNT));
}

// Drain a ring of hand-counted LDS loads: wait for every load, and keep the
// ring's registers allocated until then.  The compiler does not know an asm
// load writes its register asynchronously; a ring slot whose last load is
// never read (the tail's dummy loads) is dead to it, and a value it placed
// in that register before the wait would be overwritten when the load lands.
template <int R>
__device__ __forceinline__ void lds_drain(real (&r)[R]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  sfor<0, R>([&](auto ic) __attribute__((always_inline)) { pin(r[decltype(ic)::value]); });
}

template <int W>
struct Blk {
  // LDS ordering point.  One wave: LDS instructions of a wave execute in
  // order, so only the compiler has to be kept from reordering them.
  __device__ __forceinline__ static void sync() {
    if constexpr (W == 1) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    else __syncthreads();
  }
  // `red` must hold >= 2*W doubles; calls are bracketed by barriers (W > 1)
  // so consecutive calls may reuse it.
  __device__ __forceinline__ static real sum(real x, real* red) {
    x = wave_sum(x);
    if constexpr (W == 1) {
      return x;
    } else {
      __syncthreads();
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
      __syncthreads();
      real s = 0.0;
#pragma unroll
      for (int w = 0; w < W; ++w) s += red[w];
      return s;
    }
  }
  __device__ __forceinline__ static void argmin(real& v, int& i, real* red) {
    wave_argmin<true>(v, i);
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
  __device__ __forceinline__ static real bcast(real x, int l, real* red) {
    if constexpr (W == 1) {
      return rdlane(x, l);
    } else {
      __syncthreads();
      if ((int)threadIdx.x == l) red[0] = x;
      __syncthreads();
      return red[0];
    }
  }
  // first lane (over the workgroup) with flag set, or -1
  __device__ __forceinline__ static int first(bool flag, real* red) {
    unsigned long long m = __ballot(flag);
    int f = m ? (int)__builtin_ctzll(m) + (int)(threadIdx.x & ~63u) : 0x7fffffff;
    if constexpr (W > 1) {
      int* ired = reinterpret_cast<int*>(red);
      __syncthreads();
      if ((threadIdx.x & 63) == 0) ired[threadIdx.x >> 6] = f;
      __syncthreads();
      f = ired[0];
#pragma unroll
      for (int w = 1; w < W; ++w) f = ired[w] < f ? ired[w] : f;
    }
    return f == 0x7fffffff ? -1 : uni(f);
  }
};

// ----------------------------------------------------------------------------
// LDS layout (in doubles), one instance per workgroup
// ----------------------------------------------------------------------------
// NVM > 0: the compacted kernel (one wave) for instances with at most NVM
// free variables (hmpc_classify_kernel), NVM = 0: every instance (NV = 6N).
// QM > 0 overrides the active-set capacity.
template <int N, int NVM = 0, int QM = 0>
struct Lay {
  static constexpr int NVF = 6 * N;                 // the full input vector (outputs)
  static constexpr int NV = NVM > 0 ? NVM : NVF;    // variables (lanes) of the factor
  static constexpr int W = (NV + 63) / 64;
  static constexpr int NT = 64 * W;
  static_assert(W > 1 || NVF <= NT, "one-wave kernels keep the full vector in XS");
  // active-set capacity (registers for Qw, LDS for R); the largest active set
  // seen over 65536 random N=10 instances is 12
  static constexpr int QMAX = QM > 0 ? QM : (NV < 20 ? NV : (N <= 10 ? 20 : 48));
  static constexpr int e2(int n) { return (n + 1) & ~1; }
  static constexpr int NS = 22;                    // unique entries of S_t
  static constexpr int LCN = NV * (NV + 1) / 2;    // packed L
  // persistent
  static constexpr int XIN = 0;                    // [12]
  static constexpr int CC = XIN + 12;              // [N] contact schedule
  static constexpr int CS = CC + e2(N);            // [N][2] cos, sin of yaw
  static constexpr int BW = CS + 2 * N;            // [N][3][6] rows 9..11 of Bd_k
  static constexpr int ZB = BW + 18 * N;           // [N+1] free-response heights
  static constexpr int XS = ZB + e2(N + 1);        // [NT] primal broadcast
  static constexpr int RED = XS + NT;              // [4] cross-wave reductions (W <= 2)
  static constexpr int ZR = RED + 4;               // [2] a 0.0 for masked lanes' loads
  static constexpr int XRV = ZR + 2;               // [4] x_ref view for phase 7: address (8 B), row stride
  // active-set state (phase 6); the Cholesky's column buffers overlay it
  static constexpr int G0 = XRV + 4;
  static constexpr int UA = G0;                    // [QMAX] active multipliers
  static constexpr int ACT = UA + QMAX;            // [QMAX] active ids (int)
  static constexpr int CB = ACT + QMAX;            // [QMAX] c = Qw' w
  static constexpr int GV = CB + QMAX;             // [QMAX][2] Givens of a drop
  static constexpr int SD = GV + 2 * QMAX;         // [QMAX] subdiagonal scratch
  static constexpr int RM = SD + QMAX;             // packed upper R, col l at l(l+1)/2
  static constexpr int GS = RM + e2(QMAX * (QMAX + 1) / 2);   // [W][QMAX] Gram-Schmidt partials (W > 1)
  static constexpr int GEND = GS + (W > 1 ? W * QMAX : 0);
  static constexpr int COLB = G0;                  // [2][NT+8] (phase 4 only), 16-B aligned
  static_assert((G0 & 1) == 0, "column buffers must be 16-B aligned");
  static constexpr int U0 = (GEND > COLB + 2 * (NT + 8)) ? GEND : COLB + 2 * (NT + 8);
  // union A (phases 0-3)
  static constexpr int XLIN = U0;                  // [N][12]  rows 0..N-1
  static constexpr int PF = XLIN + 12 * N;         // [N][3]
  static constexpr int XREF = PF + e2(3 * N);      // [N][12]
  static constexpr int SS = XREF + 12 * N;         // [N][22]  S_{t}, t = 1..N
  static constexpr int DG = SS + NS * N;           // [N][12]  d_t, t = 1..N
  static constexpr int AJ = DG + 12 * N;           // [N][6]   adjoint a_t rows 6..11, t = 1..N
  static constexpr int ENDA = AJ + 6 * N;
  // union B (phases 4-7)
  static constexpr int LC = U0;                    // M = L diag(L)^-1, column-major packed
  static constexpr int XO = U0;                    // x* staging (after L is dead)
  static constexpr int ENDB = LC + e2(LCN);
  static constexpr int TOTAL0 = ENDA > ENDB ? ENDA : ENDB;
  // fp32 + fp64 refinement (HMPC_F32_REFINE builds): an fp64 region after the
  // rest, offsets in doubles from R64 -- the stage data of gen_dt_dynamics in
  // fp64 (cos/sin, rows 9..11 of Bd), u in full order, the adjoint rows
  // 6..11, the rolled-out heights z_k, each lane's full-order slot (int)
  // Part of it (R64LO) overlays the fp32 stage data CS..ZB, dead once the
  // active set is final (fp32 builds only run the refinement)
  static constexpr int R64LO = CS;                   // in reals, 8-B aligned
  static constexpr int DCS = 0;                      // [N][2]          (R64LO)
  static constexpr int DU = DCS + 2 * N;             // [6N]            (R64LO)
  static constexpr int DXZ = DU + NVF;               // [N+1]           (R64LO)
  static_assert((CS & 1) == 0 && (DXZ + N + 1) * (8 / RB) <= XS - CS, "fp64 overlay");
  static constexpr int R64 = (TOTAL0 + 1) & ~1;     // in reals, 8-B aligned
  static constexpr int DBW = 0;                      // [N][3][6]       (R64)
  static constexpr int DAJ = DBW + 18 * N;           // [N][6]
  static constexpr int DXR = DAJ + 6 * N;            // [N][12] x_ref
  static constexpr int DSLOT = DXR + 12 * N;         // [NT] int
  static constexpr int DTOT = DSLOT + NT / 2;
  static constexpr int TOTAL = kRefine ? R64 + DTOT * (8 / RB) : TOTAL0;
  static_assert(12 * (N + 1) <= LCN, "x* staging does not fit");
  static_assert(!kRefine || 24 * (N + 1) + 1 <= LCN, "fp64 x* staging does not fit");
  // start of column k of L (rows k..NV-1)
  __host__ __device__ static constexpr int cb(int k) { return k * NV - ((k * (k - 1)) >> 1); }
};

__device__ __forceinline__ int loff(int r) { return (r * (r + 1)) >> 1; }

// prefetch depth (steps) of the two-wave sweeps' LDS ring (two loads a step:
// lgkmcnt waits of 2 kRing2 - 2 <= 15)
constexpr int kRing2 = 8;
// and of the one-wave sweeps (one load a step; 8 measured -1.4 %)
constexpr int kRing1 = 4;

// ----------------------------------------------------------------------------
// triangular sweeps.  The factor is kept as the unit lower M = L diag(L)^-1,
// column-major packed in LDS with 1/L_kk in the (unit) diagonal slot of
// column k.  L^-1 b = diag(1/L) M^-1 b and L^-T b = M^-T (diag(1/L) b): one
// step's dependent chain is just readlane -> fma.
// ----------------------------------------------------------------------------
// Two-wave sweeps: every wave gets all NV entries of the right-hand side
// (rows lane and lane + 64).  `red` must hold NT doubles here (the XS row).
__device__ __forceinline__ void sweep_stage(real b, real& a0, real& a1, real* buf) {
  const int lane = threadIdx.x & 63;
  __syncthreads();
  buf[threadIdx.x] = b;
  __syncthreads();
  a0 = buf[lane];
  a1 = buf[lane + 64];
}
// y = L^-1 b (lane v holds b_v) from the LDS copy of M (the one-wave
// kernel's phase-5 forward sweep instead rides along the Cholesky).  Loads
// of step s+4 are issued at step s (a 4-deep ring of hand-counted loads).
// s0 (uniform, a
// multiple of 4): b is zero above row s0, so are the first s0 entries of y
// and the sweep starts there (constraint normals are sparse: a box or
// friction row of stage j starts at 6j).
template <class L>
__device__ __forceinline__ real tri_fwd_lds(real acc, const real* Mc, const real* zero,
                                              real dinv, real* red, int nf, int s0 = 0) {
  constexpr int NV = L::NV;
  constexpr int SEND = L::W == 1 ? (NV + 3) & ~3 : ((NV + kRing2 - 1) / kRing2) * kRing2;   // padded (steps >= NV are no-ops)
  const int tid = threadIdx.x;
  if constexpr (L::W == 1) {
    // M[tid][t] for tid > t sits at Mc[cb(t) + tid - t]; other lanes read a 0.
    // Step t's lane mask (lanes t+1 .. NV-1) and address follow from step
    // t-1's by a shift and an add (round 5: the per-step compare / select
    // chain on the scalar unit was ~12 of the step's ~19 instructions, and a
    // wave issues one instruction per 4 cycles).  Steps run in whole groups
    // of kRing1 up to SE = nf rounded up: the columns nf .. SE-1 were zeroed
    // after the Cholesky (sweep_pad_zero), the lanes >= nf hold 0.
    // whole ring groups from s0 on: only columns nf .. nf+kRing1-2 are
    // zeroed past nf (sweep_pad_zero), so s0 is held to a group boundary here
    // rather than trusted from the caller
    s0 &= ~(kRing1 - 1);
    const unsigned base = lds_addr(Mc + tid), zaddr = lds_addr(zero);
    constexpr uint64_t kLive = NV >= 64 ? ~0ull : ((1ull << NV) - 1);
    auto mask = [&](int t) -> uint64_t { return t < NV - 1 ? kLive & ~((2ull << t) - 1) : 0; };
    auto off = [&](int t) -> unsigned { return (unsigned)RB * (unsigned)(L::cb(t) - t); };
    const int SE = (nf + kRing1 - 1) & ~(kRing1 - 1);
    real ring[kRing1];
    sfor<0, kRing1>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      lds_ld1(ring[j], msel(mask(s0 + j), base + off(s0 + j), zaddr));
    });
    // the next ring refill: step t = s0 + kRing1
    uint64_t mk = mask(s0 + kRing1);
    unsigned ad = base + off(s0 + kRing1);
    unsigned inc = (unsigned)RB * (unsigned)(NV - 1 - (s0 + kRing1));   // cb(t+1)-(t+1) - (cb(t)-t) = NV-1-t
#pragma unroll 1
    for (int s = s0; s < SE; s += kRing1) {
      sfor<0, kRing1>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const int sj = s + j;
        const real ys = rdlane(acc, sj);
        lds_wait<kRing1 - 1>(ring[j]);
        acc = fma(-ring[j], ys, acc);
        lds_ld1(ring[j], msel(mk, ad, zaddr));
        mk = (mk << 1) & kLive;
        ad += inc;
        inc -= (unsigned)RB;
      });
    }
    lds_drain(ring);   // the ring's last loads are dummies
  } else {
    static_assert(L::W == 2 && NV > 64, "two-wave sweeps only");
    // Every wave runs the whole sweep on all NV rows (two per lane: lane and
    // lane + 64) instead of exchanging one value per step through LDS and a
    // barrier; wave w keeps the rows it owns.  Loads run 4 steps ahead.
    const int lane = tid & 63;
    real a0, a1;
    sweep_stage(acc, a0, a1, red);
    const unsigned b0 = lds_addr(Mc + lane), b1 = lds_addr(Mc + lane + 64), zaddr = lds_addr(zero);
    auto ad0 = [&](int s) -> unsigned {
      return (lane > s && s < NV) ? b0 + (unsigned)RB * (unsigned)(L::cb(s) - s) : zaddr;
    };
    auto ad1 = [&](int s) -> unsigned {
      return (lane + 64 > s && lane + 64 < NV && s < NV) ? b1 + (unsigned)RB * (unsigned)(L::cb(s) - s) : zaddr;
    };
    constexpr int RD = kRing2;   // s0 is a multiple of RD here
    real r0[RD], r1[RD];
    sfor<0, RD>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      lds_ld1(r0[j], ad0(s0 + j));
      lds_ld1(r1[j], ad1(s0 + j));
    });
    auto steps = [&](int s, const real& src, int off) __attribute__((always_inline)) {
      sfor<0, RD>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const int sj = s + j;
        const real ys = rdlane(src, sj - off);
        lds_wait<2 * RD - 2>(r0[j], r1[j]);
        a0 = fma(-r0[j], ys, a0);
        a1 = fma(-r1[j], ys, a1);
        lds_ld1(r0[j], ad0(sj + RD));
        lds_ld1(r1[j], ad1(sj + RD));
      });
    };
#pragma unroll 1
    for (int s = s0; s < 64; s += RD) steps(s, a0, 0);
#pragma unroll 1
    for (int s = (s0 > 64 ? s0 : 64); s < SEND; s += RD) steps(s, a1, 64);
    lds_drain(r0);   // the ring's last loads are dummies
    lds_drain(r1);
    acc = tid < 64 ? a0 : a1;
  }
  // lane v's accumulator is final once step v has read it
  return acc * dinv;
}
// z = L^-T b (lane v holds b_v), M from the LDS copy.  One wave: loads of
// step s-4 are issued at step s (a 4-deep ring of hand-counted loads).
template <class L>
__device__ __forceinline__ real tri_bwd(real acc, const real* Mc, const real* zero,
                                          real dinv, real* red, int nf) {
  constexpr int NV = L::NV;
  const int tid = threadIdx.x;
  const int cbt = tid < NV ? L::cb(tid) : 0;
  acc *= dinv;
  if constexpr (L::W == 1) {
    // M[t][tid] for tid < t sits at Mc[cbt + t - tid]; other lanes read a 0.
    // From the last free step nf-1 down: step t's mask (lanes 0 .. t-1) is
    // step t+1's shifted right, its address one entry lower (round 5, as in
    // tri_fwd_lds).  The last group's steps below 0 read 0 on every lane.
    const unsigned base = lds_addr(Mc + cbt - tid), zaddr = lds_addr(zero);
    auto mask = [&](int t) -> uint64_t { return t > 0 ? (1ull << t) - 1 : 0; };
    const int top = nf - 1;
    real ring[kRing1];
    sfor<0, kRing1>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      lds_ld1(ring[j], msel(mask(top - j), base + (unsigned)RB * (unsigned)(top - j), zaddr));
    });
    uint64_t mk = mask(top - kRing1);   // the next ring refill: step top - kRing1
    unsigned ad = base + (unsigned)RB * (unsigned)(top - kRing1);
#pragma unroll 1
    for (int s = top; s >= 0; s -= kRing1) {
      sfor<0, kRing1>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const int sj = s - j;
        // (steps below 0 of the last group read lane 0, a free variable's
        // finite value, times the 0 loaded from zaddr -- not a padding lane,
        // whose value need not be finite: ADVICE r5)
        const real zs = rdlane(acc, sj > 0 ? sj : 0);
        lds_wait<kRing1 - 1>(ring[j]);
        acc = fma(-ring[j], zs, acc);
        lds_ld1(ring[j], msel(mk, ad, zaddr));
        mk >>= 1;
        ad -= (unsigned)RB;
      });
    }
    lds_drain(ring);   // the ring's last loads are dummies
  } else {
    static_assert(L::W == 2 && NV > 64, "two-wave sweeps only");
    // as in tri_fwd_lds: each wave sweeps all rows (lane, lane + 64)
    const int lane = tid & 63;
    real a0, a1;
    sweep_stage(acc, a0, a1, red);
    const unsigned b0 = lds_addr(Mc + L::cb(lane) - lane);
    const unsigned b1 = lds_addr(Mc + (lane + 64 < NV ? L::cb(lane + 64) - (lane + 64) : 0));
    const unsigned zaddr = lds_addr(zero);
    auto ad0 = [&](int s) -> unsigned { return (lane < s && s < NV && s >= 0) ? b0 + (unsigned)RB * (unsigned)s : zaddr; };
    auto ad1 = [&](int s) -> unsigned {
      return (lane + 64 < s && s < NV && s >= 0) ? b1 + (unsigned)RB * (unsigned)s : zaddr;
    };
    constexpr int RD = kRing2;
    constexpr int STOP2 = ((NV + RD - 1) / RD) * RD - 1;   // first step, padded to the ring
    real r0[RD], r1[RD];
    sfor<0, RD>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      lds_ld1(r0[j], ad0(STOP2 - j));
      lds_ld1(r1[j], ad1(STOP2 - j));
    });
    auto steps = [&](int s, const real& src, int off) __attribute__((always_inline)) {
      sfor<0, RD>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const int sj = s - j;
        const real zs = rdlane(src, sj - off);
        lds_wait<2 * RD - 2>(r0[j], r1[j]);
        a0 = fma(-r0[j], zs, a0);
        a1 = fma(-r1[j], zs, a1);
        lds_ld1(r0[j], ad0(sj - RD));
        lds_ld1(r1[j], ad1(sj - RD));
      });
    };
#pragma unroll 1
    for (int s = STOP2; s >= 64; s -= RD) steps(s, a1, 64);
#pragma unroll 1
    for (int s = 63; s >= 0; s -= RD) steps(s, a0, 0);
    lds_wait<0>(r0[0], r1[0]);
    acc = tid < 64 ? a0 : a1;
  }
  return acc;   // lane v's accumulator is final once step v has read it
}

// ----------------------------------------------------------------------------
// the kernel
// ----------------------------------------------------------------------------
// Diagnostic build only (-DHMPC_STAMPS, tools/phase_stamps.py): s_memtime at
// every phase boundary, written over the instance's x* row at the end.  The
// product build compiles these to nothing.
#ifdef HMPC_STAMPS
#define HMPC_STAMP(i) (stamp_[i] = __builtin_amdgcn_s_memtime())
// accumulated sub-phase timers of the active set (slots 9..14)
#define HMPC_TIC(v) const long long v = __builtin_amdgcn_s_memtime()
#define HMPC_TOC(slot, v) (stamp_[slot] += __builtin_amdgcn_s_memtime() - (v))
#elif defined(HMPC_MARKS)   // phase markers in the .s (register-pressure work)
#define HMPC_STAMP(i) asm volatile(";@@PHASE " #i)
#define HMPC_TIC(v) asm volatile(";@@TIC " #v)
#define HMPC_TOC(slot, v) asm volatile(";@@TOC " #slot)
#else
#define HMPC_STAMP(i) ((void)0)
#endif
#if !defined(HMPC_STAMPS) && !defined(HMPC_MARKS)
#define HMPC_TIC(v) ((void)0)
#define HMPC_TOC(slot, v) ((void)0)
#endif

// issue priority of the chain-bound phases (the Cholesky through the active
// set): a wave in its dependent pivot/sweep chains issues first; the
// co-resident wave's throughput phases (sweeps of phase 2, Hessian rows,
// outputs) fill the gaps: +0.4-0.9 %.  Between the split's classes: the full
// kernel's waves hold the small-batch critical path (its instances are the
// longest), so they run at priority 2 outside the chain phases (3 inside),
// the compacted kernel's at 0 / 1: configs[1] +1.6 %, configs[2] and
// B = 16384 unchanged (profiles/r03_ab.json).
constexpr int kPrioCmp = 1;
constexpr int kPrioFullBase = 2;
#ifndef HMPC_WAVES_PER_EU
#define HMPC_WAVES_PER_EU(W) ((W) == 1 ? 2 : 1)
#endif
// waves / SIMD of the split's compacted class (NVM <= kCmp3W): fp64 3
// (<= 168 VGPRs), fp32 4 (<= 128, 12 B/lane of spill); a wider compacted
// kernel (2f's 5N-wide full class) runs like the full one, fp64 2, fp32 3
// (the fp32 + fp64 refinement build: 2 waves / SIMD for every class, the refinement's
// fp64 state fits without scratch: full 214 VGPRs; at 3 waves the compacted
// class spilled 60 B/lane)
constexpr int kCmpWaves = kRefine ? 2 : (sizeof(real) == 4 ? 4 : 3);
constexpr int kWideCmpWaves = kRefine ? 2 : (sizeof(real) == 4 ? 3 : 2);
constexpr int kCmp3W = 48;
// The kernel's argument block through an opaque kernarg-segment pointer:
// reads through it are fresh scalar loads where they stand, so the compiler
// does not keep the arguments of an early phase alive (in SGPRs, then
// spilled) until a late phase reads them again.  Device pass only (the host
// pass merely parses kernel bodies).
__device__ __forceinline__ const SolveArgs& opaque_args(const SolveArgs& a) {
#ifdef __HIP_DEVICE_COMPILE__
  typedef const __attribute__((address_space(4))) SolveArgs karg_t;
  karg_t* ap = (karg_t*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ap));
  return *(const SolveArgs*)ap;
#else
  return a;
#endif
}

template <int VAR, int N, typename R, int NVM = 0, int QM = 0>
__global__ void __launch_bounds__((Lay<N, NVM, QM>::NT),
                                  (NVM > 0 && NVM <= kCmp3W ? kCmpWaves
                                   : (NVM > 0 ? kWideCmpWaves : HMPC_WAVES_PER_EU((Lay<N, NVM, QM>::W)))))
solve_kernel(SolveArgs a) {
  static_assert(sizeof(R) == sizeof(real), "one arithmetic type per build");
  using L = Lay<N, NVM, QM>;
  static_assert(NVM == 0 || L::W == 1, "the compacted kernel is one wave");
  constexpr int NV = L::NV;
  constexpr int W = L::W;
  constexpr int NT = L::NT;
  constexpr int QMAX = L::QMAX;
  using B = Blk<W>;
  __shared__ __attribute__((aligned(16))) real sm[L::TOTAL];
  real* red = sm + L::RED;
  real* xs = sm + L::XS;
#ifdef HMPC_STAMPS
  long long stamp_[16] = {0};
#endif
  HMPC_STAMP(0);
  constexpr bool kCmpCls = NVM > 0 && NVM <= kCmp3W;   // the split's compacted class
  if constexpr (!kCmpCls) __builtin_amdgcn_s_setprio(kPrioFullBase);

  const int tid = threadIdx.x;
  // split launch (launch_solve_n<N>): block i solves the i-th instance of this
  // kernel's class list; blocks beyond the list's length have no work
  int64_t b = blockIdx.x;
  if (a.list) {
    if (a.lpt_hi >= 0) {   // stance-count buckets, costliest first (a.lpt)
      int i = blockIdx.x, s = a.lpt_hi;
      for (; s >= a.lpt_lo; --s) {
        const int c = a.list_count[s];
        if (i < c) break;
        i -= c;
      }
      if (s < a.lpt_lo) return;
      b = a.list[(int64_t)s * a.B + i];
    } else {
      if ((int)blockIdx.x >= *a.list_count) return;
      b = a.list[blockIdx.x];
    }
  }
  const real dt = a.dt;
  const real dtm = dt / real(a.m);

  // ---------------- phase 0: coalesced loads --------------------------------
  // x_ref / pf / C may be strided views (a resident plan, path_plan_grab
  // src/robotrunner.py:228-230: rows k, k+f, ...; batch stride 0 = shared)
  const double* xrf = a.x_ref + b * a.xref_bs;
  if (tid == 0) {   // kept in LDS, not in SGPRs, until phase 7 reads x_ref again
    reinterpret_cast<const double**>(sm + L::XRV)[0] = xrf;
    reinterpret_cast<int*>(sm + L::XRV + 2)[0] = a.xref_rs;
  }
  // Every global load is issued before the first LDS store (one memory
  // round trip instead of one per array); out-of-range lanes load element 0
  // of their array and discard it.
  {
    constexpr int NR = (12 * N + NT - 1) / NT, NP = (3 * N + NT - 1) / NT, NCC = (N + NT - 1) / NT;
    const double* xp = a.x_lin + b * 12 * (N + 1);
    const int mode = a.shift_mode;
    real vi, vr[NR], vp[NP], vc[NCC], vl[NR];
    vi = a.x_in[b * 12 + (tid < 12 ? tid : 0)];
    sfor<0, NR>([&](auto itc) __attribute__((always_inline)) {
      constexpr int it = decltype(itc)::value;
      const int i = tid + it * NT, ic = i < 12 * N ? i : 0;
      const int r = ic / 12, c = ic - 12 * r;
      vr[it] = xrf[r * a.xref_rs + c];
      // x_lin rows 0..N-1: given (mode 0) or the time shift of x_prev
      // (mode 2: [x_in; x_prev[2:]; x_prev[N]], 3f :59-62; row 0 is x_in,
      // which lane i < 12 already holds in vi)
      vl[it] = xp[mode == 0 ? ic : ((r + 1 <= N ? r + 1 : N) * 12 + c)];
    });
    sfor<0, NP>([&](auto itc) __attribute__((always_inline)) {
      constexpr int it = decltype(itc)::value;
      const int i = tid + it * NT, ic = i < 3 * N ? i : 0;
      const int r = ic / 3, c = ic - 3 * r;
      vp[it] = a.pf[b * a.pf_bs + r * a.pf_rs + c];
    });
    sfor<0, NCC>([&](auto itc) __attribute__((always_inline)) {
      constexpr int it = decltype(itc)::value;
      const int i = tid + it * NT;
      vc[it] = a.C[b * a.C_bs + (i < N ? i : 0)];
    });
    const real mu_b = a.mu ? a.mu[b] : a.mu_default;
    if (tid < 12) sm[L::XIN + tid] = vi;
    if (tid == 0) sm[L::ZR + 1] = mu_b;   // read again in phase 6
    sfor<0, NR>([&](auto itc) __attribute__((always_inline)) {
      constexpr int it = decltype(itc)::value;
      const int i = tid + it * NT;
      if (i < 12 * N) {
        sm[L::XREF + i] = vr[it];
        if (mode != 1) sm[L::XLIN + i] = (mode == 2 && i < 12) ? vi : vl[it];
      }
    });
    sfor<0, NP>([&](auto itc) __attribute__((always_inline)) {
      constexpr int it = decltype(itc)::value;
      const int i = tid + it * NT;
      if (i < 3 * N) sm[L::PF + i] = vp[it];
    });
    sfor<0, NCC>([&](auto itc) __attribute__((always_inline)) {
      constexpr int it = decltype(itc)::value;
      const int i = tid + it * NT;
      if (i < N) sm[L::CC + i] = vc[it];
    });
    if (mode == 1) {   // [x_in; x_ref]   (3f :52-53)
      __syncthreads();
      for (int i = tid; i < 12 * N; i += NT)
        sm[L::XLIN + i] = i < 12 ? sm[L::XIN + i] : sm[L::XREF + i - 12];
    }
  }
  __syncthreads();
  HMPC_STAMP(1);

  // ---------------- phase 1: gen_dt_dynamics (lane k < N) -------------------
  // (hmpc_model.h's stage_dynamics() inline: the call form costs 8 B/lane
  // more scratch in this kernel)
  if (tid < N) {
    const int k = tid;
    const real psi = sm[L::XLIN + 12 * k + 5];
    real sp, cp;
    sincos_r(psi, &sp, &cp);
    // rz(psi) = [[c, s, 0], [-s, c, 0], [0, 0, 1]]   (src/utils.py:46-51)
    const real Rz[3][3] = {{cp, sp, 0.0}, {-sp, cp, 0.0}, {0.0, 0.0, 1.0}};
    real d[3], rf[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] = sm[L::PF + 3 * k + i] - sm[L::XLIN + 12 * k + i];
    // rf = rh + Rz (pf - p)   (:84)
#pragma unroll
    for (int i = 0; i < 3; ++i) rf[i] = real(a.rh[i]) + (Rz[i][0] * d[0] + Rz[i][1] * d[1] + Rz[i][2] * d[2]);
    real T[3][3], Jw[3][3], RzT[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) RzT[i][j] = Rz[j][i];
    // J_w_inv = Rz Jinv Rz'   (:86)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        T[i][j] = Rz[i][0] * real(a.Jinv[0 * 3 + j]) + Rz[i][1] * real(a.Jinv[1 * 3 + j]) + Rz[i][2] * real(a.Jinv[2 * 3 + j]);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Jw[i][j] = T[i][0] * RzT[0][j] + T[i][1] * RzT[1][j] + T[i][2] * RzT[2][j];
    real Bwt[3][3], Bwf[3][3];
    // B[9:12, 3:6] = J_w_inv Rz'   (:89)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Bwt[i][j] = Jw[i][0] * RzT[0][j] + Jw[i][1] * RzT[1][j] + Jw[i][2] * RzT[2][j];
    real w[3];
    if constexpr (VAR == 3) {   // rhat = hat(Rz' rf); B[9:12,0:3] = Jw rhat   (:85,88)
#pragma unroll
      for (int i = 0; i < 3; ++i) w[i] = RzT[i][0] * rf[0] + RzT[i][1] * rf[1] + RzT[i][2] * rf[2];
    } else {                    // rhat = hat(rf); B[9:12,0:3] = (Jw Rz') rhat   (2f :84,88)
#pragma unroll
      for (int i = 0; i < 3; ++i) w[i] = rf[i];
    }
    // hat (src/utils.py:21-25)
    const real hw[3][3] = {{0.0, -w[2], w[1]}, {w[2], 0.0, -w[0]}, {-w[1], w[0], 0.0}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if constexpr (VAR == 3)
          Bwf[i][j] = Jw[i][0] * hw[0][j] + Jw[i][1] * hw[1][j] + Jw[i][2] * hw[2][j];
        else
          Bwf[i][j] = Bwt[i][0] * hw[0][j] + Bwt[i][1] * hw[1][j] + Bwt[i][2] * hw[2][j];
      }
    real* bw = sm + L::BW + 18 * k;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        bw[i * 6 + j] = Bwf[i][j] * dt;
        bw[i * 6 + 3 + j] = Bwt[i][j] * dt;
      }
    sm[L::CS + 2 * k] = cp;
    sm[L::CS + 2 * k + 1] = sp;
  }
  __syncthreads();
  HMPC_STAMP(2);

  // ---------------- phase 2: wave-uniform sweeps ----------------------------
  {
    // one loop runs two independent recursions side by side (ILP):
    //   free response (lane r < 12 holds xbar[r]) xbar_{k+1} = Ad_k xbar_k + Gd,
    //     d_{k+1} = W_k (xbar_{k+1} - r_k)
    //   cost-to-go (wave-uniform) S_N = W_{N-1} = 100 Q, S_t = Q + Ad_t' S_{t+1} Ad_t
    real xr = tid < 12 ? sm[L::XIN + tid] : 0.0;
    const real qr = qdiag(tid);
    // S_t entries 0..11 (translational axes and yaw) lane-parallel: lane
    // q < 4 holds block q's [pp, pv, vv] (q = 3: yaw [tt, tw, ww]), one
    // instruction stream for the four blocks.  These blocks do not depend on
    // the instance; the roll/pitch block (entries 12..21, yaw-dependent) stays
    // wave-uniform in s[].
    const real qa = tid == 0 ? kQ[0] : tid == 1 ? kQ[1] : tid == 2 ? kQ[2] : kQ[5];
    const real qc = tid == 0 ? kQ[6] : tid == 1 ? kQ[7] : tid == 2 ? kQ[8] : kQ[11];
    real ta = kTermQ * qa, tb = 0.0, tc = kTermQ * qc;
    real s[10];   // P00 P01 P11 M00 M01 M10 M11 Q00 Q01 Q11 (entries 12..21)
    s[0] = kTermQ * kQ[3]; s[1] = 0.0; s[2] = kTermQ * kQ[4];
    s[3] = s[4] = s[5] = s[6] = 0.0;
    s[7] = kTermQ * kQ[9]; s[8] = 0.0; s[9] = kTermQ * kQ[10];
    real* const tstore = sm + L::SS + 3 * (tid < 4 ? tid : 0);
    auto store_s = [&](int t) __attribute__((always_inline)) {
      if (tid < 4) {
        tstore[22 * t] = ta;
        tstore[22 * t + 1] = tb;
        tstore[22 * t + 2] = tc;
      }
      if (tid == 0)
#pragma unroll
        for (int e = 0; e < 10; ++e) sm[L::SS + 22 * t + 12 + e] = s[e];
    };
    if (tid == 2) sm[L::ZB] = xr;
    store_s(N - 1);
    // stage k's yaw cos/sin from lane k (readlane: no LDS round trip in the
    // recursions' chains).  Both loops are unrolled: the reference rows are
    // loaded up front and the gradient terms d_t stay in registers (lane
    // r < 12: component r), so no load sits inside a recursion.
    const real cpl = tid < N ? sm[L::CS + 2 * tid] : 0.0;
    const real spl = tid < N ? sm[L::CS + 2 * tid + 1] : 0.0;
    real xrf[N], dgv[N];
    sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      xrf[k] = sm[L::XREF + 12 * k + (tid < 12 ? tid : 0)];
    });
    sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      const real cp = rdlane(cpl, k), sp = rdlane(spl, k);
      xr = ad_lane(xr, dt, cp, sp) + ((tid == 8) ? -real(a.g) * dt : real(0));
      const real kf = (k == N - 1) ? kTermQ : 1.0;
      dgv[k] = kf * qr * (xr - xrf[k]);   // 0 on lanes >= 12 (qr = 0)
      if (tid == 2) sm[L::ZB + k + 1] = xr;
      constexpr int t = N - 1 - k;
      if constexpr (t >= 1) {
        const real ct = rdlane(cpl, t), st = rdlane(spl, t);
        // translational axes and yaw: [[a, b], [b, c]] with p' = p + dt v,
        // then + W_{t-1} = Q (diagonal)
        {
          const real aa = ta, bb = tb, cc = tc;
          tb = fma(dt, aa, bb);
          tc = cc + dt * (real(2) * bb + dt * aa);
          ta = aa + qa;
          tc = tc + qc;
        }
        // roll/pitch block, theta' = theta + D w with D = dt [[c, s], [-s, c]]:
        //   M' = M + P D,   Qm' = Qm + D'(M + P D) + M' D   (old M in the last term)
        const real D00 = ct * dt, D01 = st * dt, D10 = -st * dt, D11 = ct * dt;
        const real P00 = s[0], P01 = s[1], P11 = s[2];
        const real M00 = s[3], M01 = s[4], M10 = s[5], M11 = s[6];
        const real N00 = M00 + (P00 * D00 + P01 * D10), N01 = M01 + (P00 * D01 + P01 * D11);
        const real N10 = M10 + (P01 * D00 + P11 * D10), N11 = M11 + (P01 * D01 + P11 * D11);
        const real A00 = D00 * N00 + D10 * N10, A01 = D00 * N01 + D10 * N11;
        const real A11 = D01 * N01 + D11 * N11;
        const real B00 = M00 * D00 + M10 * D10, B01 = M00 * D01 + M10 * D11;
        const real B11 = M01 * D01 + M11 * D11;
        s[7] += A00 + B00;
        s[8] += A01 + B01;
        s[9] += A11 + B11;
        s[3] = N00; s[4] = N01; s[5] = N10; s[6] = N11;
        s[0] += kQ[3]; s[2] += kQ[4];
        s[7] += kQ[9]; s[9] += kQ[10];
        store_s(t - 1);
      }
    });
    B::sync();
    // adjoint a_N = d_N, a_t = d_t + Ad_t' a_{t+1} (lane-parallel): the
    // gradient of the tracking cost w.r.t. x_t.  Only rows 6..11 are kept
    // (the nonzero rows of Bd).
    real ar = dgv[N - 1];
    if (tid >= 6 && tid < 12) sm[L::AJ + 6 * (N - 1) + tid - 6] = ar;
    sfor<1, N>([&](auto ic) __attribute__((always_inline)) {
      constexpr int t = N - decltype(ic)::value;   // N-1 .. 1
      ar = adt_lane(ar, dt, rdlane(cpl, t), rdlane(spl, t)) + dgv[t - 1];
      if (tid >= 6 && tid < 12) sm[L::AJ + 6 * (t - 1) + tid - 6] = ar;
    });
  }
  __syncthreads();
  HMPC_STAMP(3);

  // ---------------- phase 3: Hessian row (lower part) + gradient ------------
  // Variable map.  One wave (W == 1): the FREE variables only, compacted in
  // stage order -- stage j holds its stance forces (3f fx fy fz, 2f fx fz;
  // none when it swings) and then its three torques -- nf <= NV of them.
  // Lane v owns compacted variable v = (stage vj, component vc); lanes >= nf
  // are padding (identity rows, no constraints).  The fixed variables (swing
  // forces :134-136, 2f fy 2f :129) are not in the factor at all, so swing
  // windows factor, sweep and search a smaller problem.  Two waves: lane v
  // owns variable 6 vj + vc and fixed variables are identity rows in place.
  constexpr int KF = VAR == 3 ? 3 : 2;   // free forces of a stance stage
  const real ubar_z_alias = (sm[L::CC + N - 1] != 0.0) ? 2.0 * a.m * a.g : 0.0;
  auto is_fixed = [&](int k, int c) -> bool {   // swing f = 0 (:134-136), 2f fy = 0 (2f :129)
    return (c < 3 && sm[L::CC + k] == 0.0) || (VAR == 2 && c == 1);
  };
  // stance stages as a wave-uniform bit mask (one wave)
  const uint64_t smask = __ballot(tid < N && sm[L::CC + (tid < N ? tid : 0)] != 0.0);
  // first compacted variable of stage j (uniform)
  auto stage_off = [&](int j) -> int {
    return 3 * j + KF * __builtin_popcountll(smask & ((1ull << j) - 1));
  };
  const int nf = W == 1 ? uni(3 * N + KF * __builtin_popcountll(smask)) : NV;
  // stage / component of lane t's compacted variable (W == 1)
  auto vmap = [&](int t, int& vj, int& vc) __attribute__((always_inline)) {
    vj = 0;
    vc = 3;
    sfor<0, N>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const bool st = (smask >> j) & 1;
      const int r = t - stage_off(j);
      const int cs = st ? (VAR == 3 ? r : (r == 0 ? 0 : r + 1)) : r + 3;
      const bool in = r >= 0 && r < (st ? 3 + KF : 3);
      vj = in ? j : vj;
      vc = in ? cs : vc;
    });
  };
  int vj3, vc3;
  bool active_lane, my_fixed;   // owns a variable of the factor; an identity row
  if constexpr (W == 1) {
    vmap(tid, vj3, vc3);
    active_lane = tid < nf;
    my_fixed = !active_lane;
  } else {
    vj3 = tid / 6;
    vc3 = tid - 6 * (tid / 6);
    active_lane = tid < NV;
    my_fixed = active_lane && is_fixed(vj3, vc3);
  }

  real Rg[NV];   // row `tid` of H (lower part), then the Cholesky trailing row
  real hv = 0.0;
  {
    const int ii = active_lane ? vj3 : 0;
    const int ci = active_lane ? vc3 : 0;
    // my impulse b = Bd_i e_c (rows 6..11) and f = S_{i+1} b; zero for fixed
    // variables and idle lanes, whose rows of H are then zero (their unit
    // diagonal is added at the pivot, as is every 2 V_i: phase 4)
    const real rowm = (active_lane && !my_fixed) ? 1.0 : 0.0;
    const real cpi = sm[L::CS + 2 * ii], spi = sm[L::CS + 2 * ii + 1];
    const real* bwi = sm + L::BW + 18 * ii;
    real e0[12], f[12];
#pragma unroll
    for (int r = 0; r < 6; ++r) e0[r] = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) e0[6 + r] = ci < 3 ? rowm * bv<VAR>(r, ci, dtm, cpi, spi) : 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) e0[9 + r] = rowm * bwi[6 * r + ci];
    s_times<true>(sm + L::SS + 22 * ii, e0, f);
    // gradient: h_v = 2 b' a_{i+1} (b = Bd_i e_c, a = adjoint of phase 2)
    real hacc = 0.0;
#pragma unroll
    for (int r = 0; r < 6; ++r) hacc = fma(e0[6 + r], sm[L::AJ + 6 * ii + r], hacc);
    // H[v, (j, c2)] = 2 Bd_j[:,c2]' g_j with g_i = f, g_j = Ad_{j+1}' g_{j+1}
    // (j < i).  Only the lower triangle is ever read (the Cholesky publishes
    // column k from lanes >= k and overwrites register k), so entries right
    // of the diagonal keep whatever finite value falls out; the diagonal
    // block needs no special case (its 2 V_i goes in at the pivot).
    real g[12];
#pragma unroll
    for (int r = 0; r < 12; ++r) g[r] = f[r];
    auto advance = [&](auto jc, const real* smj) __attribute__((always_inline)) {   // g -> g_j
      constexpr int j = decltype(jc)::value;
      if constexpr (j < N - 1) {
        const real cp1 = smj[L::CS + 2 * (j + 1)], sp1 = smj[L::CS + 2 * (j + 1) + 1];
        real gn[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) gn[r] = g[r];
        adt_times(gn, dt, cp1, sp1);
#pragma unroll
        for (int r = 0; r < 12; ++r) g[r] = (ii > j) ? gn[r] : g[r];
      }
    };
    if constexpr (W == 1) {
      // The compacted column index of (j, c2) is wave-uniform but not known
      // at compile time, and registers cannot be indexed at run time: each
      // lane writes its row into a packed lower-triangular image of H in LDS
      // (row v at v(v+1)/2, over the dead union A: S and the adjoint are in
      // registers by now), then reads it back by compile-time column.
      // Entries right of the diagonal are not written (a per-lane scratch
      // slot in the column buffers takes them); padding lanes read a zero
      // row (XS, zeroed here).
      real* hp = sm + L::LC;
      const unsigned rowa = lds_addr(hp + ((tid * (tid + 1)) >> 1));
      const unsigned dumpa = lds_addr(sm + L::COLB + tid);
      xs[tid] = 0.0;
      B::sync();   // every lane's S / adjoint reads are issued before the first H store
      real cp_up = 0.0, sp_up = 0.0;   // cos / sin of the stage above (advance)
      sfor<0, N>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = N - 1 - decltype(jc)::value;
        // stage j's rows 9..11 of Bd and cos / sin in one LDS round trip (ten
        // broadcast loads, one wait): the compiler otherwise sinks each load
        // next to its product and waits for it there, three round trips per
        // entry of H in series
        real2 bwp[9], csp;
        {
          const unsigned sb = lds_addr(sm + opaque_zero());
          sfor<0, 9>([&](auto ic) __attribute__((always_inline)) {
            constexpr int i = decltype(ic)::value;
            lds_ld2<RB * (L::BW + 18 * j + 2 * i)>(bwp[i], sb);
          });
          lds_ld2<RB * (L::CS + 2 * j)>(csp, sb);
          lds_wait<0>(bwp[0], bwp[1], bwp[2], bwp[3]);
          lds_wait<0>(bwp[4], bwp[5], bwp[6], bwp[7]);
          lds_wait<0>(bwp[8], csp);
        }
        real bw[18];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
          bw[2 * i] = bwp[i].x;
          bw[2 * i + 1] = bwp[i].y;
        }
        if constexpr (j < N - 1) {   // g -> g_j = Ad_{j+1}' g_{j+1} (as advance())
          real gn[12];
#pragma unroll
          for (int r = 0; r < 12; ++r) gn[r] = g[r];
          adt_times(gn, dt, cp_up, sp_up);
#pragma unroll
          for (int r = 0; r < 12; ++r) g[r] = (ii > j) ? gn[r] : g[r];
        }
        const real cp = csp.x, sp = csp.y;
        cp_up = cp;
        sp_up = sp;
        const bool st = (smask >> j) & 1;   // uniform
        const int o = stage_off(j);
        auto put = [&](int w, real val) __attribute__((always_inline)) {
          const unsigned ad = (w <= tid && active_lane) ? rowa + (unsigned)RB * (unsigned)w : dumpa;
          *(lds_real*)ad = val;
        };
        if (st) {   // the stance forces (2f: fx, fz)
          sfor<0, 3>([&](auto c2c) __attribute__((always_inline)) {
            constexpr int c2 = decltype(c2c)::value;
            if constexpr (!(VAR == 2 && c2 == 1))
              put(o + (VAR == 3 ? c2 : (c2 == 0 ? 0 : 1)), bd_dot<VAR>(c2, g, bw, dtm, cp, sp));
          });
        }
        const int ot = o + (st ? KF : 0);   // the torques
        sfor<3, 6>([&](auto c2c) __attribute__((always_inline)) {
          constexpr int c2 = decltype(c2c)::value;
          put(ot + c2 - 3, bd_dot<VAR>(c2, g, bw, dtm, cp, sp));
        });
      });
      B::sync();
      const real* row = active_lane ? hp + ((tid * (tid + 1)) >> 1) : xs;
      sfor<0, NV>([&](auto wc) __attribute__((always_inline)) {
        constexpr int w = decltype(wc)::value;
        Rg[w] = row[w];
      });
    } else {
      sfor<0, N>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = N - 1 - decltype(jc)::value;
        const real* smj = sm + opaque_zero();   // keeps this step's loads here
        advance(std::integral_constant<int, j>{}, smj);
        const real cp = smj[L::CS + 2 * j], sp = smj[L::CS + 2 * j + 1];
        const real* bw = smj + L::BW + 18 * j;
        // fixed columns (swing forces :134-136) of stage j: zero
        const real stance_j = smj[L::CC + j] != 0.0 ? 1.0 : 0.0;
        sfor<0, 6>([&](auto c2c) __attribute__((always_inline)) {
          constexpr int c2 = decltype(c2c)::value;
          constexpr int w = 6 * j + c2;
          real val;
          if constexpr (VAR == 2 && c2 == 1) val = 0.0;   // 2f fy (2f :129)
          else if constexpr (c2 < 3) val = stance_j * bd_dot<VAR>(c2, g, bw, dtm, cp, sp);
          else val = bd_dot<VAR>(c2, g, bw, dtm, cp, sp);
          Rg[w] = val;
          pin(Rg[w]);
        });
      });
    }
    if (active_lane && !my_fixed) {
      real ub = 0.0;
      if (vc3 == 2) ub = a.uref_aliased ? ubar_z_alias : ((sm[L::CC + vj3] != 0.0) ? 2.0 * a.m * a.g : 0.0);
      const real Vj = (vj3 == N - 1) ? 0.0 : kRdiag;
      hv = real(2) * hacc - real(2) * Vj * ub;
    }
  }
  real wv = -hv;   // the forward sweep's accumulator (phase 4)
  __syncthreads();   // union A (XLIN/XREF/PF/S/DG) is dead from here on
  HMPC_STAMP(4);
  __builtin_amdgcn_s_setprio(kCmpCls ? kPrioCmp : 3);

  int status = ST_SOLVED;
  real dinv = 0.0;
  // the diagonal of H not built in phase 3: 1 for a fixed variable (identity
  // row/column), else 2 V_i (R * kuf: every stage but the last, 3f :114,132,139)
  auto diag_extra = [&](int stage, bool fixed) -> real {
    return fixed ? 1.0 : ((stage != N - 1) ? 2.0 * kRdiag : 0.0);
  };

  // ---------------- phase 4: Cholesky ---------------------------------------
  // Right-looking, lane v holds row v of the trailing matrix in registers
  // (register j = column j).  Step k publishes column k (lanes >= k) through
  // LDS; every lane then updates its registers j > k.  Step k's multipliers
  // M[i][k] = L[i][k] / L[k][k] go column-major to LDS (1/L_kk on the
  // diagonal) for the sweeps; phase 5's forward substitution runs inside
  // the steps.  Column loads are issued before the pivot
  // arithmetic (hand-counted waits).  Only the lower triangle of the
  // registers is meaningful; the diagonal's 2 V_i (or a fixed variable's 1)
  // is added to the pivot (diag_extra).
  //   NV <= 64 (one wave): every step unrolled -- no runtime index, no selects.
  //   NV >  64: blocks of 8 steps share one runtime loop body (code size).
  {
    if (tid == 0) sm[L::ZR] = 0.0;
    // non-positive pivots, counted: `if (piv <= 0) status = ...` per step
    // kept 60 condition masks alive in SGPRs (and spilled)
    real nbad = 0.0;
    uint64_t okall = ~0ull;   // the one-wave path's pivot signs (an SGPR mask)
    auto nld_of = [](int lo, int ch) constexpr {   // b128 loads of chunk ch of [lo, NV)
      return (NV - lo - 8 * ch) >= 8 ? 4 : (NV - lo - 8 * ch + 1) / 2;
    };
    if constexpr (W == 1) {
      // Lookahead: step k publishes column k+1 and issues its first load
      // chunk right after its own first chunk (which holds column k+1), and
      // does step k+1's pivot arithmetic there, so the LDS round trip and the
      // pivot chain of step k+1 overlap step k's remaining updates.
      // Fixed variables (swing forces, 2f fy) are identity rows/columns of H:
      // their steps update nothing and are skipped (uniform branch on a
      // ballot of the fixed lanes; 2f fy at compile time).
      constexpr int CW = 4;   // columns per load chunk
      auto nldc = [](int ja, int ch) constexpr {   // b128 loads of chunk ch of [ja, NV)
        return (NV - ja - CW * ch) >= CW ? CW / 2
                                         : ((NV - ja - CW * ch) > 0 ? (NV - ja - CW * ch + 1) / 2 : 0);
      };
      const real dx = diag_extra(vj3, my_fixed);   // lane s: the extra of pivot s
      real2 nb[CW / 2];                 // chunk 0 of the next step
      real p_rs = 0.0, p_tk = 0.0;   // next step's 1/L_kk and M[tid][k]
      // the two column buffers' LDS addresses, held in registers (opaque):
      // otherwise every step rematerialises them with v_movs
      unsigned colb[2] = {lds_addr(sm + L::COLB), lds_addr(sm + L::COLB + NT + 8)};
      asm volatile("" : "+v"(colb[0]), "+v"(colb[1]));
      auto ahead = [&](auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        constexpr int JS = (s + 1) & ~1;
        // lane masks of a step come from an opaque copy of its index: hoisted
        // out of the unrolled steps they would pin ~100 SGPRs (and spill)
        real* col = sm + L::COLB + (s & 1) * (NT + 8);
        const real mine = Rg[s];
        // unmasked: the updates read rows > s only (lanes < s hold
        // don't-care upper-triangle values there, lanes >= NV are never read)
        col[tid] = mine;
        B::sync();
        const unsigned cb0 = colb[s & 1];
        sfor<0, nldc(JS, 0)>([&](auto ic) __attribute__((always_inline)) {
          constexpr int i = decltype(ic)::value;
          lds_ld2<RB * (JS + 2 * i)>(nb[i], cb0);
        });
        const real piv = rdlane(mine + dx, s);
        const uint64_t pos = __ballot(piv > real(0));   // all lanes or none
        const real pv = pos ? piv : real(1);
        okall &= pos;                       // folded into status after the loop
        asm volatile("" : "+s"(okall));     // (materialised here, not sunk to the end)
        p_rs = rsq_nr(pv);
        p_tk = (mine * p_rs) * p_rs;
      };
      ahead(std::integral_constant<int, 0>{});
      constexpr uint64_t kLive = NV >= 64 ? ~0ull : ((1ull << NV) - 1);
      const unsigned tb = lds_addr(sm + tid);
      // steps 0 .. nf-1 only: the compacted factor has no fixed variables,
      // and the padding rows beyond nf are the identity (never stepped)
      ladder<0, NV>(nf, [&](auto kc) __attribute__((always_inline)) {
        constexpr int k = decltype(kc)::value;
        constexpr int JA = (k + 1) & ~1;   // 16-B aligned start of the update
        constexpr int NCH = (NV - JA + CW - 1) / CW;
        constexpr int NAHEAD = (k + 1 < NV) ? 1 + nldc((k + 2) & ~1, 0) : 0;   // LDS ops of ahead()
        const real rs = p_rs, tk = p_tk;
        if constexpr (k == 0) lds_wait<0>(nb[0], nb[1]);   // chunk 0 (later steps: waited at the previous one's end)
        // every lane updates: a lane <= k changes only its registers > k, the
        // upper triangle of its row (don't-care, overwritten at their step)
        const real nt = -tk;
        // lane masks of this step, compile-time constants (msel)
        constexpr uint64_t m_eq = 1ull << k;
        constexpr uint64_t m_ge = kLive & ~(m_eq - 1);
        constexpr uint64_t m_gt = m_ge & ~m_eq;
        // branch-free store of column k of M (other lanes: the column buffer
        // of step k+1, which ahead() rewrites after this store)
        {
          constexpr int DOFF = RB * (L::COLB + ((k + 1) & 1) * (NT + 8));
          constexpr int LOFF = RB * (L::LC + L::cb(k) - k);
          const unsigned ad = msel(m_ge, tb + (unsigned)(LOFF - DOFF), tb);
          *(lds_real*)(ad + DOFF) = msel(m_eq, rs, tk);
        }
        // phase 5's forward substitution w = M^-1 (-h) rides along: w_k is
        // final here, rows below take -M[i][k] w_k (off the step's chain)
        wv = fma(msel(m_gt, tk, real(0)), -rdlane(wv, k), wv);
        const unsigned cbase = colb[k & 1];
        // chunks >= 1 go through a 3-deep ring: chunk ch+2 is issued while
        // chunk ch is consumed (one chunk ahead left the LDS latency exposed)
        real2 buf[3][CW / 2];
        auto load = [&](auto chc) __attribute__((always_inline)) {
          constexpr int ch = decltype(chc)::value;
          if constexpr (ch >= 1 && ch < NCH) {
            sfor<0, nldc(JA, ch)>([&](auto ic) __attribute__((always_inline)) {
              constexpr int i = decltype(ic)::value;
              lds_ld2<RB * (JA + CW * ch + 2 * i)>(buf[ch % 3][i], cbase);
            });
          }
        };
        auto nl = [](int ja, int ch) constexpr {   // loads of chunk ch (0 beyond the row)
          return (ch >= 1 && ch < (NV - ja + CW - 1) / CW) ? ((NV - ja - CW * ch) >= CW ? CW / 2
                                                                 : (NV - ja - CW * ch + 1) / 2)
                                                           : 0;
        };
        auto update = [&](auto chc, const real2 (&bf)[CW / 2]) __attribute__((always_inline)) {
          constexpr int ch = decltype(chc)::value;
          sfor<0, CW>([&](auto ic) __attribute__((always_inline)) {
            constexpr int i = decltype(ic)::value;
            constexpr int j = JA + CW * ch + i;
            if constexpr (j > k && j < NV) {
              const real cv = (i & 1) ? bf[i / 2].y : bf[i / 2].x;
              Rg[j] = fma(nt, cv, Rg[j]);
              pin(Rg[j]);
            }
          });
        };
        load(std::integral_constant<int, 1>{});
        load(std::integral_constant<int, 2>{});
        if constexpr (NCH > 0) update(std::integral_constant<int, 0>{}, nb);
        if constexpr (k + 1 < NV) ahead(std::integral_constant<int, k + 1>{});
        sfor<1, NCH>([&](auto chc) __attribute__((always_inline)) {
          constexpr int ch = decltype(chc)::value;
          load(std::integral_constant<int, ch + 2>{});
          // LDS ops issued after chunk ch's loads (issue order: chunks 1,
          // 2, ahead(), then chunk c+2 at iteration c)
          constexpr int younger = ch == 1 ? nl(JA, 2) + NAHEAD + nl(JA, 3)
                                : ch == 2 ? NAHEAD + nl(JA, 3) + nl(JA, 4)
                                          : nl(JA, ch + 1) + nl(JA, ch + 2);
          lds_wait<younger>(buf[ch % 3][0], buf[ch % 3][1]);
          update(chc, buf[ch % 3]);
        });
        // the next step's chunk 0 (the lookahead) is waited for here, at the
        // end of this step rather than at the start of the next: the same
        // wait point, but before the ladder's exit test, so no LDS load is in
        // flight where an early exit (nf < NV) merges with the others (the
        // compiler may copy or reassign nb's registers at a merge; a variant
        // that let it do so returned wrong optima)
        if constexpr (k + 1 < NV) lds_wait<0>(nb[0], nb[1]);
      });
      // sweep_pad_zero: columns nf .. nf+kRing1-2 of M were never stepped
      // (stale LDS); zero them so the forward sweeps run whole ring groups
      // past nf without a per-step bound (tri_fwd_lds)
#pragma unroll
      for (int c0 = 0; c0 < kRing1 - 1; ++c0) {
        const int c = nf + c0;
        if (c < NV && tid > c && tid < NV) sm[L::LC + L::cb(c) + tid - c] = real(0);
      }
    } else {
      real mine = Rg[0];   // A[tid][k] of the current step
      // pivot extras (diag_extra) by lane, behind the column buffers (the
      // active-set state there is not live yet); the first step's barrier
      // publishes them
      real* dxa = sm + L::COLB + 2 * (NT + 8);
      static_assert(L::COLB + 2 * (NT + 8) + NT <= L::U0, "pivot extras do not fit");
      dxa[tid] = diag_extra(vj3, my_fixed);
      sfor<0, (NV + 7) / 8>([&](auto bc) __attribute__((always_inline)) {
        constexpr int bb = decltype(bc)::value;
        constexpr int J0 = 8 * bb;
        constexpr int KEND = (J0 + 8 < NV) ? J0 + 8 : NV;
        constexpr int NCH = (NV - J0 + 7) / 8;
#pragma unroll 1
        for (int k = J0; k < KEND; ++k) {
          real* col = sm + L::COLB + (k & 1) * (NT + 8);
          col[tid] = (tid >= k && tid < NV) ? mine : 0.0;
          if (tid == k) col[NT] = wv;   // w_k (final) for the riding forward sweep
          B::sync();
          const real piv = col[k] + dxa[k];
          const real wk = col[NT];
          const unsigned cbase = lds_addr(col + J0);
          real2 buf[2][4];
          auto load = [&](auto chc) __attribute__((always_inline)) {
            constexpr int ch = decltype(chc)::value;
            if constexpr (ch < NCH) {
              sfor<0, nld_of(J0, ch)>([&](auto ic) __attribute__((always_inline)) {
                constexpr int i = decltype(ic)::value;
                lds_ld2<RB * (8 * ch + 2 * i)>(buf[ch % 2][i], cbase);
              });
            }
          };
          load(std::integral_constant<int, 0>{});
          const real pv = piv > 0.0 ? piv : 1.0;
          nbad += (piv > real(0)) ? real(0) : real(1);   // folded into status after the loop
        pin(nbad);                          // (materialised here, not sunk to the end)
          const real rs = rsq_nr(pv);
          const real tk = (mine * rs) * rs;
          const bool below = tid > k && tid < NV;
          const real mk = below ? tk : 0.0;
          wv = fma(-mk, wk, wv);   // phase 5's forward substitution (as one wave)
          // unmasked: the published column is 0 above row k, so a lane <= k
          // changes only its upper triangle (registers > k, never read)
          const real nt = -tk;
          real nxt = 0.0;
          sfor<0, NCH>([&](auto chc) __attribute__((always_inline)) {
            constexpr int ch = decltype(chc)::value;
            load(std::integral_constant<int, ch + 1>{});
            constexpr int younger = ch + 1 < NCH ? nld_of(J0, ch + 1) : 0;
            lds_wait<younger>(buf[ch % 2][0], buf[ch % 2][1], buf[ch % 2][2], buf[ch % 2][3]);
            sfor<0, 8>([&](auto ic) __attribute__((always_inline)) {
              constexpr int i = decltype(ic)::value;
              constexpr int j = J0 + 8 * ch + i;
              if constexpr (j < NV) {
                const real cv = (i & 1) ? buf[ch % 2][i / 2].y : buf[ch % 2][i / 2].x;
                real r = fma(nt, cv, Rg[j]);
                if constexpr (j < KEND) r = (j == k) ? mk : r;
                Rg[j] = r;
                pin(Rg[j]);
                if constexpr (j > J0 && j <= J0 + 8) nxt = (j == k + 1) ? Rg[j] : nxt;
              }
            });
          });
          if (tid >= k && tid < NV) sm[L::LC + L::cb(k) + tid - k] = (tid == k) ? rs : tk;
          mine = nxt;
          // (no barrier here: a wave rewrites this buffer at step k+2 only
          // after the barrier of step k+1, which every wave reaches after
          // its step-k reads)
        }
      });
    }
    __syncthreads();
    if (nbad != 0.0 || okall == 0) status = ST_NUMERICAL;
    dinv = tid < NV ? sm[L::LC + L::cb(tid < NV ? tid : 0)] : 0.0;   // 1 / L[tid][tid]
    if constexpr (W == 1) dinv = active_lane ? dinv : real(1);   // padding: never stepped
  }
  HMPC_STAMP(5);

  const real* Lc = sm + L::LC;
  const real* zero = sm + L::ZR;

  // ---------------- phase 5: v0 = -L^-T L^-1 h -------------------------------
  real v = 0.0;
  {
    real y;
    y = wv * dinv;   // L^-1 (-h), swept during the Cholesky
    v = tri_bwd<L>(y, Lc, zero, dinv, xs, nf);
  }
  HMPC_STAMP(6);

  // per-instance scalars needed after the factorisation are re-derived here
  // rather than kept live across it (they were spilled there)
  const real mu = sm[L::ZR + 1];   // staged in phase 0
  const real dtm2 = dt / real(a.m) + real(0) * (real)opaque_zero();
  // stage / component of my variable, recomputed from an opaque thread id:
  // phase 3's copies would stay alive (spilled) across the factorisation
  const int tid_o = tid + opaque_zero();
  int vj, vc;
  if constexpr (W == 1) {
    vmap(tid_o, vj, vc);
    active_lane = tid_o < nf;
  } else {
    vj = (tid_o * 43) >> 8;   // tid / 6 for tid < 128
    vc = tid_o - 6 * vj;
  }
  // the full-order slot of my variable in XS (padding lanes: a spare slot)
  const int fidx = W == 1 ? (active_lane ? 6 * vj + vc : NT - 1) : tid_o;

  // ---------------- phase 6: Goldfarb-Idnani, range-space form --------------
  // Constraints owned by lane v (id = 4 v + slot), all as n'v >= b:
  //   c in 3..5 : slot0  v >= -lim,  slot1 -v >= -lim          (:123-128)
  //   c == 3    : slot2  z_k >= 0.1, k = stage, 2 <= k <= N-1  (:129)
  //   c == 2    : slot0  fz >= 0,    slot1 -fz >= -206          (:145-146)
  //   c in 0..1 : slot0 -f + mu fz >= 0, slot1 f + mu fz >= 0   (:141-144)
  //   (stance only for c <= 2; 2f has no fy rows)
  int iters = 0;
  const real zmin_gap_k0 = sm[L::XIN + 2] - real(kZmin);    // z_0 row: constant
  const real zmin_gap_k1 = sm[L::ZB + 1] - kZmin;     // z_1 row: constant
  if (zmin_gap_k0 < -kTolR || zmin_gap_k1 < -kTolR) status = ST_INFEAS;
  // coefficient of fz_j in z_k (j <= k-2): dt * (dt/m) * (k-1-j), stance only
  // (Bd[8][2] = dt/m in both variants)
  const real zc = dt * dtm2;

  const bool stance_me = active_lane && vc <= 2 && sm[L::CC + vj] != 0.0;
  int nslots = 0;
  if (active_lane) {
    if (vc >= 3) nslots = (vc == 3 && vj >= 2) ? 3 : 2;
    else if (stance_me && !(VAR == 2 && vc == 1)) nslots = 2;
  }
  // |n| of my z row (stance stages j <= k-2): a uniform, unrolled masked sum
  // (a per-lane loop would diverge and wait on one LDS load per trip)
  real s2 = 0.0;
  sfor<0, (N > 2 ? N - 2 : 0)>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const real cz = zc * (real)(vj - 1 - j);
    const real m = (j <= vj - 2 && sm[L::CC + j] != 0.0) ? 1.0 : 0.0;
    s2 = fma(m * cz, cz, s2);
  });
  const real znorm = (active_lane && vc == 3 && vj >= 2) ? sqrt(s2) : 0.0;
  // slot 0/1 coefficients of my constraints (see the table above)
  real a0 = 1.0, muf = 0.0, k0 = 0.0, k1 = 0.0, inv01 = 1.0;
  if (vc >= 3) {
    k0 = k1 = tau_lim(vc);
  } else if (vc == 2) {
    k1 = kFzMax;
  } else {
    a0 = -1.0;
    muf = mu;
    inv01 = real(1) / sqrt(real(1) + mu * mu);
  }
  int actmask = 0;

  real* Rm = sm + L::RM;   // packed upper, column k at loff(k)
  real* ua = sm + L::UA;
  int* act = reinterpret_cast<int*>(sm + L::ACT);
  real* cbv = sm + L::CB;
  real* gv = sm + L::GV;
  real* sdg = sm + L::SD;
  real Qw[QMAX];   // row `tid` of the orthonormal basis of L^-1 N_A
#pragma unroll
  for (int l = 0; l < QMAX; ++l) Qw[l] = 0.0;
  int q = 0;
  const int max_iter = 4 * NV + 50;

  // coefficient of lane `i`'s variable in constraint `id`, and its rhs
  // (stage, component) of the variable of lane o (uniform o)
  auto owner = [&](int o, int& oj, int& oc) __attribute__((always_inline)) {
    if constexpr (W == 1) {
      oj = __builtin_amdgcn_readlane(vj, o);
      oc = __builtin_amdgcn_readlane(vc, o);
    } else {
      oj = o / 6;
      oc = o - 6 * oj;
    }
  };
  auto coef_of = [&](int id, int i) -> real {   // (i: this lane)
    const int o = id >> 2, sl = id & 3;
    int oj, oc;
    owner(o, oj, oc);
    if (!active_lane) return 0.0;
    if (oc >= 3) {
      if (sl == 0) return i == o ? 1.0 : 0.0;
      if (sl == 1) return i == o ? -1.0 : 0.0;
      // z-row of stage oj over fz_j, j <= oj-2
      if (vc != 2 || vj > oj - 2 || sm[L::CC + vj] == 0.0) return 0.0;
      return zc * (real)(oj - 1 - vj);
    }
    if (oc == 2) return i == o ? (sl == 0 ? 1.0 : -1.0) : 0.0;
    if (i == o) return sl == 0 ? -1.0 : 1.0;
    if (vj == oj && vc == 2) return mu;
    return 0.0;
  };
  auto rhs_of = [&](int id) -> real {
    const int o = id >> 2, sl = id & 3;
    int oj, oc;
    owner(o, oj, oc);
    if (oc >= 3) {
      if (sl < 2) return -tau_lim(oc);
      return real(kZmin) - sm[L::ZB + oj];
    }
    if (oc == 2) return sl == 0 ? 0.0 : -kFzMax;
    return 0.0;
  };

  bool done = status != ST_SOLVED;
  while (!done) {
    // ---- slacks of my constraints; pick the most violated ----
    HMPC_TIC(t_scan);
    xs[fidx] = v;   // full order (fixed variables: 0)
    B::sync();
    // branch-free: slots 0/1 are +-a0 v + muf fz_stage + k0/k1; slot 2 the
    // z row ZB_k + zc ((k-1) S1 - S2) with S1 = sum C_j fz_j, S2 = sum j C_j fz_j
    // over j <= k-2 (prefix sums over a uniform trip count)
    real z1 = 0.0, z2 = 0.0;
    sfor<0, (N > 2 ? N - 2 : 0)>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const real val = sm[L::CC + j] * xs[6 * j + 2];
      const real msk = (j <= vj - 2) ? 1.0 : 0.0;
      z1 = fma(msk, val, z1);
      z2 = fma(msk * (real)j, val, z2);
    });
    const real fzs = xs[6 * (active_lane ? vj : 0) + 2];
    const real sc0 = fma(a0, v, fma(muf, fzs, k0)) * inv01;
    const real sc1 = fma(-a0, v, fma(muf, fzs, k1)) * inv01;
    const real zrow = (sm[L::ZB + (active_lane ? vj : 0)] - real(kZmin)) + zc * fma((real)(vj - 1), z1, -z2);
    const real sc2 = znorm > 0.0 ? zrow / znorm : ((zrow < -kTolR) ? -INFINITY : INFINITY);
    real best = INFINITY;
    int bid = 0x7fffffff;
    {   // (selects: a slot that is not a candidate offers (inf, none))
      const bool c0 = nslots > 0 && !(actmask & 1), c1 = nslots > 1 && !(actmask & 2);
      const bool c2 = nslots > 2 && !(actmask & 4);
      argmin_combine_sel(best, bid, c0 ? sc0 : real(INFINITY), c0 ? 4 * tid : 0x7fffffff);
      argmin_combine_sel(best, bid, c1 ? sc1 : real(INFINITY), c1 ? 4 * tid + 1 : 0x7fffffff);
      argmin_combine_sel(best, bid, c2 ? sc2 : real(INFINITY), c2 ? 4 * tid + 2 : 0x7fffffff);
    }
    B::argmin(best, bid, red);
    HMPC_TOC(9, t_scan);
    if (!(best < -kTolR)) break;   // primal feasible: optimal
    const int p = uni(bid);
    const real bp = rhs_of(p);
    const real np_me = coef_of(p, tid);
    real u_plus = 0.0;
    // w = L^-1 n_p
    HMPC_TIC(t_fwd);
    const int s0 = B::first(np_me != 0.0, red);   // first nonzero of n_p (-1: none)
    const real wfull = tri_fwd_lds<L>(np_me, Lc, zero, dinv, xs, nf, s0 > 0 ? (s0 & ~(W == 1 ? 3 : kRing2 - 1)) : 0);
    const real wnorm2 = B::sum(wfull * wfull, red);
    HMPC_TOC(10, t_fwd);

    // ---- inner loop: step towards satisfying constraint p ----
    while (true) {
      if (++iters > max_iter) { status = ST_MAXIT; done = true; break; }
      const int qu = uni(q);
      // w_perp = (I - Qw Qw') w and c = Qw' w by modified Gram-Schmidt; a
      // second pass when the first one cancels more than half the norm
      HMPC_TIC(t_gs);
      real wp = wfull, zn = wnorm2;
#pragma unroll 1
      for (int pass = 0; pass < 2 && qu > 0; ++pass) {
        if constexpr (W == 1) {   // modified Gram-Schmidt: no barriers in one wave
          // (a classical form in blocks of four independent sums measured
          // -0.3 % at configs[2], no gain at configs[1]: DESIGN.md 7)
          ladder<0, QMAX>(qu, [&](auto lc) __attribute__((always_inline)) {
            constexpr int l = decltype(lc)::value;
            const real cl = B::sum(Qw[l] * wp, red);
            wp = fma(-cl, Qw[l], wp);
            if (tid == 0) cbv[l] = (pass == 0) ? cl : cbv[l] + cl;
          });
        } else {   // classical Gram-Schmidt: all q projections behind one exchange
          real* part = sm + L::GS;
          ladder<0, QMAX>(qu, [&](auto lc) __attribute__((always_inline)) {
            constexpr int l = decltype(lc)::value;
            const real pl = wave_sum(Qw[l] * wp);
            if ((tid & 63) == 0) part[(tid >> 6) * QMAX + l] = pl;
          });
          __syncthreads();
          ladder<0, QMAX>(qu, [&](auto lc) __attribute__((always_inline)) {
            constexpr int l = decltype(lc)::value;
            const real cl = part[l] + part[QMAX + l];
            wp = fma(-cl, Qw[l], wp);
            if (tid == 0) cbv[l] = (pass == 0) ? cl : cbv[l] + cl;
          });
        }
        const real n2 = B::sum(wp * wp, red);
        const bool enough = n2 > real(0.25) * zn;
        zn = n2;
        if (enough) break;
      }
      B::sync();
      HMPC_TOC(11, t_gs);
      // primal direction z = L^-T w_perp (lane v gets z_v)
      HMPC_TIC(t_bwd);
      const real zi = tri_bwd<L>(wp, Lc, zero, dinv, xs, nf);
      HMPC_TOC(12, t_bwd);
      HMPC_TIC(t_dual);
      // dual direction r = R^-1 c (lanes l < q), back substitution
      // (the diagonal's reciprocals first, one division per lane off the
      // substitution's chain, which is then readlane -> mul -> fma; the
      // updates are selects, not exec-masked branches -- round 5)
      real rcur = tid < qu ? cbv[tid] : 0.0, rmine = 0.0;
      const int td = tid < qu ? tid : 0;
      const real rinv = real(1) / Rm[loff(td) + td];
      // each step's R column is loaded one step ahead (its LDS latency off
      // the readlane -> mul -> fma chain)
      const int lt = qu > 0 ? qu - 1 : 0;
      real rv_n = Rm[loff(lt) + (tid < lt ? tid : 0)];
      for (int l = qu - 1; l >= 0; --l) {
        const real rv = rv_n;
        const int ln = l > 0 ? l - 1 : 0;
        rv_n = Rm[loff(ln) + (tid < ln ? tid : 0)];
        const real rl = B::bcast(rcur, l, red) * B::bcast(rinv, l, red);
        rmine = (tid == l) ? rl : rmine;
        rcur = (tid < l) ? fma(-rv, rl, rcur) : rcur;
      }
      // partial step length t1 (drop candidate)
      real t1 = INFINITY;
      int kdrop = 0x7fffffff;
      if (tid < qu && rmine > 0.0) { t1 = ua[tid] / rmine; kdrop = tid; }
      B::argmin(t1, kdrop, red);
      // full step length t2 (n_p' z = |w_perp|^2)
      const real sp_ = B::sum(np_me * v, red) - bp;
      const bool has_z = zn > kZnRel * wnorm2;
      const real t2 = has_z ? -sp_ / zn : INFINITY;
      const real t = t1 < t2 ? t1 : t2;
      if (!(t < INFINITY)) { status = ST_INFEAS; done = true; break; }
      if (has_z) v = fma(t, zi, v);
      if (tid < qu) ua[tid] -= t * rmine;
      u_plus += t;
      B::sync();
      HMPC_TOC(13, t_dual);
      HMPC_TIC(t_upd);
      if (has_z && t == t2) {
        // ---- add p: new basis column w_perp / |w_perp|, R column [c; rho] ----
        // active set beyond the register/LDS capacity: handed to the
        // overflow pass (hmpc_ric.hip, capacity NV) when the caller set one up
        if (qu >= QMAX) { status = a.ovf_count ? ST_OVERFLOW : ST_NUMERICAL; done = true; break; }
        const real rho = sqrt(zn);
        const real qn = wp / rho;
        // (selects over every register, not a branch per index: branches that
        // store to different elements get merged into one dynamically
        // indexed store, and the array lands in scratch)
#pragma unroll
        for (int l = 0; l < QMAX; ++l) Qw[l] = (l == qu) ? qn : Qw[l];
        if (tid < qu) Rm[loff(qu) + tid] = cbv[tid];
        if (tid == qu) Rm[loff(qu) + qu] = rho;
        if (tid == 0) { act[qu] = p; ua[qu] = u_plus; }
        if (tid == (p >> 2)) actmask |= 1 << (p & 3);
        q = qu + 1;
        B::sync();
        HMPC_TOC(14, t_upd);
        break;
      }
      // ---- drop active constraint kdrop ----
      {
        const int k = uni(kdrop);
        const int idk = act[k];
        if (tid == (idk >> 2)) actmask &= ~(1 << (idk & 3));
        // shift R columns k+1..q-1 left; remember the subdiagonals
        for (int m = k; m + 1 < qu; ++m) {
          real val = 0.0;
          if (tid <= m + 1) val = Rm[loff(m + 1) + tid];
          B::sync();
          if (tid <= m) Rm[loff(m) + tid] = val;
          if (tid == m + 1) sdg[m] = val;
          B::sync();
        }
        // shift the active list and multipliers
        {
          int an = 0;
          real un = 0.0;
          if (tid >= k && tid + 1 < qu) { an = act[tid + 1]; un = ua[tid + 1]; }
          B::sync();
          if (tid >= k && tid + 1 < qu) { act[tid] = an; ua[tid] = un; }
          B::sync();
        }
        // Givens to restore the triangle: rows (l, l+1), l = k..q-2
        for (int l = k; l + 1 < qu; ++l) {
          const real aa = Rm[loff(l) + l], bb = sdg[l];
          const real hh = sqrt(aa * aa + bb * bb);
          const real cg = aa / hh, sg = bb / hh;
          B::sync();
          if (tid == l) { Rm[loff(l) + l] = hh; gv[2 * l] = cg; gv[2 * l + 1] = sg; }
          const int mcol = tid;   // columns m > l hold rows l, l+1
          if (mcol > l && mcol + 1 < qu) {
            const real rl = Rm[loff(mcol) + l], rl1 = Rm[loff(mcol) + l + 1];
            Rm[loff(mcol) + l] = cg * rl + sg * rl1;
            Rm[loff(mcol) + l + 1] = -sg * rl + cg * rl1;
          }
          B::sync();
        }
        // the same rotations on the basis columns (Qw <- Qw G')
#pragma unroll
        for (int l = 0; l + 1 < QMAX; ++l) {
          const bool rot = l >= k && l + 1 < qu;
          const int lg = rot ? l : 0;
          const real cg = gv[2 * lg], sg = gv[2 * lg + 1];
          const real x0 = Qw[l], x1 = Qw[l + 1];
          Qw[l] = rot ? cg * x0 + sg * x1 : x0;
          Qw[l + 1] = rot ? -sg * x0 + cg * x1 : x1;
        }
#pragma unroll
        for (int l = 0; l < QMAX; ++l) Qw[l] = (l == qu - 1) ? 0.0 : Qw[l];
        q = qu - 1;
        B::sync();
        HMPC_TOC(14, t_upd);
      }
    }
  }
  // ---------------- fp32 solve + fp64 refinement (kRefine builds) -----------
  // configs[4]: the fp32 factors and active set, then a.refine
  // corrections of the KKT system of that active set with fp64 residuals --
  //   r1 = N_A lam - (H u + h)  (the gradient by an fp64 rollout + adjoint,
  //        the reference's dynamics rebuilt in fp64 from the fp64 inputs)
  //   r2 = b_A - N_A' u         (the active rows in fp64)
  // solved with L^-1 N_A = Qw R: w = L^-1 r1, c = Qw' w, t = R^-T r2,
  // dlam = R^-1 (t - c), du = L^-T (w - Qw c + Qw t).  An fp64 check of every
  // row and multiplier then confirms the active set; an instance that fails
  // it (or any non-solved fp32 instance) goes to the fp64 overflow pass.
  if constexpr (kRefine) {
    static_assert(W == 1, "the refinement runs in one-wave kernels");
    if (uni(status) != ST_SOLVED && a.ovf_count) status = ST_OVERFLOW;
    if (uni(status) == ST_SOLVED) {
      // stamps (diagnostic build): 7 = the refinement's start, 15 = cycles in
      // the corrections, 8 = the end of the fp64 check
      HMPC_STAMP(7);
      const SolveArgs& ka = opaque_args(a);   // (fresh loads of the arguments)
      double* d64 = reinterpret_cast<double*>(sm + L::R64);
      double* dlo = reinterpret_cast<double*>(sm + L::R64LO);
      int* dslot = reinterpret_cast<int*>(d64 + L::DSLOT);
      const double dt64 = ka.dt, dtm64 = ka.dt / ka.m;
      const double mu64 = ka.mu ? ka.mu[b] : ka.mu_default;
      const double zc64 = dt64 * dtm64;
      const double* xrf7 = reinterpret_cast<const double* const*>(sm + L::XRV)[0];
      const int xrs = reinterpret_cast<const int*>(sm + L::XRV + 2)[0];
      // gen_dt_dynamics in fp64 (lane k < N: stage k), on the linearisation
      // rows as phase 0 builds them from the fp64 inputs
      if (tid < N) {
        const int k = tid;
        const double* xp = ka.x_lin + b * 12 * (N + 1);
        const int mode = ka.shift_mode;
        auto xl = [&](int c) -> double {
          if (mode == 0) return xp[12 * k + c];
          if (k == 0) return ka.x_in[b * 12 + c];
          return mode == 1 ? xrf7[(k - 1) * xrs + c] : xp[12 * (k + 1 <= N ? k + 1 : N) + c];
        };
        const double p3[3] = {xl(0), xl(1), xl(2)};
        const double* pfp = ka.pf + b * ka.pf_bs + k * ka.pf_rs;
        const double pf3[3] = {pfp[0], pfp[1], pfp[2]};
        stage_dynamics_vals<VAR, double>(k, xl(5), p3, pf3, ka.Jinv, ka.rh, dt64, dlo + L::DCS, d64 + L::DBW);
      }
      // u in full order (fixed variables 0), each lane's full-order slot
      for (int i = tid; i < L::NVF; i += NT) dlo[L::DU + i] = 0.0;
      dslot[tid] = active_lane ? fidx : 0;
      for (int i = tid; i < 12 * N; i += NT) {   // x_ref rows
        const int r = i / 12;
        d64[L::DXR + i] = xrf7[r * xrs + i - 12 * r];
      }
      const double xin64 = ka.x_in[b * 12 + (tid < 12 ? tid : 0)];
      B::sync();
      double u64 = (double)v;
      if (active_lane) dlo[L::DU + fidx] = u64;
      const int qu = uni(q);
      double lam = tid < qu ? (double)ua[tid] : 0.0;
      const double qr = qdiag(tid);
      const int rw = (tid >= 9 && tid < 12) ? tid - 9 : 0;
      const int rv = (tid >= 6 && tid < 9) ? tid - 6 : 0;
      const double gdt = tid == 8 ? -ka.g * dt64 : 0.0;
      const double u2mg = 2.0 * ka.m * ka.g;
      const double ub_alias = (sm[L::CC + N - 1] != 0.0) ? u2mg : 0.0;
      B::sync();
      double dg[N];   // W_k (x_{k+1} - r_k) on lanes < 12
      // u -> x (fp64, lane r < 12 holds x[r]): dg, the heights z_k and, with
      // OUT, x* staged at xo and the objective (phase 7's terms)
      auto rollout = [&](auto outc, double* xo, double& objl) __attribute__((always_inline)) {
        constexpr bool OUT = decltype(outc)::value;
        double xr = tid < 12 ? xin64 : 0.0;
        if (tid == 2) dlo[L::DXZ] = xr;
        if constexpr (OUT) {
          if (tid < 12) xo[tid] = xr;
        }
        const double rdu = tid < 6 ? kRdiag : 0.0;
        const int tu = tid < 6 ? tid : 0;
        sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
          constexpr int k = decltype(kc)::value;
          const double cp = dlo[L::DCS + 2 * k], sp = dlo[L::DCS + 2 * k + 1];
          const double* bwr = d64 + L::DBW + 18 * k + 6 * rw;
          const double* uk = dlo + L::DU + 6 * k;
          double bw_u = 0.0;
#pragma unroll
          for (int c = 0; c < 6; ++c) bw_u = fma(bwr[c], uk[c], bw_u);
          double bv_u;
          if constexpr (VAR == 3) {
            bv_u = dtm64 * uk[rv];
          } else {   // Rz' dt/m
            const double u0 = uk[0], u1 = uk[1], u2 = uk[2];
            bv_u = (rv == 0) ? dtm64 * (cp * u0 - sp * u1) : ((rv == 1) ? dtm64 * (sp * u0 + cp * u1) : dtm64 * u2);
          }
          const double bu = (tid >= 9 && tid < 12) ? bw_u : ((tid >= 6 && tid < 9) ? bv_u : 0.0);
          xr = ad_lane(xr, dt64, cp, sp, tid) + bu + gdt;
          const double kf = (k == N - 1) ? kTermQ : 1.0;
          const double e = xr - d64[L::DXR + 12 * k + (tid < 12 ? tid : 0)];
          dg[k] = kf * qr * e;
          if (tid == 2) dlo[L::DXZ + k + 1] = xr;
          if constexpr (OUT) {
            objl = fma(kf * qr * e, e, objl);
            if constexpr (k < N - 1) {
              const double ub = ka.uref_aliased ? ub_alias : ((sm[L::CC + k] != 0.0) ? u2mg : 0.0);
              const double du = uk[tu] - (tid == 2 ? ub : 0.0);
              objl = fma(rdu * du, du, objl);
            }
            if (tid < 12) xo[12 * (k + 1) + tid] = xr;
          }
        });
      };
      // constraint id's coefficient on this lane's variable, fp64 (coef_of)
      auto coef64 = [&](int id) -> double {
        const int o = id >> 2, sl = id & 3;
        const int oj = __builtin_amdgcn_readlane(vj, o), oc = __builtin_amdgcn_readlane(vc, o);
        if (!active_lane) return 0.0;
        if (oc >= 3) {
          if (sl == 0) return tid == o ? 1.0 : 0.0;
          if (sl == 1) return tid == o ? -1.0 : 0.0;
          if (vc != 2 || vj > oj - 2 || sm[L::CC + vj] == 0.0) return 0.0;
          return zc64 * (double)(oj - 1 - vj);
        }
        if (oc == 2) return tid == o ? (sl == 0 ? 1.0 : -1.0) : 0.0;
        if (tid == o) return sl == 0 ? -1.0 : 1.0;
        return (vj == oj && vc == 2) ? mu64 : 0.0;
      };
      // n' u - b of constraint id, fp64 (the row at the rolled-out u)
      auto slack64 = [&](int id) -> double {
        const int o = id >> 2, sl = id & 3;
        const int fo = dslot[o], oj = fo / 6, oc = fo - 6 * oj;
        const double uo = dlo[L::DU + fo], fz = dlo[L::DU + 6 * oj + 2];
        if (oc >= 3) return sl == 0 ? uo + tau_lim(oc) : (sl == 1 ? tau_lim(oc) - uo : dlo[L::DXZ + oj] - kZmin);
        if (oc == 2) return sl == 0 ? fz : kFzMax - fz;
        return sl == 0 ? fma(mu64, fz, -uo) : fma(mu64, fz, uo);
      };
      double objl = 0.0;
      const int nref = ka.refine;
      double lastdu = INFINITY;   // |du| of the last correction (no correction: not converged)
      const int tq = tid < qu ? tid : 0;
      const double rinv64 = 1.0 / (double)Rm[loff(tq) + tq];   // (R is fixed during the corrections)
      HMPC_TIC(t_ref);
#pragma unroll 1
      for (int it = 0; it < nref; ++it) {
        rollout(std::false_type{}, nullptr, objl);
        // adjoint rows 6..11 (phase 2's recursion on the rollout)
        {
          double ar = dg[N - 1];
          if (tid >= 6 && tid < 12) d64[L::DAJ + 6 * (N - 1) + tid - 6] = ar;
          sfor<1, N>([&](auto ic) __attribute__((always_inline)) {
            constexpr int t = N - decltype(ic)::value;
            ar = adt_lane(ar, dt64, dlo[L::DCS + 2 * t], dlo[L::DCS + 2 * t + 1], tid) + dg[t - 1];
            if (tid >= 6 && tid < 12) d64[L::DAJ + 6 * (t - 1) + tid - 6] = ar;
          });
        }
        B::sync();
        // r1 = N_A lam - (H u + h): the gradient 2 Bd' a + 2 V (u - u_ref) (phase 3's h_v at u)
        double r1 = 0.0;
        if (active_lane) {
          const double cpi = dlo[L::DCS + 2 * vj], spi = dlo[L::DCS + 2 * vj + 1];
          const double* aj = d64 + L::DAJ + 6 * vj;
          const double* bwi = d64 + L::DBW + 18 * vj;
          double hacc = 0.0;
#pragma unroll
          for (int r = 0; r < 3; ++r) hacc = fma(vc < 3 ? bv<VAR>(r, vc, dtm64, cpi, spi) : 0.0, aj[r], hacc);
#pragma unroll
          for (int r = 0; r < 3; ++r) hacc = fma(bwi[6 * r + vc], aj[3 + r], hacc);
          const double ub = vc == 2 ? (ka.uref_aliased ? ub_alias : ((sm[L::CC + vj] != 0.0) ? u2mg : 0.0)) : 0.0;
          const double Vj = (vj == N - 1) ? 0.0 : kRdiag;
          r1 = -2.0 * fma(Vj, u64 - ub, hacc);
        }
#pragma unroll 1
        for (int l = 0; l < qu; ++l) r1 = fma(rdlane(lam, l), coef64(act[l]), r1);
        // r2 = b_A - N_A' u (lane l < q: active row l)
        const double r2 = tid < qu ? -slack64(act[tid < qu ? tid : 0]) : 0.0;
        // the correction, on the fp32 factors
        real w = tri_fwd_lds<L>((real)r1, Lc, zero, dinv, xs, nf, 0);
        real cvec = 0;
        ladder<0, QMAX>(qu, [&](auto lc) __attribute__((always_inline)) {
          constexpr int l = decltype(lc)::value;
          const real cl = B::sum(Qw[l] * w, red);
          w = fma(-cl, Qw[l], w);
          cvec = tid == l ? cl : cvec;
        });
        B::sync();
        double tcur = r2, tmine = 0.0;   // t = R^-T r2 (reciprocals of R's diagonal: rinv64)
#pragma unroll 1
        for (int l = 0; l < qu; ++l) {
          const double tl = rdlane(tcur, l) * rdlane(rinv64, l);
          const double rv = (double)Rm[loff(tid > l && tid < qu ? tid : l) + l];
          tmine = (tid == l) ? tl : tmine;
          tcur = (tid > l && tid < qu) ? fma(-rv, tl, tcur) : tcur;
        }
        double rcur = tid < qu ? tmine - (double)cvec : 0.0, dlam = 0.0;   // dlam = R^-1 (t - c)
#pragma unroll 1
        for (int l = qu - 1; l >= 0; --l) {
          const double rl = rdlane(rcur, l) * rdlane(rinv64, l);
          const double rv = (double)Rm[loff(l) + (tid < l ? tid : 0)];
          dlam = (tid == l) ? rl : dlam;
          rcur = (tid < l) ? fma(-rv, rl, rcur) : rcur;
        }
        real zq = w;   // w - Qw c + Qw t
        ladder<0, QMAX>(qu, [&](auto lc) __attribute__((always_inline)) {
          constexpr int l = decltype(lc)::value;
          zq = fma((real)rdlane(tmine, l), Qw[l], zq);
        });
        const real du = tri_bwd<L>(zq, Lc, zero, dinv, xs, nf);
        u64 += active_lane ? (double)du : 0.0;
        lastdu = active_lane ? fabs((double)du) : 0.0;
        lam += dlam;
        if (active_lane) dlo[L::DU + fidx] = u64;
        B::sync();
        // converged: a correction below kRefineStop on every lane leaves an
        // error <= 0.25 x kRefineStop = 1e-7 (contraction <= cond x eps32 <= 0.2)
        if (!__ballot(lastdu > kRefineStop)) break;
      }
      HMPC_TOC(15, t_ref);
      // outputs: x* (staged over L, dead now) and the objective from an fp64
      // rollout of the refined u
      double* xo = reinterpret_cast<double*>(sm + ((L::XO + 1) & ~1));
      rollout(std::true_type{}, xo, objl);
      const double objv = wave_sum(objl);
      // the fp64 check: every row of this lane (slots as in the slack scan,
      // scaled by the row norms) and the multipliers
      double worst = INFINITY;
      if (active_lane) {
        const int id0 = 4 * tid;
        if (vc >= 3) {
          worst = fmin(slack64(id0), slack64(id0 + 1));
          if (vc == 3 && vj >= 2 && znorm > 0) worst = fmin(worst, slack64(id0 + 2) / (double)znorm);
        } else if (sm[L::CC + vj] != 0.0 && !(VAR == 2 && vc == 1)) {
          const double sc = vc == 2 ? 1.0 : 1.0 / sqrt(1.0 + mu64 * mu64);
          worst = fmin(slack64(id0), slack64(id0 + 1)) * sc;
        }
      }
      // ... and the convergence: the last correction's size bounds the error
      // left after it (contraction ~1/20 measured, cond x eps32 <= 0.2 bound:
      // |du| <= kRefineDu leaves <= 8e-7, inside the fp64 path's 1e-6)
      const bool bad = __ballot(worst < -kRefineTol || (tid < qu && lam < -kRefineTol) || lastdu > kRefineDu) != 0;
      if (bad) {
        status = ka.ovf_count ? ST_OVERFLOW : ST_NUMERICAL;
      } else {
        B::sync();
        if (tid < L::NVF) ka.u[b * L::NVF + tid] = dlo[L::DU + tid];
#ifndef HMPC_STAMPS
        if (ka.x)
          for (int i = tid; i < 12 * (N + 1); i += NT) ka.x[b * 12 * (N + 1) + i] = xo[i];
#else
        HMPC_STAMP(8);
        if (ka.x && tid == 0)
          for (int i = 0; i < 16; ++i)
            reinterpret_cast<long long*>(ka.x)[b * 12 * (N + 1) + i] = stamp_[i];
#endif
        if (tid == 0) {
          if (ka.obj) ka.obj[b] = objv;
          ka.status[b] = ST_SOLVED;
          if (ka.iters) ka.iters[b] = iters;
          if (ka.active) ka.active[b] = q;
        }
        return;
      }
    }
  }
  HMPC_STAMP(7);
  __builtin_amdgcn_s_setprio(kCmpCls ? 0 : kPrioFullBase);

  // an overflowed instance writes nothing but its status and its place in
  // the overflow list (x_lin may be this solve's input, mpcontrol shift)
  if (uni(status) == ST_OVERFLOW) {
    if (tid == 0) {
      a.status[b] = ST_OVERFLOW;
      a.ovf_list[atomicAdd(a.ovf_count, 1)] = (int32_t)b;
    }
    return;
  }
  if constexpr (kRefine) {   // (no fp64 pass to hand it to: the status alone)
    if (tid == 0) a.status[b] = status == ST_SOLVED ? ST_NUMERICAL : status;
    return;
  }

  // ---------------- phase 7: outputs ----------------------------------------
  // u* straight out; x* by a lane-parallel forward simulation (lane r < 12
  // holds x[r]) staged in LDS and written coalesced at the end (per-step
  // 96-byte stores cost ~1.9x the bytes at the memory side); the objective
  // as a per-lane sum + one reduction.
  // x_ref again (its LDS copy is gone): every row's load is issued here,
  // ahead of the rollout, so no memory round trip sits inside it
  const double* xrf7 = reinterpret_cast<const double* const*>(sm + L::XRV)[0];
  const int xrs = reinterpret_cast<const int*>(sm + L::XRV + 2)[0];
  real xrg[N];
  sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    xrg[k] = xrf7[k * xrs + (tid < 12 ? tid : 0)];
  });
  xs[fidx] = v;   // full order (fixed variables: 0)
  __syncthreads();   // L is dead: XO aliases it
  if (tid < L::NVF) a.u[b * L::NVF + tid] = xs[tid];
  {
    real* xo = sm + L::XO;
    real xr = tid < 12 ? sm[L::XIN + tid] : 0.0;
    if (tid < 12) xo[tid] = xr;
    const real qr = qdiag(tid_o);   // (not CSE-d with phase 2's copy)
    const int rw = (tid >= 9 && tid < 12) ? tid - 9 : 0;   // my row of Bd's omega block
    const int rv = (tid >= 6 && tid < 9) ? tid - 6 : 0;    // my row of Bd's velocity block
    // the objective's terms are branch-free: lanes >= 12 carry qr = 0 (and a
    // finite x, x_ref), lanes >= 6 a zero input weight, so their products
    // add exact zeros instead of splitting the wave at every stage
    const real rdu = tid_o < 6 ? real(kRdiag) : real(0);
    const int tu = tid_o < 6 ? tid_o : 0;
    const real ubz = tid_o == 2 ? real(1) : real(0);
    const real gdt = tid_o == 8 ? -real(a.g) * dt : real(0);
    real objl = 0.0;
    // the rollout first (x in registers), the objective after it: the x_ref
    // loads issued above then land while the rollout runs instead of stalling
    // its first stage (round 5)
    real xk[N];
    sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      const real cp = sm[L::CS + 2 * k], sp = sm[L::CS + 2 * k + 1];
      const real* bwr = sm + L::BW + 18 * k + 6 * rw;
      const real* uk = xs + 6 * k;
      real bw_u = 0.0;
#pragma unroll
      for (int c = 0; c < 6; ++c) bw_u = fma(bwr[c], uk[c], bw_u);
      real bv_u = 0.0;
      if constexpr (VAR == 3) {
        bv_u = dtm2 * uk[rv];
      } else {   // Rz' dt/m
        const real u0 = uk[0], u1 = uk[1], u2 = uk[2];
        bv_u = (rv == 0) ? dtm2 * (cp * u0 - sp * u1) : ((rv == 1) ? dtm2 * (sp * u0 + cp * u1) : dtm2 * u2);
      }
      const real bu = (tid >= 9 && tid < 12) ? bw_u : ((tid >= 6 && tid < 9) ? bv_u : 0.0);
      xr = ad_lane(xr, dt, cp, sp) + bu + gdt;
      xk[k] = xr;
      if constexpr (k < N - 1) {
        // (C[k] != 0 is bit k of smask: no LDS round trip inside the rollout)
        const real ub = ((smask >> (a.uref_aliased ? N - 1 : k)) & 1) ? 2.0 * a.m * a.g : 0.0;
        const real du = fma(-ubz, ub, uk[tu]);
        objl = fma(rdu * du, du, objl);
      }
      if (tid < 12) xo[12 * (k + 1) + tid] = xr;
    });
    sfor<0, N>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      const real kf = (k == N - 1) ? kTermQ : 1.0;
      const real e = xk[k] - xrg[k];
      objl = fma(kf * qr * e, e, objl);
    });
    const real objv = B::sum(objl, red);
    __syncthreads();
#ifndef HMPC_STAMPS
    if (a.x)
      for (int i = tid; i < 12 * (N + 1); i += NT) a.x[b * 12 * (N + 1) + i] = xo[i];
#else
    HMPC_STAMP(8);
    if (a.x && tid == 0)
      for (int i = 0; i < 16; ++i)
        reinterpret_cast<long long*>(a.x)[b * 12 * (N + 1) + i] = stamp_[i];
#endif
    if (tid == 0) {
      if (a.obj) a.obj[b] = objv;
      a.status[b] = status;
      if (a.iters) a.iters[b] = iters;
      if (a.active) a.active[b] = q;
    }
  }
}

// Split launch: each instance goes to the compacted one-wave kernel (at most
// NVM free variables: NVM-wide rows, 3 waves / SIMD) or to the full kernel,
// by the number of stance stages of its contact schedule C (free variables
// nf = 3N + (3f: 3, 2f: 2) x stance stages).  One thread per instance; the
// two class lists are appended block by block (one atomic per block and list):
// list A at split_list[0..B), list B at split_list[B..2B), lengths in
// split_count[0..1] (zero at the launch; the overflow pass zeroes them).
constexpr int kClsT = 1024;   // classify threads per block
// a.lpt (small batches): one list per stance-stage count s = 0..N instead
// (bucket s at split_list[s B ..), its length in split_count[s]); each class
// kernel then takes its buckets costliest first (longest-processing-time
// order: at B = 4096 the slowest instances start first instead of last).
template <int VAR, int N>
__global__ void __launch_bounds__(kClsT) classify_buckets_kernel(SolveArgs a) {
  __shared__ int wc[kClsT / 64][N + 1];
  __shared__ int base[N + 1];
  const int64_t i = (int64_t)blockIdx.x * kClsT + threadIdx.x;
  const bool in = i < a.B;
  int nst = 0;
  if (in) {
    const double* c = a.C + i * a.C_bs;
#pragma unroll
    for (int k = 0; k < N; ++k) nst += c[k] != 0.0 ? 1 : 0;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t mine = 0;
#pragma unroll
  for (int s = 0; s <= N; ++s) {
    const uint64_t m = __ballot(in && nst == s);
    mine = (in && nst == s) ? m : mine;
    if (lane == 0) wc[w][s] = __builtin_popcountll(m);
  }
  __syncthreads();
  if (threadIdx.x <= N) {   // thread s: exclusive scan of bucket s over the waves, one atomic
    const int s = threadIdx.x;
    int t = 0;
    for (int v = 0; v < kClsT / 64; ++v) {
      const int c = wc[v][s];
      wc[v][s] = t;
      t += c;
    }
    base[s] = t ? atomicAdd(a.split_count + s, t) : 0;
  }
  __syncthreads();
  if (in) a.split_list[(int64_t)nst * a.B + base[nst] + wc[w][nst] + __builtin_popcountll(mine & ((1ull << lane) - 1))] = (int32_t)i;
}
// SW: the all-swing windows (no stance stage) form a third list at
// split_list[2B..3B), length split_count[2] (hmpc_swing.hip's class)
template <int VAR, int N, int NVM, bool SW = false>
__global__ void __launch_bounds__(kClsT) classify_kernel(SolveArgs a) {
  // (one atomic per block and list: per-wave atomics on the two counters
  // serialised at the L2 and made this pass 25 us of a 1.3 ms step)
  __shared__ int wc[kClsT / 64][3];
  __shared__ int base[3];
  const int64_t i = (int64_t)blockIdx.x * kClsT + threadIdx.x;
  const bool in = i < a.B;
  int nst = 0;
  if (in) {
    const double* c = a.C + i * a.C_bs;
#pragma unroll
    for (int k = 0; k < N; ++k) nst += c[k] != 0.0 ? 1 : 0;
  }
  const int nf = 3 * N + (VAR == 3 ? 3 : 2) * nst;
  const bool sw = SW && in && nst == 0;
  const bool cmp = in && !sw && nf <= NVM, full = in && !sw && !cmp;
  const uint64_t mc = __ballot(cmp), mf = __ballot(full), ms = __ballot(sw);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    wc[w][0] = __builtin_popcountll(mc);
    wc[w][1] = __builtin_popcountll(mf);
    wc[w][2] = __builtin_popcountll(ms);
  }
  __syncthreads();
  if (threadIdx.x < (SW ? 3 : 2)) {   // exclusive scan of list t's wave counts, one atomic
    const int t = threadIdx.x;
    int tc = 0;
    for (int v = 0; v < kClsT / 64; ++v) {
      const int c = wc[v][t];
      wc[v][t] = tc;
      tc += c;
    }
    base[t] = tc ? atomicAdd(a.split_count + t, tc) : 0;
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1;
  if (cmp) a.split_list[base[0] + wc[w][0] + __builtin_popcountll(mc & lt)] = (int32_t)i;
  if (full) a.split_list[a.B + base[1] + wc[w][1] + __builtin_popcountll(mf & lt)] = (int32_t)i;
  if (SW && sw) a.split_list[2 * a.B + base[2] + wc[w][2] + __builtin_popcountll(ms & lt)] = (int32_t)i;
}

}  // namespace

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

#ifndef HMPC_LAUNCH_SUFFIX
#define HMPC_LAUNCH_SUFFIX
#endif
#if defined(HMPC_CMP_NV) && HMPC_CMP_NV > 0
// the split's compacted kernel launches from a translation unit of its own
// (-DHMPC_CMP_ONLY): the objects build in parallel
// (one launcher per build flavour: HMPC_LAUNCH_SUFFIX, e.g. _f32)
#define HMPC_CMP_LAUNCH HMPC_CAT(HMPC_CAT(launch_cmp_n, HMPC_INST_N), HMPC_LAUNCH_SUFFIX)
#define HMPC_FULL2F_LAUNCH HMPC_CAT(HMPC_CAT(launch_full2f_n, HMPC_INST_N), HMPC_LAUNCH_SUFFIX)
bool HMPC_CMP_LAUNCH(int variant, const SolveArgs& a, hipStream_t s);
// 2f's full class: at most 5N free variables (3N torques + 2N stance forces;
// f_y is fixed), so a 5N-wide compacted kernel replaces the 6N-wide full one
// when 5N rows fit one wave (same capacity as the full kernel)
#if 5 * HMPC_INST_N > HMPC_CMP_NV && 5 * HMPC_INST_N <= 64
#define HMPC_FULL2F_NV (5 * HMPC_INST_N)
#define HMPC_FULL2F_Q (Lay<HMPC_INST_N>::QMAX)
bool HMPC_FULL2F_LAUNCH(const SolveArgs& a, hipStream_t s);
#endif
#endif
// the all-swing class (hmpc_swing.hip, fp64 objects built with HMPC_SWING):
// two instances per wave
#if defined(HMPC_SWING) && HMPC_SWING && !defined(HMPC_CMP_ONLY)
#define HMPC_SWING_LAUNCH HMPC_CAT(launch_swing_n, HMPC_INST_N)
bool HMPC_SWING_LAUNCH(const SolveArgs& a, hipStream_t s);
int HMPC_CAT(swing_qmax_n, HMPC_INST_N)();
#endif
#ifdef HMPC_CMP_ONLY
bool HMPC_CMP_LAUNCH(int variant, const SolveArgs& a, hipStream_t s) {
  if (variant == 3)
    hipLaunchKernelGGL((solve_kernel<3, HMPC_INST_N, real, HMPC_CMP_NV, HMPC_CMP_Q>), dim3((unsigned)a.B), dim3(64),
                       0, s, a);
  else
    hipLaunchKernelGGL((solve_kernel<2, HMPC_INST_N, real, HMPC_CMP_NV, HMPC_CMP_Q>), dim3((unsigned)a.B), dim3(64),
                       0, s, a);
  return true;
}
#ifdef HMPC_FULL2F_NV
bool HMPC_FULL2F_LAUNCH(const SolveArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((solve_kernel<2, HMPC_INST_N, real, HMPC_FULL2F_NV, HMPC_FULL2F_Q>), dim3((unsigned)a.B), dim3(64),
                     0, s, a);
  return true;
}
#endif
#else
bool HMPC_CAT(HMPC_CAT(launch_solve_n, HMPC_INST_N), HMPC_LAUNCH_SUFFIX)(int variant, const SolveArgs& a,
                                                                     hipStream_t s) {
  constexpr int N = HMPC_INST_N;
  constexpr int NT = Lay<N>::NT;
  if (a.B <= 0) return true;
  if (variant != 2 && variant != 3) return false;
  SolveArgs af = a;
  af.list = nullptr;
  af.list_count = nullptr;
#if defined(HMPC_CMP_NV) && HMPC_CMP_NV > 0
  if (a.split_list && a.split_count) {   // classify, then one launch per class
    const unsigned cb = (unsigned)((a.B + kClsT - 1) / kClsT);
    SolveArgs ac = af;
    ac.list = a.split_list;
    ac.list_count = a.split_count;
    af.list = a.split_list + a.B;
    af.list_count = a.split_count + 1;
#ifdef HMPC_SWING_LAUNCH
    constexpr bool kSw = true;
#else
    constexpr bool kSw = false;
#endif
    SolveArgs as = af;   // the all-swing class (kSw): list 2, or bucket 0
    as.list = a.split_list + 2 * a.B;
    as.list_count = a.split_count + 2;
    if (a.lpt && a.split_nbkt >= N + 1) {
      // bucket ranges: the compacted class takes s <= smax, the full class the rest
      const int smax = (HMPC_CMP_NV - 3 * N) / (variant == 3 ? 3 : 2);
      ac.list = af.list = a.split_list;
      ac.list_count = af.list_count = a.split_count;
      // (the all-swing class runs in index order only: with longest-first
      // order at B = 4096 it cost 8-12 %, configs[1] 24.3 -> 22.3 M, since
      // those windows are the cheapest and fill the tail as bucket 0 of the
      // compacted class; profiles/r05_ab.json)
      ac.lpt_lo = 0;
      ac.lpt_hi = smax;
      af.lpt_lo = smax + 1;
      af.lpt_hi = N;
      as.list = a.split_list;
      as.list_count = a.split_count;
      if (variant == 3) hipLaunchKernelGGL((classify_buckets_kernel<3, N>), dim3(cb), dim3(kClsT), 0, s, a);
      else hipLaunchKernelGGL((classify_buckets_kernel<2, N>), dim3(cb), dim3(kClsT), 0, s, a);
    } else {
      if (variant == 3) hipLaunchKernelGGL((classify_kernel<3, N, HMPC_CMP_NV, kSw>), dim3(cb), dim3(kClsT), 0, s, a);
      else hipLaunchKernelGGL((classify_kernel<2, N, HMPC_CMP_NV, kSw>), dim3(cb), dim3(kClsT), 0, s, a);
    }
    // the classes run concurrently: the full kernel on the caller's
    // stream, the compacted one on the split stream, joined back before the
    // overflow pass (one kernel's tail fills with the other's waves)
    hipStream_t s2 = s;
    if (a.split_stream && a.split_fork && a.split_join) {
      if (hipEventRecord(a.split_fork, s) != hipSuccess) return false;
      if (hipStreamWaitEvent(a.split_stream, a.split_fork, 0) != hipSuccess) return false;
      s2 = a.split_stream;
    }
    // The classes' order on the two streams (interleaved A/B, profiles/r05_ab.json):
    //   large batches: swing then full on the caller's stream, compacted on the
    //   split stream -- configs[2] (B = 65536) 57.0 -> 58.8 M solves/s;
    //   otherwise full on the caller's stream, swing then compacted on the split
    //   stream -- B = 16384 45.5 vs 42.1 M, configs[1] 22.3 vs 18.5 M.
    // Re-measured at round end (r05_knob_*): full first at B = 65536 62.6 vs
    // 63.8 M; the swing class in the longest-first order costs 10-12 % at
    // B = 4096 (28.4 -> 25.6 M at configs[1]) and nothing at 8192.
    auto full_on = [&](hipStream_t st) {
      if (variant == 3) hipLaunchKernelGGL((solve_kernel<3, N, real>), dim3((unsigned)a.B), dim3(NT), 0, st, af);
#ifdef HMPC_FULL2F_NV
      else HMPC_FULL2F_LAUNCH(af, st);
#else
      else hipLaunchKernelGGL((solve_kernel<2, N, real>), dim3((unsigned)a.B), dim3(NT), 0, st, af);
#endif
    };
    auto cmp_on = [&](hipStream_t st) { HMPC_CMP_LAUNCH(variant, ac, st); };
#ifdef HMPC_SWING_LAUNCH
    auto swing_on = [&](hipStream_t st) { HMPC_SWING_LAUNCH(as, st); };
#else
    auto swing_on = [&](hipStream_t) { (void)as; };
#endif
#ifndef HMPC_SWING_FIRST_B
#define HMPC_SWING_FIRST_B 32768
#endif
    if (kSw && !a.lpt && a.B >= HMPC_SWING_FIRST_B) {
      swing_on(s);
      full_on(s);
      cmp_on(s2);
    } else {
      full_on(s);
      if (!a.lpt) swing_on(s2);
      cmp_on(s2);
    }
    if (s2 != s) {
      if (hipEventRecord(a.split_join, s2) != hipSuccess) return false;
      if (hipStreamWaitEvent(s, a.split_join, 0) != hipSuccess) return false;
    }
    return true;
  }
#endif
  if (variant == 3) hipLaunchKernelGGL((solve_kernel<3, N, real>), dim3((unsigned)a.B), dim3(NT), 0, s, af);
  else hipLaunchKernelGGL((solve_kernel<2, N, real>), dim3((unsigned)a.B), dim3(NT), 0, s, af);
  return true;
}

#ifdef HMPC_REAL_FP64
// the fp64 objects only (HMPC_LAUNCH_SUFFIX empty): the full-class kernel
// (any free-variable count) over a caller's list -- HMPC_PREC_F32_REFINED's
// fallback pass re-solves the instances its fp64 check rejected here, at the
// dense kernel's speed, instead of in the generic capacity-6N pass
bool HMPC_CAT(HMPC_CAT(launch_list_n, HMPC_INST_N), HMPC_LAUNCH_SUFFIX)(int variant, const SolveArgs& a,
                                                                    hipStream_t s) {
  constexpr int N = HMPC_INST_N;
  if (a.B <= 0) return true;
  if (!a.list || !a.list_count) return false;
  if (variant == 3) hipLaunchKernelGGL((solve_kernel<3, N, real>), dim3((unsigned)a.B), dim3(Lay<N>::NT), 0, s, a);
#ifdef HMPC_FULL2F_NV
  else HMPC_FULL2F_LAUNCH(a, s);
#else
  else hipLaunchKernelGGL((solve_kernel<2, N, real>), dim3((unsigned)a.B), dim3(Lay<N>::NT), 0, s, a);
#endif
  return true;
}
#endif

// this object's active-set capacity and kernel names (hmpc_active_capacity,
// hmpc_kernel_name: read from here, not restated in the C API)
#define HMPC_STR2(x) #x
#define HMPC_STR(x) HMPC_STR2(x)
// (the split's classes: the smallest capacity; the names of every class)
#if defined(HMPC_CMP_NV) && HMPC_CMP_NV > 0
#define HMPC_SPLIT_NV HMPC_CMP_NV
constexpr int kCapCmp = Lay<HMPC_INST_N, HMPC_CMP_NV, HMPC_CMP_Q>::QMAX;
#else
#define HMPC_SPLIT_NV 0
constexpr int kCapCmp = 1 << 30;
#endif
int HMPC_CAT(HMPC_CAT(qmax_solve_n, HMPC_INST_N), HMPC_LAUNCH_SUFFIX)() {
  int q = Lay<HMPC_INST_N>::QMAX < kCapCmp ? Lay<HMPC_INST_N>::QMAX : kCapCmp;
#ifdef HMPC_SWING_LAUNCH
  const int qs = HMPC_CAT(swing_qmax_n, HMPC_INST_N)();
  q = qs < q ? qs : q;
#endif
  return q;
}
int HMPC_CAT(HMPC_CAT(split_nv_n, HMPC_INST_N), HMPC_LAUNCH_SUFFIX)() { return HMPC_SPLIT_NV; }
const char* HMPC_CAT(HMPC_CAT(name_solve_n, HMPC_INST_N), HMPC_LAUNCH_SUFFIX)(int variant) {
  // (the template arguments as rocprofv3 demangles them; split classes:
  // all-swing + compacted + full).  Built once per variant, thread-safely
  // (function-local statics).
  if (variant != 2 && variant != 3) return "";
  auto build = [](int var) {
    std::string name;
    const char* real_s = HMPC_STR(HMPC_REAL);
    char buf[160];
    auto add = [&](const char* k, int nv, int q) {
      snprintf(buf, sizeof buf, "%shmpc::%s<%d, %d, %s, %d, %d>", name.empty() ? "" : " + ", k, var,
               HMPC_INST_N, real_s, nv, q);
      name += buf;
    };
#if defined(HMPC_CMP_NV) && HMPC_CMP_NV > 0
#ifdef HMPC_SWING_LAUNCH
    snprintf(buf, sizeof buf, "hmpc::swing_kernel<%d, %d>", HMPC_INST_N, HMPC_CAT(swing_qmax_n, HMPC_INST_N)());
    name += buf;
#endif
    add("solve_kernel", HMPC_CMP_NV, HMPC_CMP_Q);
#ifdef HMPC_FULL2F_NV
    if (var == 2) add("solve_kernel", HMPC_FULL2F_NV, HMPC_FULL2F_Q);
    else add("solve_kernel", 0, 0);
#else
    add("solve_kernel", 0, 0);
#endif
#else
    add("solve_kernel", 0, 0);
#endif
    return name;
  };
  static const std::string n2 = build(2), n3 = build(3);
  return variant == 2 ? n2.c_str() : n3.c_str();
}
#endif  // HMPC_CMP_ONLY

}  // namespace hmpc
