// Internal interface between the C ABI (hmpc_capi.cpp) and the kernels
// (hmpc_kernels.hip).  Not installed; include/hmpc.h is the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hmpc {

// Problem constants of Mpc.__init__ (src/mpc_cvx_euler_3f.py:12-39) plus the
// per-call batch pointers.  Passed to the kernel by value.
struct SolveArgs {
  const double* x_in;    // [B,12]
  const double* x_lin;   // [B,N+1,12]
  const double* x_ref;   // [B,N,12]
  const double* pf;      // [B,N,3]
  const double* C;       // [B,N]
  const double* mu;      // [B] or nullptr
  double* u;             // [B,N,6]
  double* x;             // [B,N+1,12] or nullptr
  double* obj;           // [B] or nullptr
  int32_t* status;       // [B]
  int32_t* iters;        // [B] or nullptr
  int32_t* active;       // [B] final active-set size, or nullptr
  int64_t B;
  double dt, m, g, mu_default;
  double Jinv[9];
  double rh[3];
  int uref_aliased;
  // mpcontrol support: when shift_mode != 0 the kernel builds x_lin itself
  //   1: x_lin = [x_in; x_ref]                 (init pass 1)
  //   2: x_lin = [x_in; x_prev[2:]; x_prev[N]] (time shift of the previous x*)
  // and x_lin points at x_prev (mode 2).
  int shift_mode;
  // element strides of the x_ref / pf / C views (contiguous: 12N, 12 / 3N, 3
  // / N); a batch stride of 0 shares one plan window across the batch
  int64_t xref_bs, pf_bs, C_bs;
  int xref_rs, pf_rs;
  // global workspace of the generic-horizon kernel (hmpc_wide.hip): one
  // WideLayout(N).total block per resident workgroup
  double* ws;
  int64_t ws_stride;   // in elements of the arithmetic type
  int ws_groups;
  // HMPC_PREC_*: 0 fp64 (fastest kernel for N), 1 fp32 (dense fp32 build
  // where compiled, else generic), 2 fp64 generic, 3 fp64 Riccati, 4 fp64
  // dense, 5 fp32 generic, 6 fp32 + fp64 refinement
  int precision;
  // the fp64 corrections of the refined fp32 build (HMPC_PREC_F32_REFINED)
  int refine;
  // Active-set overflow (hmpc_ric.hip): an instance whose active set outgrows
  // the LDS capacity of its kernel appends its index to ovf_list (count in
  // *ovf_count; ovf_count[1] is the Riccati instance counter, [2] the
  // overflow pass's done counter: zero at the launch -- the overflow pass
  // zeroes all three at its end) and is re-solved by the overflow
  // pass with capacity 6N (R in the global workspace rws, rws_stride doubles
  // per resident workgroup).  ovf_count == nullptr: overflow = ST_NUMERICAL.
  int32_t* ovf_count;
  int32_t* ovf_list;
  // running total of the instances the overflow pass re-solved on this
  // context (hmpc_overflow_total), or nullptr
  unsigned long long* ovf_total;
  // a second overflow header (HMPC_PREC_F32_REFINED): the instances of
  // ovf_list were first re-solved by the fp64 dense kernel (launch_solve_fp64_list),
  // whose own overflows went to this pass's list; the pass zeroes that first
  // header (count, counters, split counts) too and counts its instances in
  // ovf_total.  nullptr: one header.
  int32_t* ovf_hdr1;
  double* rws;
  int64_t rws_stride;
  // Riccati kernel (persistent): instance counter (zeroed before the launch),
  // resident workgroups and their K / Dinv workspace (kws_stride doubles each)
  int32_t* work;
  // the number of tickets (instances of a.list) when shorter than B, or nullptr
  const int32_t* work_bound;
  int ric_groups;
  double* kws;
  int64_t kws_stride;
  // the Riccati factorisation kernel's output (ric_kinst_stride): K / Dinv and
  // a pivot flag per instance, kinst_stride doubles each; nullptr = the solve
  // kernel factorises in its own slot
  double* kinst;
  int64_t kinst_stride;
  // Dense split launch (hmpc_kernels.hip, objects built with HMPC_CMP_NV):
  // [compacted count | full count] (zero at the launch, zeroed again by the
  // overflow pass at its end) and the two class lists [2][B]; nullptr = one
  // launch of the full kernel.  list / list_count: set per launch by the
  // launcher (the kernel's class list), nullptr = block i solves instance i.
  int32_t* split_count;
  int32_t* split_list;
  const int32_t* list;
  const int32_t* list_count;
  // lpt != 0 (small batches, chosen by the C ABI): longest-first order.  The
  // dense split's class lists are then buckets by stance-stage count
  // (list[s * B ..], count list_count[s]) and a launch serves buckets
  // lpt_lo..lpt_hi, costliest (most stance stages) first (lpt_hi < 0: one
  // plain list); the Riccati kernel's work queue walks its buckets the same
  // way.  split_nbkt: the bucket counters the overflow pass zeroes.
  int lpt;
  int lpt_lo, lpt_hi, split_nbkt;
  // the split's second class runs concurrently on split_stream (forked from
  // and joined back into the caller's stream by the two events); nullptr:
  // both classes on the caller's stream, one after the other
  hipStream_t split_stream;
  hipEvent_t split_fork, split_join;
};

// The Riccati kernel (hmpc_ric.hip): any horizon 1 <= N <= kRicNmax, one
// wavefront per instance.
constexpr int kRicNmax = 64;
// default precision: dedicated dense kernels win up to this horizon
constexpr int kDenseNmax = 10;
constexpr int ST_OVERFLOW = 4;   // internal: re-solved by the overflow pass
// LDS capacity of R for the main pass at horizon N
// Active-set capacity of the main Riccati kernel's LDS-resident R and its
// occupancy (waves per SIMD): the largest capacity <= min(64, 6N) whose LDS
// fits 8 workgroups per CU (2 waves / SIMD, the register budget compiled into
// ric_kernel<VAR, 2>) with capacity >= 32, else 4 workgroups per CU (1 wave /
// SIMD).  Larger active sets go to the overflow pass.
int ric_qcap(int N);
// ... for a batch of B instances (the Runner's N = 60 at small batches runs a
// capacity-64 solve kernel, hmpc_ric.hip)
int ric_qcap_batch(int N, int64_t B);
int ric_occ(int N);
// the compile-time horizon the Riccati kernel for N runs with (0: runtime N)
int ric_static_n(int N);
// dynamic LDS bytes of the Riccati kernel at horizon N (R in LDS with
// capacity qcap, or none when qcap == 0: overflow pass)
size_t ric_lds_bytes(int N, int qcap);
int64_t ric_kws_stride(int N);   // per-workgroup K / Dinv workspace (doubles)
int64_t ric_rws_stride(int N);   // per-workgroup overflow block: R (6N capacity) + workspace
int ric_groups(int variant, int N);   // resident workgroups of the main Riccati kernel
// per-instance K / Dinv block of the Riccati factorisation kernel, doubles
// (0: the factorisation stays in the solve kernel)
int64_t ric_kinst_stride(int N, int64_t B);
// stance-count buckets of the Riccati kernel's longest-first work queue at
// horizon N (0: plain index order); their lists take buckets x B ints
int ric_lpt_buckets(int N);
bool launch_solve_ric(int variant, int N, const SolveArgs& a, hipStream_t stream);
// the fp64 dense kernel of horizon N (its full class: any free-variable
// count) over a.list / *a.list_count, one workgroup per entry, grid a.B; false
// when no dense fp64 object serves N.  HMPC_PREC_F32_REFINED's fallback pass.
bool launch_solve_fp64_list(int variant, int N, const SolveArgs& a, hipStream_t s);
// N = 60 with the large-batch capacity (47): a second-tier pass of the
// capacity-64 solve kernel over the main pass's overflow list (a.list, count
// *a.work_bound, its own ticket counter a.work) before the generic pass
bool ric_has_tier2(int N, int64_t B);
bool launch_solve_ric_tier2(int variant, int N, const SolveArgs& a, hipStream_t s);
// the overflow pass over a.ovf_list (count on the device), <= groups workgroups
bool launch_solve_ric_overflow(int variant, int N, const SolveArgs& a, int groups, hipStream_t s);

// Horizons without a dedicated kernel run on the generic kernel up to this N.
constexpr int kWideNmax = 128;

// Per-instance workspace of the generic-horizon kernel, in elements of its
// arithmetic type.  The two NV x NV blocks (H -> L, J = L^-T Q) dominate:
// 2.1 MB at N = 60 in fp64.
struct WideLayout {
  int64_t XIN, CC, CS, BW, ZB, XL, XR, PF, SS, DG, AJ;         // per stage
  int64_t HV, XV, DV, ZV, WV, UO, RV, UA, FR, POS, ACT, ISA;   // per variable
  int64_t RM, H, J, total;
  __host__ __device__ explicit WideLayout(int N) {
    const int64_t NV = 6 * (int64_t)N;
    auto up = [](int64_t x) { return (x + 15) & ~(int64_t)15; };   // 128-B aligned
    int64_t o = 0;
    XIN = o; o = up(o + 12);
    CC = o; o = up(o + N);
    CS = o; o = up(o + 2 * N);
    BW = o; o = up(o + 18 * N);
    ZB = o; o = up(o + N + 1);
    XL = o; o = up(o + 12 * N);
    XR = o; o = up(o + 12 * N);
    PF = o; o = up(o + 3 * N);
    SS = o; o = up(o + 22 * N);
    DG = o; o = up(o + 12 * N);
    AJ = o; o = up(o + 6 * N);
    HV = o; o = up(o + NV);
    XV = o; o = up(o + NV);
    DV = o; o = up(o + NV);
    ZV = o; o = up(o + NV);
    WV = o; o = up(o + NV);
    UO = o; o = up(o + NV);
    RV = o; o = up(o + NV);
    UA = o; o = up(o + NV + 1);
    FR = o; o = up(o + NV);          // int slots (one per double)
    POS = o; o = up(o + NV);
    ACT = o; o = up(o + NV + 1);
    ISA = o; o = up(o + 4 * NV);
    RM = o;   // (R lives in LDS; kept for layout compatibility, no space)
    H = o; o = up(o + NV * NV);
    J = o; o = up(o + NV * NV);
    total = o;
  }
};

// The Runner's plant (hmpc_plant.hip): n_steps RK4 steps of dynamics_ct with
// the input held, per robot (src/robotrunner.py:104-113,126-164).
struct PlantArgs {
  int64_t B;
  int n_steps;
  double dt, m, g;
  double J[9], Jinv[9], rh[3];
  double* X;              // [B,13] in/out (SE(3) state, quaternion w-first)
  const double* U;        // row b at U + b*U_bs (first 6 entries: the held input)
  int64_t U_bs;
  const double* pf;       // step s of robot b at pf + b*pf_bs + s*pf_ss
  int64_t pf_bs, pf_ss;
  double* X_hist;         // [B,n_steps,13] or nullptr
  double* x_out;          // [B,12] convert(X) after the last step, or nullptr
};
void launch_plant(const PlantArgs& a, hipStream_t s);
void launch_convert(int64_t B, const double* X, double* x, hipStream_t s);
// the CasADi variant's kernel (hmpc_cas.hip): R slots of cas_ws_stride
// doubles per resident workgroup in a.kws, instance counter a.work,
// a.ric_groups workgroups
constexpr int kCasNmax = 11;
size_t cas_lds_bytes(int N);
int64_t cas_ws_stride(int N);
int cas_groups(int N);
bool launch_solve_cas(int N, const SolveArgs& a, hipStream_t s);
// the Runner's planner (hmpc_planner.hip)
int64_t plan_scratch_bytes(int64_t B, int T);
bool launch_plan(int64_t B, int N_run, int N_k, double dt, int curve, double t_p, double phi_switch,
                 double t_start, int step_adjustment, const double* x_in, const double* xf, double* x_ref,
                 double* pf_ref, double* C_map, void* scratch, hipStream_t s);
// the planner's device error word inside its scratch (nonzero: the reference
// would raise IndexError or keep more footstep peaks than fit)
const int32_t* plan_error_word(int64_t B, int T, const void* scratch);
bool launch_gait(int n_steps, int mpc_factor, int N, double dt, double mpc_dt, double t_p,
                 double phi_switch, double t_start, double t0, double* C_calls, double* s_hist,
                 hipStream_t s);

// Which kernel solves (variant, N) at a precision (HMPC_PREC_*).
enum class Kernel { None, Dense, DenseF32, DenseF32R, Riccati, Wide, Cas };
Kernel pick_kernel(int variant, int N, int precision);
// Launch the solve kernel for (variant, N, a.precision).  Returns false when
// no kernel serves that combination.  Dense and Riccati kernels honour
// a.ovf_count (the caller then runs launch_solve_ric_overflow).
bool launch_solve(int variant, int N, const SolveArgs& a, hipStream_t stream);
// the generic-horizon kernel (any 1 <= N <= kWideNmax); a.ws must be set
bool launch_solve_wide(int variant, int N, const SolveArgs& a, hipStream_t stream);
// the dedicated dense kernel's active-set capacity (-1: none) and name, as
// its own object reports them (hmpc_kernels.hip); flavor 0 fp64, 1 fp32,
// 2 fp32 + fp64 refinement
int dense_qmax(int N, int flavor);
// free-variable bound of the dense split's compacted kernel (0: no split)
int dense_split_nv(int N, int flavor);
const char* dense_name(int variant, int N, int flavor);
bool horizon_supported(int variant, int N);   // compiled, or generic (N <= kWideNmax)
bool horizon_compiled(int variant, int N);    // a dedicated one-wavefront kernel
int supported_horizons(int variant, int* Ns, int cap);

}  // namespace hmpc
