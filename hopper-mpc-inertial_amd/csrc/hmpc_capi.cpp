// hmpc_capi.cpp -- the C ABI declared in include/hmpc.h.
//
// A context is the device-side counterpart of one reference ``Mpc`` object
// (src/mpc_cvx_euler_3f.py:12-39): it holds the constants and, for the
// host-pointer entry points, staging buffers on its device.  Nothing here
// computes on the CPU: every solve is a kernel launch.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "../../include/hmpc.h"
#include "hmpc_internal.h"

struct hmpc_ctx {
  int variant;
  int N;
  int device;
  double t, m, g, mu;
  double Jinv[9];
  double rh[3];
  int uref_mode;
  int precision = HMPC_PREC_F64;
  int refine = 5;   // fp64 corrections of HMPC_PREC_F32_REFINED (hmpc_set_refinement)
  int order = HMPC_ORDER_AUTO;   // instance order of the dense split / Riccati queue (hmpc_set_order)
  std::string err;
  // staging buffers (host API) and mpcontrol scratch
  void* dbuf = nullptr;
  size_t dbuf_bytes = 0;
  int32_t* scratch_i32 = nullptr;
  int64_t scratch_n = 0;
  // generic-horizon kernel workspace (hmpc_wide.hip)
  double* wsbuf = nullptr;
  int wsgroups = 0;
  // active-set overflow pass (hmpc_ric.hip): [overflow count | Riccati
  // instance counter | done counter | split counts (up to N + 1 <= 13
  // buckets) | list of ovf_cap ids] and the global R blocks of its workgroups
  int32_t* ovf = nullptr;
  int64_t ovf_cap = 0;
  unsigned long long* ovf_total = nullptr;   // hmpc_overflow_total
  // the counters need a zeroing before the next solve (fresh buffer, or a
  // solve whose overflow pass -- which zeroes them at its end -- did not run)
  bool ovf_dirty = true;
  bool ovf_total_failed = false;   // the diagnostic counter could not be allocated
  bool ovf2_zeroed = false;   // the second overflow header (run_solve) is zero
  int ric_cap_last = 0;   // the Riccati main pass's active-set capacity in the last solve (0: none yet)
  double* rws = nullptr;
  // dense split launch: the three class lists [3][split_cap], or (longest-first
  // order) up to N + 1 stance-count buckets of split_cap entries; the Riccati
  // kernel's longest-first queue uses the same buffer for its buckets
  int32_t* split = nullptr;
  int64_t split_cap = 0;
  int split_nbuf = 0;   // lists of split_cap entries the buffer holds
  // the last Riccati solve at a one-wave horizon ran the fused kernel (no
  // per-instance K / Dinv buffer: beyond its 4 GB bound or out of memory)
  bool ric_fused = false;
  // the last dense solve ran in longest-first order (the all-swing class
  // then stays in the compacted class, hmpc_kernels.hip)
  bool dense_lpt = false;
  hipStream_t split_stream = nullptr;   // the compacted class's stream
  hipEvent_t split_fork = nullptr, split_join = nullptr;
  // Riccati kernel: per-workgroup K / Dinv workspace of its resident grid
  double* kws = nullptr;
  int ric_groups = 0;
  // Riccati factorisation kernel: K / Dinv per instance (kinst_cap instances)
  double* kinst = nullptr;
  int64_t kinst_cap = 0;
  // planner scratch (footstep counter, peak lists)
  void* plan_scratch = nullptr;
  int64_t plan_scratch_bytes = 0;
  hipStream_t own_stream = nullptr;
  // cross-stream ordering: the workspaces and self-resetting counters above
  // are per context, so a solve issued on another stream than the last one
  // first waits for the last one's completion event (no silent race)
  hipEvent_t last_ev = nullptr;
  hipStream_t last_stream = nullptr;
  bool has_last = false;
};

namespace {

int fail_hip(hmpc_ctx* c, hipError_t e, const char* where) {
  if (c) c->err = std::string(where) + ": " + hipGetErrorString(e);
  return HMPC_ERR_HIP;
}

#define HMPC_HIP(ctx, call)                                   \
  do {                                                        \
    hipError_t e_ = (call);                                   \
    if (e_ != hipSuccess) return fail_hip((ctx), e_, #call);  \
  } while (0)

hmpc::SolveArgs make_args(hmpc_ctx* c, int64_t B, const double* x_in, const double* x_lin,
                          const double* x_ref, const double* pf, const double* C,
                          const double* mu, double* u, double* x, double* obj, int32_t* status,
                          int32_t* iters, int shift_mode) {
  hmpc::SolveArgs a;
  a.x_in = x_in; a.x_lin = x_lin; a.x_ref = x_ref; a.pf = pf; a.C = C; a.mu = mu;
  a.u = u; a.x = x; a.obj = obj; a.status = status; a.iters = iters; a.active = nullptr;
  a.B = B;
  a.dt = c->t; a.m = c->m; a.g = c->g; a.mu_default = c->mu;
  memcpy(a.Jinv, c->Jinv, sizeof(a.Jinv));
  memcpy(a.rh, c->rh, sizeof(a.rh));
  a.uref_aliased = c->uref_mode == HMPC_UREF_ALIASED ? 1 : 0;
  a.shift_mode = shift_mode;
  const int N = c->N;
  a.xref_bs = 12 * (int64_t)N; a.xref_rs = 12;
  a.pf_bs = 3 * (int64_t)N; a.pf_rs = 3;
  a.C_bs = N;
  a.ws = nullptr; a.ws_stride = 0; a.ws_groups = 0;
  a.ovf_count = nullptr; a.ovf_list = nullptr; a.rws = nullptr; a.rws_stride = 0;
  a.ovf_total = nullptr;
  a.ovf_hdr1 = nullptr;
  a.work = nullptr; a.work_bound = nullptr; a.kws = nullptr; a.kws_stride = 0; a.ric_groups = 0;
  a.kinst = nullptr; a.kinst_stride = 0;
  a.split_count = nullptr; a.split_list = nullptr; a.list = nullptr; a.list_count = nullptr;
  a.lpt = 0; a.lpt_lo = 0; a.lpt_hi = -1; a.split_nbkt = 0;
  a.split_stream = nullptr; a.split_fork = nullptr; a.split_join = nullptr;
  a.precision = c->precision;
  a.refine = c->refine;
  return a;
}

// Horizons without a dedicated kernel: make sure the context's workspace
// covers min(B, kMaxGroups) resident workgroups and point the args at it.
constexpr int kMaxGroups = 512;
constexpr size_t kWsBudget = (size_t)4 << 30;   // bytes

int prepare_ws(hmpc_ctx* c, int64_t B, hmpc::SolveArgs& a) {
  if (hmpc::pick_kernel(c->variant, c->N, c->precision) != hmpc::Kernel::Wide) return HMPC_OK;
  const hmpc::WideLayout Lw(c->N);
  const size_t per = (size_t)Lw.total * sizeof(double);
  int64_t want = B < kMaxGroups ? B : kMaxGroups;
  const int64_t cap = (int64_t)(kWsBudget / per) > 0 ? (int64_t)(kWsBudget / per) : 1;
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  if (want > c->wsgroups) {
    if (c->wsbuf) (void)hipFree(c->wsbuf);
    c->wsbuf = nullptr;
    c->wsgroups = 0;
    hipError_t e = hipMalloc(&c->wsbuf, per * (size_t)want);
    if (e != hipSuccess) {
      c->err = std::string("workspace hipMalloc: ") + hipGetErrorString(e);
      return HMPC_ERR_NOMEM;
    }
    c->wsgroups = (int)want;
  }
  a.ws = c->wsbuf;
  a.ws_stride = Lw.total;
  a.ws_groups = c->wsgroups;
  return HMPC_OK;
}

// Overflow pass geometry: workgroups (each with an R block of capacity 6N and
// a K / Dinv workspace in global memory) looping over the instances whose
// active set outgrew the main kernel's capacity.
constexpr int kOvfGroups = 128;
// ints before the overflow list in the counter buffer (see hmpc_ctx::ovf)
constexpr int kOvfHeader = 16;

// Longest-first order (stance-stage buckets, most stance stages first; the
// dense split's class lists and the Riccati kernel's work queue) pays where
// the batch is a few instances per resident wave, so the instances that start
// last set the step time.  Interleaved A/B (profiles/r04_ab.json): dense
// configs[1] (B = 4096) 19.9 -> 24.1 M solves/s, B = 16384 -1.7 %, configs[2]
// (B = 65536) -0.4 %; Riccati N = 60 at 4 instances per workgroup 1.30 ->
// 1.46 M, configs[3] at 128 per workgroup -6 %.
constexpr int64_t kDenseLptMaxB = 8192;
constexpr int64_t kRicLptPerGroup = 8;
bool longest_first(const hmpc_ctx* c, int64_t B) {
  if (c->order == HMPC_ORDER_INDEX) return false;
  if (c->order == HMPC_ORDER_LONGEST_FIRST) return true;
  if (hmpc::pick_kernel(c->variant, c->N, c->precision) == hmpc::Kernel::Riccati)   // (at most one
    // instance per resident workgroup: all start at once, the order is moot and
    // the bucket pass would be pure latency -- the Runner's B = 1)
    return B > (int64_t)c->ric_groups && B <= kRicLptPerGroup * (int64_t)c->ric_groups;
  return B <= kDenseLptMaxB;
}

// The context's second stream and its fork / join events (the dense split's
// concurrent class).
int ensure_fork(hmpc_ctx* c) {
  if (c->split_stream) return HMPC_OK;
  if (hipStreamCreateWithFlags(&c->split_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->split_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->split_join, hipEventDisableTiming) != hipSuccess) {
    c->err = "split stream / events";
    return HMPC_ERR_HIP;
  }
  return HMPC_OK;
}

// The class / bucket lists: nlist lists of B entries (grow-only).
int ensure_split(hmpc_ctx* c, int64_t B, int nlist, const char* what) {
  if (B <= c->split_cap && nlist <= c->split_nbuf) return HMPC_OK;
  if (c->split) (void)hipFree(c->split);
  c->split = nullptr;
  const int64_t cap = B > c->split_cap ? B : c->split_cap;
  const int nb = nlist > c->split_nbuf ? nlist : c->split_nbuf;
  c->split_cap = 0;
  c->split_nbuf = 0;
  hipError_t e = hipMalloc(&c->split, sizeof(int32_t) * (size_t)nb * (size_t)cap);
  if (e != hipSuccess) { c->split = nullptr; c->err = what; return HMPC_ERR_NOMEM; }
  c->split_cap = cap;
  c->split_nbuf = nb;
  return HMPC_OK;
}

// Buffers of the dense / Riccati kernels: [overflow count | instance counter |
// pad | overflow list], the overflow pass's blocks, the Riccati kernel's
// per-workgroup K / Dinv workspace.
int prepare_ric(hmpc_ctx* c, int64_t B, hmpc::SolveArgs& a) {
  const hmpc::Kernel k = hmpc::pick_kernel(c->variant, c->N, c->precision);
  a.ovf_count = nullptr; a.ovf_list = nullptr; a.rws = nullptr; a.rws_stride = 0;
  a.work = nullptr; a.work_bound = nullptr; a.kws = nullptr; a.kws_stride = 0; a.ric_groups = 0;
  a.kinst = nullptr; a.kinst_stride = 0;
  a.split_count = nullptr; a.split_list = nullptr;
  if (k == hmpc::Kernel::Cas) {   // instance counter + R slots, no overflow pass
    if (!c->ovf) {
      hipError_t e = hipMalloc(&c->ovf, sizeof(int32_t) * 4);
      if (e != hipSuccess) { c->err = "counter hipMalloc"; return HMPC_ERR_NOMEM; }
      c->ovf_cap = 0;
    }
    if (c->ric_groups == 0) {
      const int g = hmpc::cas_groups(c->N);
      if (g < 1) { c->err = "CasADi-variant kernel occupancy query"; return HMPC_ERR_HIP; }
      hipError_t e = hipMalloc(&c->kws, sizeof(double) * hmpc::cas_ws_stride(c->N) * g);
      if (e != hipSuccess) { c->kws = nullptr; c->err = "CasADi-variant workspace hipMalloc"; return HMPC_ERR_NOMEM; }
      c->ric_groups = g;
    }
    a.work = c->ovf + 1;
    a.kws = c->kws;
    a.kws_stride = hmpc::cas_ws_stride(c->N);
    a.ric_groups = c->ric_groups;
    return HMPC_OK;
  }
  // (the fp32 dense build hands its overflows to the same fp64 pass)
  if ((k != hmpc::Kernel::Dense && k != hmpc::Kernel::DenseF32 && k != hmpc::Kernel::DenseF32R &&
       k != hmpc::Kernel::Riccati) ||
      c->N > hmpc::kRicNmax)
    return HMPC_OK;
  const int64_t rstride = hmpc::ric_rws_stride(c->N);
  if (!c->rws) {
    hipError_t e = hipMalloc(&c->rws, sizeof(double) * rstride * kOvfGroups);
    if (e != hipSuccess) { c->rws = nullptr; c->err = "overflow workspace hipMalloc"; return HMPC_ERR_NOMEM; }
  }
  if (B > c->ovf_cap) {
    if (c->ovf) (void)hipFree(c->ovf);
    c->ovf = nullptr;
    c->ovf_cap = 0;
    // [header | list of B] twice: the second pair serves the generic pass
    // behind HMPC_PREC_F32_REFINED's fp64 dense fallback pass (run_solve)
    hipError_t e = hipMalloc(&c->ovf, sizeof(int32_t) * 2 * (size_t)(B + kOvfHeader));
    if (e != hipSuccess) { c->err = "overflow list hipMalloc"; return HMPC_ERR_NOMEM; }
    c->ovf_cap = B;
    c->ovf_dirty = true;
    c->ovf2_zeroed = false;
  }
  a.ovf_count = c->ovf;
  a.work = c->ovf + 1;
  a.ovf_list = c->ovf + kOvfHeader;
  if (!c->ovf_total && !c->ovf_total_failed) {
    // a diagnostic counter: zeroed and synchronised once at allocation (the
    // null-stream memset is then ordered before any solve stream's kernel),
    // and a failed allocation leaves it unavailable rather than failing the
    // solve
    if (hipMalloc(&c->ovf_total, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->ovf_total, 0, sizeof(unsigned long long)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
      if (c->ovf_total) (void)hipFree(c->ovf_total);
      c->ovf_total = nullptr;
      c->ovf_total_failed = true;
    }
  }
  a.ovf_total = c->ovf_total;
  // the dense kernel's split launch (compacted kernel for the instances with
  // few free variables): class counts next to the overflow counters, which
  // the overflow pass zeroes together at its end
  const bool split = (k == hmpc::Kernel::Dense && hmpc::dense_split_nv(c->N, 0) > 0) ||
                     (k == hmpc::Kernel::DenseF32 && hmpc::dense_split_nv(c->N, 1) > 0) ||
                     (k == hmpc::Kernel::DenseF32R && hmpc::dense_split_nv(c->N, 2) > 0);
  if (split && c->N + 1 <= kOvfHeader - 3) {
    // (up to N + 1 stance-count buckets of B entries -- longest-first order --
    // or the three class lists)
    int rc = ensure_split(c, B, c->N + 1 > 3 ? c->N + 1 : 3, "split list hipMalloc");
    if (rc != HMPC_OK) return rc;
    rc = ensure_fork(c);
    if (rc != HMPC_OK) return rc;
    a.split_count = c->ovf + 3;
    a.split_list = c->split;
    a.split_nbkt = c->N + 1;
    a.lpt = longest_first(c, B) ? 1 : 0;
    c->dense_lpt = a.lpt != 0;
    a.split_stream = c->split_stream;
    a.split_fork = c->split_fork;
    a.split_join = c->split_join;
  }
  a.rws = c->rws;
  a.rws_stride = rstride;
  if (k == hmpc::Kernel::Riccati) {
    if (c->ric_groups == 0) {
      const int g = hmpc::ric_groups(c->variant, c->N);
      if (g < 1) { c->err = "Riccati kernel occupancy query"; return HMPC_ERR_HIP; }
      hipError_t e = hipMalloc(&c->kws, sizeof(double) * hmpc::ric_kws_stride(c->N) * g);
      if (e != hipSuccess) { c->kws = nullptr; c->err = "Riccati workspace hipMalloc"; return HMPC_ERR_NOMEM; }
      c->ric_groups = g;
    }
    a.kws = c->kws;
    a.kws_stride = hmpc::ric_kws_stride(c->N);
    a.ric_groups = c->ric_groups;
    // the factorisation kernel's per-instance K / Dinv blocks (a speed-up
    // only: without the memory the solve kernel factorises itself)
    const int64_t ks = hmpc::ric_kinst_stride(c->N, B);
    if (ks > 0) {
      if (B > c->kinst_cap) {
        if (c->kinst) (void)hipFree(c->kinst);
        c->kinst = nullptr;
        c->kinst_cap = 0;
        if (hipMalloc(&c->kinst, sizeof(double) * (size_t)ks * (size_t)B) == hipSuccess) c->kinst_cap = B;
        else { c->kinst = nullptr; (void)hipGetLastError(); }
      }
      if (c->kinst) {
        a.kinst = c->kinst;
        a.kinst_stride = ks;
      }
    }
    c->ric_fused = hmpc::ric_occ(c->N) == 1 && a.kinst == nullptr;
    c->ric_cap_last = a.kinst ? hmpc::ric_qcap_batch(c->N, B) : hmpc::ric_qcap(c->N);
    // the longest-first work queue: stance-count buckets (<= 13 counters in
    // the overflow header), lists of B entries each
    const int nb = hmpc::ric_lpt_buckets(c->N);
    a.lpt = 0;
    if (longest_first(c, B) && nb > 0 && nb <= kOvfHeader - 3) {
      int rc = ensure_split(c, B, nb, "work-queue bucket hipMalloc");   // (nb <= 13 lists, not N + 1)
      if (rc != HMPC_OK) return rc;
      a.split_count = c->ovf + 3;
      a.split_list = c->split;
      a.split_nbkt = nb;
      a.lpt = 1;
    }
  }
  return HMPC_OK;
}

// The second overflow header and list (run_solve: HMPC_PREC_F32_REFINED's
// fp64 fallback pass, the N = 60 second tier)
int32_t* ovf_hdr2(hmpc_ctx* c) { return c->ovf + kOvfHeader + c->ovf_cap; }

// One solve pass over the batch: the main kernel, then (dense / Riccati
// kernels) the overflow pass over the instances it handed on.  Stream-ordered.
// HMPC_PREC_F32_REFINED hands on the instances its fp64 check rejected
// (0.6 % of configs[4]): they are re-solved first by the fp64 dense kernel
// over that list (its full class: the dense kernel's speed), and only what
// outgrows that kernel's capacity goes on to the generic capacity-6N pass,
// through the second header and list.
int run_solve(hmpc_ctx* c, hmpc::SolveArgs a, hipStream_t s) {
  int rc = prepare_ws(c, a.B, a);
  if (rc != HMPC_OK) return rc;
  rc = prepare_ric(c, a.B, a);
  if (rc != HMPC_OK) return rc;
  // [overflow count | instance counter | overflow-pass done counter | split
  // counts]: zeroed here only when dirty -- the overflow pass, which follows
  // every main pass that has one, zeroes them at its end (stream order: the
  // next solve's kernels see them zero).  The CasADi kernel has no overflow
  // pass.
  const hmpc::Kernel kk = hmpc::pick_kernel(c->variant, c->N, c->precision);
  const bool fb = a.ovf_count && kk == hmpc::Kernel::DenseF32R;
  // N = 60 at the large-batch capacity: the capacity-64 kernel takes the
  // overflow list first (the Runner's robots share their 48-59-row calls)
  const bool t2 = a.ovf_count && kk == hmpc::Kernel::Riccati && a.kinst && hmpc::ric_has_tier2(c->N, a.B);
  if (a.work && (!a.ovf_count || c->ovf_dirty)) {
    hipError_t e = hipMemsetAsync(a.work - 1, 0, (a.ovf_count ? kOvfHeader : 3) * sizeof(int32_t), s);
    if (e != hipSuccess) return fail_hip(c, e, "hipMemsetAsync(overflow count)");
  }
  if ((fb || t2) && (!c->ovf2_zeroed || c->ovf_dirty)) {   // (the generic pass zeroes it at its end)
    hipError_t e = hipMemsetAsync(ovf_hdr2(c), 0, kOvfHeader * sizeof(int32_t), s);
    if (e != hipSuccess) return fail_hip(c, e, "hipMemsetAsync(second overflow count)");
    c->ovf2_zeroed = true;
  }
  c->ovf_dirty = true;   // until the overflow pass is launched
  if (!hmpc::launch_solve(c->variant, c->N, a, s)) {
    c->err = "no kernel for this (variant, N, precision)";
    return HMPC_ERR_UNSUPPORTED;
  }
  if (fb) {
    hmpc::SolveArgs f = a;   // the fp64 dense kernel over the main pass's overflow list
    f.precision = HMPC_PREC_F64;
    f.list = a.ovf_list;
    f.list_count = a.ovf_count;
    f.lpt = 0;
    f.lpt_lo = 0;
    f.lpt_hi = -1;
    f.split_count = nullptr;
    f.split_list = nullptr;
    f.ovf_count = ovf_hdr2(c);
    f.ovf_list = ovf_hdr2(c) + kOvfHeader;
    if (!hmpc::launch_solve_fp64_list(c->variant, c->N, f, s)) {
      c->err = "fp64 fallback pass launch";
      return HMPC_ERR_UNSUPPORTED;
    }
    hmpc::SolveArgs o = a;   // the generic pass over what that kernel handed on
    o.ovf_count = f.ovf_count;
    o.ovf_list = f.ovf_list;
    o.ovf_hdr1 = a.ovf_count;
    if (!hmpc::launch_solve_ric_overflow(c->variant, c->N, o, kOvfGroups, s)) {
      c->err = "overflow pass launch";
      return HMPC_ERR_UNSUPPORTED;
    }
  } else if (t2) {
    hmpc::SolveArgs f = a;   // the capacity-64 solve kernel over the main pass's overflow list
    f.list = a.ovf_list;
    f.list_count = a.ovf_count;
    f.work_bound = a.ovf_count;
    f.split_nbkt = 1;
    f.lpt = 0;
    f.work = ovf_hdr2(c) + 1;
    f.ovf_count = ovf_hdr2(c);
    f.ovf_list = ovf_hdr2(c) + kOvfHeader;
    if (!hmpc::launch_solve_ric_tier2(c->variant, c->N, f, s)) {
      c->err = "second-tier pass launch";
      return HMPC_ERR_UNSUPPORTED;
    }
    hmpc::SolveArgs o = a;   // the generic pass over what that kernel handed on
    o.ovf_count = f.ovf_count;
    o.ovf_list = f.ovf_list;
    o.ovf_hdr1 = a.ovf_count;
    if (!hmpc::launch_solve_ric_overflow(c->variant, c->N, o, kOvfGroups, s)) {
      c->err = "overflow pass launch";
      return HMPC_ERR_UNSUPPORTED;
    }
  } else if (a.ovf_count && !hmpc::launch_solve_ric_overflow(c->variant, c->N, a, kOvfGroups, s)) {
    c->err = "overflow pass launch";
    return HMPC_ERR_UNSUPPORTED;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail_hip(c, e, "solve launch");
  c->ovf_dirty = a.ovf_count == nullptr;
  return HMPC_OK;
}

// Is s capturing a graph?  Work enqueued during a capture does not run then:
// its replays run whenever the caller launches them, outside the context's
// ordering (include/hmpc.h), so neither hook below touches a capture.
bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

// Before work on stream s: when the context's last eager call went to another
// stream, s waits for it (the context's workspaces and counters are shared by
// every stream).  The completion event is recorded on that stream here, at
// the switch -- it then covers everything enqueued there so far, the call
// included -- not after every call: an event record per solve is a marker
// packet between consecutive solves on one stream, 4 us of a 0.13 ms
// configs[1] step.  So the last call's stream must stay valid
// until the context's next call (include/hmpc.h).  Skipped while s captures:
// a wait on an event recorded outside the capture is not a graph edge, and
// mark_stream does not remember a capturing stream.
int order_stream(hmpc_ctx* c, hipStream_t s) {
  if (capturing(s)) return HMPC_OK;
  if (c->has_last && c->last_stream != s) {
    if (!c->last_ev) {
      hipError_t e = hipEventCreateWithFlags(&c->last_ev, hipEventDisableTiming);
      if (e != hipSuccess) return fail_hip(c, e, "hipEventCreate");
    }
    hipError_t e = hipEventRecord(c->last_ev, c->last_stream);
    if (e != hipSuccess) return fail_hip(c, e, "hipEventRecord(last call's stream)");
    e = hipStreamWaitEvent(s, c->last_ev, 0);
    if (e != hipSuccess) return fail_hip(c, e, "hipStreamWaitEvent(last call of this context)");
  }
  return HMPC_OK;
}

// After work on stream s: remember it (eager calls only; a replay of a
// captured call runs whenever the caller launches it)
int mark_stream(hmpc_ctx* c, hipStream_t s) {
  if (capturing(s)) return HMPC_OK;
  c->last_stream = s;
  c->has_last = true;
  return HMPC_OK;
}

__global__ void combine_status(int64_t B, const int32_t* s1, const int32_t* i1, int32_t* s2,
                               int32_t* i2) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  if (s1[i] > s2[i]) s2[i] = s1[i];
  if (i2) i2[i] += i1[i];
}

int check_solve_args(hmpc_ctx* c, int64_t B, const void* x_in, const void* x_lin,
                     const void* x_ref, const void* pf, const void* C, const void* u,
                     const void* status) {
  if (!c) return HMPC_ERR_ARG;
  if (B < 0) { c->err = "B < 0"; return HMPC_ERR_ARG; }
  if (B == 0) return HMPC_OK;
  if (B > 0x7fffffffLL) { c->err = "B exceeds the grid limit"; return HMPC_ERR_ARG; }
  if (!x_in || !x_lin || !x_ref || !pf || !C || !u || !status) {
    c->err = "null input/output pointer";
    return HMPC_ERR_ARG;
  }
  return HMPC_OK;
}

}  // namespace

extern "C" {

int hmpc_version(void) { return 10502; }

int hmpc_supported_horizons(int variant, int* Ns, int cap) {
  return hmpc::supported_horizons(variant, Ns, cap);
}

int hmpc_create(hmpc_ctx** out, int variant, int N, double t, double m, double g, double mu,
                const double* Jinv, const double* rh, int uref_mode, int device) {
  if (!out || !Jinv || !rh) return HMPC_ERR_ARG;
  *out = nullptr;
  if (variant != HMPC_VARIANT_3F && variant != HMPC_VARIANT_2F && variant != HMPC_VARIANT_CAS) return HMPC_ERR_ARG;
  if (uref_mode != HMPC_UREF_ALIASED && uref_mode != HMPC_UREF_PER_STAGE) return HMPC_ERR_ARG;
  if (!(t > 0.0) || !(m > 0.0) || N <= 0) return HMPC_ERR_ARG;
  if (!hmpc::horizon_supported(variant, N)) return HMPC_ERR_UNSUPPORTED;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return HMPC_ERR_HIP;
  hmpc_ctx* c = new (std::nothrow) hmpc_ctx();
  if (!c) return HMPC_ERR_NOMEM;
  c->variant = variant; c->N = N; c->device = device;
  c->t = t; c->m = m; c->g = g; c->mu = mu;
  memcpy(c->Jinv, Jinv, sizeof(c->Jinv));
  memcpy(c->rh, rh, sizeof(c->rh));
  c->uref_mode = uref_mode;
  *out = c;
  return HMPC_OK;
}

int hmpc_destroy(hmpc_ctx* c) {
  if (!c) return HMPC_ERR_ARG;
  (void)hipSetDevice(c->device);
  if (c->dbuf) (void)hipFree(c->dbuf);
  if (c->scratch_i32) (void)hipFree(c->scratch_i32);
  if (c->wsbuf) (void)hipFree(c->wsbuf);
  if (c->ovf) (void)hipFree(c->ovf);
  if (c->rws) (void)hipFree(c->rws);
  if (c->split) (void)hipFree(c->split);
  if (c->ovf_total) (void)hipFree(c->ovf_total);
  if (c->split_stream) (void)hipStreamDestroy(c->split_stream);
  if (c->split_fork) (void)hipEventDestroy(c->split_fork);
  if (c->split_join) (void)hipEventDestroy(c->split_join);
  if (c->kws) (void)hipFree(c->kws);
  if (c->kinst) (void)hipFree(c->kinst);
  if (c->plan_scratch) (void)hipFree(c->plan_scratch);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->last_ev) (void)hipEventDestroy(c->last_ev);
  delete c;
  return HMPC_OK;
}

const char* hmpc_last_error(hmpc_ctx* c) { return c ? c->err.c_str() : ""; }

int hmpc_overflow_total(hmpc_ctx* c, int64_t* total) {
  if (!c || !total) return HMPC_ERR_ARG;
  *total = 0;
  if (!c->ovf_total) return HMPC_OK;   // no solve with an overflow pass yet
  if (c->has_last) HMPC_HIP(c, hipStreamSynchronize(c->last_stream));
  unsigned long long v = 0;
  HMPC_HIP(c, hipMemcpy(&v, c->ovf_total, sizeof v, hipMemcpyDeviceToHost));
  *total = (int64_t)v;
  return HMPC_OK;
}

int hmpc_active_capacity(hmpc_ctx* c) {
  if (!c) return -1;
  switch (hmpc::pick_kernel(c->variant, c->N, c->precision)) {
    case hmpc::Kernel::Dense:
      return hmpc::dense_qmax(c->N, 0);
    case hmpc::Kernel::DenseF32:
      return hmpc::dense_qmax(c->N, 1);
    case hmpc::Kernel::DenseF32R:
      return hmpc::dense_qmax(c->N, 2);
    case hmpc::Kernel::Riccati:   // (of the last solve: N = 60 small batches run capacity 64)
      return c->ric_cap_last ? c->ric_cap_last : hmpc::ric_qcap(c->N);
    case hmpc::Kernel::Cas:
      return 18 * c->N;
    case hmpc::Kernel::Wide:
      return 0;
    default:
      return -1;
  }
}

const char* hmpc_kernel_name(hmpc_ctx* c) {
  if (!c) return "";
  const bool v3 = c->variant == HMPC_VARIANT_3F;
  switch (hmpc::pick_kernel(c->variant, c->N, c->precision)) {
    case hmpc::Kernel::Dense: {
      // (the classes of the last solve: in longest-first order the all-swing
      // windows stay in the compacted class)
      const char* n = hmpc::dense_name(c->variant, c->N, 0);
      const char* rest = strstr(n, " + ");
      if (c->dense_lpt && strncmp(n, "hmpc::swing_kernel", 18) == 0 && rest) return rest + 3;
      return n;
    }
    case hmpc::Kernel::DenseF32:
      return hmpc::dense_name(c->variant, c->N, 1);
    case hmpc::Kernel::DenseF32R:
      return hmpc::dense_name(c->variant, c->N, 2);
    case hmpc::Kernel::Cas:
      return "hmpc::cas_kernel";
    case hmpc::Kernel::Riccati:
      // (template arguments as rocprofv3 demangles them: variant, occupancy,
      // compile-time horizon and capacity, 0 = runtime, part; the one-wave
      // horizons run the factorisation kernel first -- for batches within its
      // buffer bound, hmpc_ric.hip ric_kinst_stride; the fused kernel when
      // the context's last solve was beyond it)
      if (hmpc::ric_occ(c->N) == 2) {
        if (hmpc::ric_static_n(c->N) == 20) return v3 ? "hmpc::ric_kernel<3, 2, 20, 38, 0>" : "hmpc::ric_kernel<2, 2, 20, 38, 0>";
        return v3 ? "hmpc::ric_kernel<3, 2, 0, 0, 0>" : "hmpc::ric_kernel<2, 2, 0, 0, 0>";
      }
      if (c->ric_fused) {   // the last solve's batch was beyond the K / Dinv buffer bound
        if (hmpc::ric_static_n(c->N) == 60) return v3 ? "hmpc::ric_kernel<3, 1, 60, 47, 0>" : "hmpc::ric_kernel<2, 1, 60, 47, 0>";
        return v3 ? "hmpc::ric_kernel<3, 1, 0, 0, 0>" : "hmpc::ric_kernel<2, 1, 0, 0, 0>";
      }
      if (hmpc::ric_static_n(c->N) == 60 && c->ric_cap_last == 64)   // the last solve's small batch
        return v3 ? "hmpc::ric_factor_kernel<3, 60, 47> + hmpc::ric_kernel<3, 1, 60, 64, 2>"
                  : "hmpc::ric_factor_kernel<2, 60, 47> + hmpc::ric_kernel<2, 1, 60, 64, 2>";
      if (hmpc::ric_static_n(c->N) == 60)
        return v3 ? "hmpc::ric_factor_kernel<3, 60, 47> + hmpc::ric_kernel<3, 1, 60, 47, 2>"
                  : "hmpc::ric_factor_kernel<2, 60, 47> + hmpc::ric_kernel<2, 1, 60, 47, 2>";
      return v3 ? "hmpc::ric_factor_kernel<3, 0, 0> + hmpc::ric_kernel<3, 1, 0, 0, 2>"
                : "hmpc::ric_factor_kernel<2, 0, 0> + hmpc::ric_kernel<2, 1, 0, 0, 2>";
    case hmpc::Kernel::Wide:
      if (c->precision == HMPC_PREC_F32 || c->precision == HMPC_PREC_F32_GENERIC)
        return v3 ? "hmpc::wide_kernel<3, float>" : "hmpc::wide_kernel<2, float>";
      return v3 ? "hmpc::wide_kernel<3, double>" : "hmpc::wide_kernel<2, double>";
    default:
      return "";
  }
}

int hmpc_set_precision(hmpc_ctx* c, int precision) {
  if (!c) return HMPC_ERR_ARG;
  if (precision != HMPC_PREC_F64 && precision != HMPC_PREC_F32 && precision != HMPC_PREC_F64_GENERIC &&
      precision != HMPC_PREC_F64_RICCATI && precision != HMPC_PREC_F64_DENSE &&
      precision != HMPC_PREC_F32_GENERIC && precision != HMPC_PREC_F32_REFINED) {
    c->err = "unknown precision";
    return HMPC_ERR_ARG;
  }
  if (hmpc::pick_kernel(c->variant, c->N, precision) == hmpc::Kernel::None) {
    c->err = "no kernel for this (variant, N) at that precision";
    return HMPC_ERR_UNSUPPORTED;
  }
  c->precision = precision;
  return HMPC_OK;
}

int hmpc_set_order(hmpc_ctx* c, int order) {
  if (!c) return HMPC_ERR_ARG;
  if (order != HMPC_ORDER_AUTO && order != HMPC_ORDER_INDEX && order != HMPC_ORDER_LONGEST_FIRST) {
    c->err = "order must be HMPC_ORDER_AUTO, _INDEX or _LONGEST_FIRST";
    return HMPC_ERR_ARG;
  }
  c->order = order;
  return HMPC_OK;
}

int hmpc_set_refinement(hmpc_ctx* c, int corrections) {
  if (!c) return HMPC_ERR_ARG;
  if (corrections < 0 || corrections > 16) {
    c->err = "corrections outside [0, 16]";
    return HMPC_ERR_ARG;
  }
  c->refine = corrections;
  return HMPC_OK;
}

int hmpc_solve_batch_stats(hmpc_ctx* c, int64_t B, const double* x_in, const double* x_lin,
                           const double* x_ref, const double* pf, const double* C, const double* mu,
                           double* u, double* x, double* obj, int32_t* status, int32_t* iters,
                           int32_t* active, void* stream) {
  int rc = check_solve_args(c, B, x_in, x_lin, x_ref, pf, C, u, status);
  if (rc != HMPC_OK || B == 0) return rc;
  HMPC_HIP(c, hipSetDevice(c->device));
  hmpc::SolveArgs a = make_args(c, B, x_in, x_lin, x_ref, pf, C, mu, u, x, obj, status, iters, 0);
  a.active = active;
  if ((rc = order_stream(c, (hipStream_t)stream)) != HMPC_OK) return rc;
  if ((rc = run_solve(c, a, (hipStream_t)stream)) != HMPC_OK) return rc;
  return mark_stream(c, (hipStream_t)stream);
}

int hmpc_solve_batch(hmpc_ctx* c, int64_t B, const double* x_in, const double* x_lin,
                     const double* x_ref, const double* pf, const double* C, const double* mu,
                     double* u, double* x, double* obj, int32_t* status, int32_t* iters,
                     void* stream) {
  return hmpc_solve_batch_stats(c, B, x_in, x_lin, x_ref, pf, C, mu, u, x, obj, status, iters, nullptr,
                                stream);
}

int hmpc_time_solve_batch(hmpc_ctx* c, int64_t B, const double* x_in, const double* x_lin,
                          const double* x_ref, const double* pf, const double* C,
                          const double* mu, double* u, double* x, double* obj, int32_t* status,
                          int32_t* iters, int reps, void* stream, double* ms) {
  int rc = check_solve_args(c, B, x_in, x_lin, x_ref, pf, C, u, status);
  if (rc != HMPC_OK) return rc;
  if (reps <= 0 || !ms || B == 0) { c->err = "reps <= 0, ms == NULL or B == 0"; return HMPC_ERR_ARG; }
  HMPC_HIP(c, hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  hmpc::SolveArgs a = make_args(c, B, x_in, x_lin, x_ref, pf, C, mu, u, x, obj, status, iters, 0);
  if ((rc = order_stream(c, s)) != HMPC_OK) return rc;
  rc = run_solve(c, a, s);   // validates the combination and sizes the workspaces
  if (rc != HMPC_OK) return rc;
  struct Ev {   // destroyed on every exit path
    hipEvent_t e = nullptr;
    ~Ev() { if (e) (void)hipEventDestroy(e); }
  } e0, e1;
  HMPC_HIP(c, hipEventCreate(&e0.e));
  HMPC_HIP(c, hipEventCreate(&e1.e));
  HMPC_HIP(c, hipEventRecord(e0.e, s));
  for (int r = 0; r < reps; ++r) {
    rc = run_solve(c, a, s);
    if (rc != HMPC_OK) return rc;
  }
  HMPC_HIP(c, hipEventRecord(e1.e, s));
  if ((rc = mark_stream(c, s)) != HMPC_OK) return rc;
  HMPC_HIP(c, hipEventSynchronize(e1.e));
  float t = 0.f;
  HMPC_HIP(c, hipEventElapsedTime(&t, e0.e, e1.e));
  *ms = (double)t / reps;
  return HMPC_OK;
}

int hmpc_solve_batch_host(hmpc_ctx* c, int64_t B, const double* x_in, const double* x_lin,
                          const double* x_ref, const double* pf, const double* C,
                          const double* mu, double* u, double* x, double* obj, int32_t* status,
                          int32_t* iters) {
  int rc = check_solve_args(c, B, x_in, x_lin, x_ref, pf, C, u, status);
  if (rc != HMPC_OK || B == 0) return rc;
  HMPC_HIP(c, hipSetDevice(c->device));
  const int N = c->N;
  const size_t nd_in = 12 + 12 * (N + 1) + 12 * N + 3 * N + N + 1;
  const size_t nd_out = 6 * N + 12 * (N + 1) + 1;
  const size_t bytes = (size_t)B * (8 * (nd_in + nd_out) + 8) + 256;
  if (bytes > c->dbuf_bytes) {
    if (c->dbuf) (void)hipFree(c->dbuf);
    c->dbuf = nullptr;
    c->dbuf_bytes = 0;
    HMPC_HIP(c, hipMalloc(&c->dbuf, bytes));
    c->dbuf_bytes = bytes;
  }
  if (!c->own_stream) HMPC_HIP(c, hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
  hipStream_t s = c->own_stream;
  // the context's workspaces are shared with the device entry points, which
  // run on the caller's streams: drain the device first (this entry point is
  // synchronous anyway)
  HMPC_HIP(c, hipDeviceSynchronize());
  double* p = (double*)c->dbuf;
  double* d_xin = p; p += B * 12;
  double* d_xlin = p; p += B * 12 * (N + 1);
  double* d_xref = p; p += B * 12 * N;
  double* d_pf = p; p += B * 3 * N;
  double* d_C = p; p += B * N;
  double* d_mu = p; p += B;
  double* d_u = p; p += B * 6 * N;
  double* d_x = p; p += B * 12 * (N + 1);
  double* d_obj = p; p += B;
  int32_t* d_st = (int32_t*)p;
  int32_t* d_it = d_st + B;
  HMPC_HIP(c, hipMemcpyAsync(d_xin, x_in, 8 * B * 12, hipMemcpyHostToDevice, s));
  HMPC_HIP(c, hipMemcpyAsync(d_xlin, x_lin, 8 * B * 12 * (N + 1), hipMemcpyHostToDevice, s));
  HMPC_HIP(c, hipMemcpyAsync(d_xref, x_ref, 8 * B * 12 * N, hipMemcpyHostToDevice, s));
  HMPC_HIP(c, hipMemcpyAsync(d_pf, pf, 8 * B * 3 * N, hipMemcpyHostToDevice, s));
  HMPC_HIP(c, hipMemcpyAsync(d_C, C, 8 * B * N, hipMemcpyHostToDevice, s));
  if (mu) HMPC_HIP(c, hipMemcpyAsync(d_mu, mu, 8 * B, hipMemcpyHostToDevice, s));
  hmpc::SolveArgs a = make_args(c, B, d_xin, d_xlin, d_xref, d_pf, d_C, mu ? d_mu : nullptr,
                                d_u, d_x, d_obj, d_st, d_it, 0);
  rc = run_solve(c, a, s);
  if (rc != HMPC_OK) return rc;
  HMPC_HIP(c, hipMemcpyAsync(u, d_u, 8 * B * 6 * N, hipMemcpyDeviceToHost, s));
  if (x) HMPC_HIP(c, hipMemcpyAsync(x, d_x, 8 * B * 12 * (N + 1), hipMemcpyDeviceToHost, s));
  if (obj) HMPC_HIP(c, hipMemcpyAsync(obj, d_obj, 8 * B, hipMemcpyDeviceToHost, s));
  HMPC_HIP(c, hipMemcpyAsync(status, d_st, 4 * B, hipMemcpyDeviceToHost, s));
  if (iters) HMPC_HIP(c, hipMemcpyAsync(iters, d_it, 4 * B, hipMemcpyDeviceToHost, s));
  HMPC_HIP(c, hipStreamSynchronize(s));
  c->has_last = false;   // drained: nothing of this context is in flight
  return HMPC_OK;
}

namespace {

// Mpc.mpcontrol (src/mpc_cvx_euler_3f.py:41-69) for B instances; `view`
// carries the x_ref / pf / C strides (contiguous or a resident plan).
int mpcontrol_impl(hmpc_ctx* c, int64_t B, int init, const double* x_in, const double* x_ref,
                   const double* pf, const double* C, const double* mu, double* x_prev,
                   double* u, double* obj, int32_t* status, int32_t* iters, void* stream,
                   const hmpc::SolveArgs* view) {
  if (c->variant == HMPC_VARIANT_CAS) {   // its mpcontrol has no init / time shift (cas :112)
    c->err = "mpcontrol: the CasADi variant solves one QP per call (hmpc_solve_batch)";
    return HMPC_ERR_UNSUPPORTED;
  }
  HMPC_HIP(c, hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  int rc = order_stream(c, s);
  if (rc != HMPC_OK) return rc;
  auto args = [&](int32_t* st, int32_t* it, double* ob, int mode) {
    hmpc::SolveArgs a = make_args(c, B, x_in, x_prev, x_ref, pf, C, mu, u, x_prev, ob, st, it, mode);
    if (view) {
      a.xref_bs = view->xref_bs; a.xref_rs = view->xref_rs;
      a.pf_bs = view->pf_bs; a.pf_rs = view->pf_rs;
      a.C_bs = view->C_bs;
    }
    return a;
  };
  if (init) {
    if (B > c->scratch_n) {
      if (c->scratch_i32) (void)hipFree(c->scratch_i32);
      c->scratch_i32 = nullptr;
      c->scratch_n = 0;
      HMPC_HIP(c, hipMalloc(&c->scratch_i32, 8 * B));
      c->scratch_n = B;
    }
    int32_t* s1 = c->scratch_i32;
    int32_t* i1 = c->scratch_i32 + B;
    // pass 1: linearise about [x_in; x_ref]  (src/mpc_cvx_euler_3f.py:50-58)
    if ((rc = run_solve(c, args(s1, i1, nullptr, 1), s)) != HMPC_OK) return rc;
    // pass 2: linearise about x* of pass 1 (in place: each workgroup reads
    // its x_lin before writing x*)
    if ((rc = run_solve(c, args(status, iters, obj, 0), s)) != HMPC_OK) return rc;
    const int tpb = 256;
    hipLaunchKernelGGL(combine_status, dim3((unsigned)((B + tpb - 1) / tpb)), dim3(tpb), 0, s, B,
                       s1, i1, status, iters);
  } else {
    // time shift of the previous x*  (src/mpc_cvx_euler_3f.py:59-62)
    if ((rc = run_solve(c, args(status, iters, obj, 2), s)) != HMPC_OK) return rc;
  }
  HMPC_HIP(c, hipGetLastError());
  return mark_stream(c, s);
}

}  // namespace

int hmpc_mpcontrol_batch(hmpc_ctx* c, int64_t B, int init, const double* x_in,
                         const double* x_ref, const double* pf, const double* C,
                         const double* mu, double* x_prev, double* u, double* obj,
                         int32_t* status, int32_t* iters, void* stream) {
  int rc = check_solve_args(c, B, x_in, x_prev, x_ref, pf, C, u, status);
  if (rc != HMPC_OK || B == 0) return rc;
  return mpcontrol_impl(c, B, init, x_in, x_ref, pf, C, mu, x_prev, u, obj, status, iters, stream,
                        nullptr);
}

int hmpc_mpcontrol_plan_batch(hmpc_ctx* c, int64_t B, int init, const double* x_in,
                              const double* x_ref_plan, const double* pf_plan, int64_t T,
                              int64_t plan_bstride, int64_t k, int mpc_factor, const double* C,
                              int64_t C_bstride, const double* mu, double* x_prev, double* u,
                              double* obj, int32_t* status, int32_t* iters, void* stream) {
  int rc = check_solve_args(c, B, x_in, x_prev, x_ref_plan, pf_plan, C, u, status);
  if (rc != HMPC_OK || B == 0) return rc;
  const int N = c->N;
  if (mpc_factor <= 0 || k < 0 || T <= 0 || k + (int64_t)(N - 1) * mpc_factor >= T) {
    c->err = "plan window k + (N-1)*mpc_factor outside [0, T)";
    return HMPC_ERR_ARG;
  }
  if (plan_bstride != 0 && plan_bstride < T) {
    c->err = "plan_bstride must be 0 (shared plan) or >= T";
    return HMPC_ERR_ARG;
  }
  if (C_bstride != 0 && C_bstride < N) {
    c->err = "C_bstride must be 0 (shared schedule) or >= N";
    return HMPC_ERR_ARG;
  }
  if ((int64_t)mpc_factor * 12 > 0x7fffffff / 2) { c->err = "mpc_factor too large"; return HMPC_ERR_ARG; }
  hmpc::SolveArgs view;
  view.xref_bs = 12 * plan_bstride; view.xref_rs = 12 * mpc_factor;
  view.pf_bs = 3 * plan_bstride; view.pf_rs = 3 * mpc_factor;
  view.C_bs = C_bstride;
  return mpcontrol_impl(c, B, init, x_in, x_ref_plan + 12 * k, pf_plan + 3 * k, C, mu, x_prev, u,
                        obj, status, iters, stream, &view);
}

int hmpc_plant_batch(hmpc_ctx* c, int64_t B, int n_steps, double dt, const double* J, double* X,
                     const double* U, int64_t U_bstride, const double* pf, int64_t pf_bstride,
                     int64_t pf_sstride, double* X_hist, double* x_out, void* stream) {
  if (!c) return HMPC_ERR_ARG;
  if (B < 0 || n_steps < 0 || !(dt > 0.0)) { c->err = "B < 0, n_steps < 0 or dt <= 0"; return HMPC_ERR_ARG; }
  if (B == 0) return HMPC_OK;
  if (!J || !X || !U || !pf) { c->err = "null pointer"; return HMPC_ERR_ARG; }
  if (U_bstride < 0 || pf_bstride < 0 || pf_sstride < 0) { c->err = "negative stride"; return HMPC_ERR_ARG; }
  HMPC_HIP(c, hipSetDevice(c->device));
  hmpc::PlantArgs a;
  a.B = B; a.n_steps = n_steps; a.dt = dt; a.m = c->m; a.g = c->g;
  memcpy(a.J, J, sizeof(a.J));
  memcpy(a.Jinv, c->Jinv, sizeof(a.Jinv));
  memcpy(a.rh, c->rh, sizeof(a.rh));
  a.X = X; a.U = U; a.U_bs = U_bstride;
  a.pf = pf; a.pf_bs = pf_bstride; a.pf_ss = pf_sstride;
  a.X_hist = X_hist; a.x_out = x_out;
  hmpc::launch_plant(a, (hipStream_t)stream);
  HMPC_HIP(c, hipGetLastError());
  return HMPC_OK;
}

int hmpc_convert_batch(hmpc_ctx* c, int64_t B, const double* X, double* x, void* stream) {
  if (!c) return HMPC_ERR_ARG;
  if (B < 0) { c->err = "B < 0"; return HMPC_ERR_ARG; }
  if (B == 0) return HMPC_OK;
  if (!X || !x) { c->err = "null pointer"; return HMPC_ERR_ARG; }
  HMPC_HIP(c, hipSetDevice(c->device));
  hmpc::launch_convert(B, X, x, (hipStream_t)stream);
  HMPC_HIP(c, hipGetLastError());
  return HMPC_OK;
}

int hmpc_plan_batch(hmpc_ctx* c, int64_t B, int N_run, int N_k, double dt, int curve, double t_p,
                    double phi_switch, double t_start, int step_adjustment, const double* x_in,
                    const double* xf, double* x_ref, double* pf_ref, double* C_map, void* stream) {
  if (!c) return HMPC_ERR_ARG;
  if (B < 0 || N_run < 2 || N_k < 0 || !(dt > 0.0) || !(t_p > 0.0)) {
    c->err = "B < 0, N_run < 2, N_k < 0, dt <= 0 or t_p <= 0";
    return HMPC_ERR_ARG;
  }
  if (B == 0) return HMPC_OK;
  if (!x_in || !xf || !x_ref || !pf_ref) { c->err = "null pointer"; return HMPC_ERR_ARG; }
  HMPC_HIP(c, hipSetDevice(c->device));
  const int64_t need = hmpc::plan_scratch_bytes(B, N_run + N_k);
  if (need > c->plan_scratch_bytes) {
    if (c->plan_scratch) (void)hipFree(c->plan_scratch);
    c->plan_scratch = nullptr;
    c->plan_scratch_bytes = 0;
    hipError_t e = hipMalloc(&c->plan_scratch, (size_t)need);
    if (e != hipSuccess) { c->err = "planner scratch hipMalloc"; return HMPC_ERR_NOMEM; }
    c->plan_scratch_bytes = need;
  }
  int rc = order_stream(c, (hipStream_t)stream);   // the planner scratch is per context
  if (rc != HMPC_OK) return rc;
  if (!hmpc::launch_plan(B, N_run, N_k, dt, curve, t_p, phi_switch, t_start, step_adjustment, x_in, xf,
                         x_ref, pf_ref, C_map, c->plan_scratch, (hipStream_t)stream)) {
    c->err = "planner launch";
    return HMPC_ERR_HIP;
  }
  HMPC_HIP(c, hipGetLastError());
  if ((rc = mark_stream(c, (hipStream_t)stream)) != HMPC_OK) return rc;
  // once per run, not per solve: wait for the plan and read its error word
  // (the reference raises IndexError in these cases: src/robotrunner.py:211-223)
  int32_t err = 0;
  HMPC_HIP(c, hipMemcpyAsync(&err, hmpc::plan_error_word(B, N_run + N_k, c->plan_scratch), sizeof(err),
                             hipMemcpyDeviceToHost, (hipStream_t)stream));
  HMPC_HIP(c, hipStreamSynchronize((hipStream_t)stream));
  if (err) {
    c->err = std::string("plan: ") + ((err & 1) ? "more footstep peaks than the device planner keeps (64); " : "") +
             ((err & 2) ? "peak + step_adjustment outside the plan (reference: IndexError); " : "") +
             ((err & 4) ? "footstep counter past the end of idx_pf (reference: IndexError)" : "");
    return HMPC_ERR_ARG;
  }
  return HMPC_OK;
}

int hmpc_gait_batch(hmpc_ctx* c, int n_steps, int mpc_factor, int N, double dt, double mpc_dt, double t_p,
                    double phi_switch, double t_start, double t0, double* C_calls, double* s_hist,
                    void* stream) {
  if (!c) return HMPC_ERR_ARG;
  if (n_steps < 0 || mpc_factor < 1 || N < 1 || !(dt > 0.0) || !(mpc_dt > 0.0) || !(t_p > 0.0)) {
    c->err = "n_steps < 0, mpc_factor < 1, N < 1 or a non-positive time";
    return HMPC_ERR_ARG;
  }
  if (n_steps == 0) return HMPC_OK;
  if (!C_calls) { c->err = "null pointer"; return HMPC_ERR_ARG; }
  HMPC_HIP(c, hipSetDevice(c->device));
  hmpc::launch_gait(n_steps, mpc_factor, N, dt, mpc_dt, t_p, phi_switch, t_start, t0, C_calls, s_hist,
                    (hipStream_t)stream);
  HMPC_HIP(c, hipGetLastError());
  return HMPC_OK;
}

}  // extern "C"
