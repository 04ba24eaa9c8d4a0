// Maps (variant, N, precision) onto a solve kernel:
//   * a dedicated one-/two-wavefront kernel (hmpc_kernels.hip, one object per
//     horizon in HMPC_HORIZON_LIST, see build.sh),
//   * the Riccati kernel (hmpc_ric.hip) for every other N <= kRicNmax,
//   * the generic dense kernel (hmpc_wide.hip) beyond that, and for the
//     fp32 / fp64-generic A/B precisions.
#include "hmpc_internal.h"

#ifndef HMPC_HORIZON_LIST
#define HMPC_HORIZON_LIST(X) X(5) X(10) X(20)
#endif
// horizons with an fp32 build of the dense kernel (launch_solve_n<N>_f32) and
// with an fp32 + fp64-refinement build (launch_solve_n<N>_f32r)
#ifndef HMPC_F32_LIST
#define HMPC_F32_LIST(X) X(10)
#endif
#ifndef HMPC_F32R_LIST
#define HMPC_F32R_LIST(X) X(10)
#endif

namespace hmpc {

#define HMPC_DECL(n)                                                       \
  bool launch_solve_n##n(int variant, const SolveArgs& a, hipStream_t s); \
  bool launch_list_n##n(int variant, const SolveArgs& a, hipStream_t s);  \
  int qmax_solve_n##n();                                                  \
  int split_nv_n##n();                                                    \
  const char* name_solve_n##n(int variant);
HMPC_HORIZON_LIST(HMPC_DECL)
#undef HMPC_DECL
#define HMPC_DECL(n)                                                           \
  bool launch_solve_n##n##_f32(int variant, const SolveArgs& a, hipStream_t s); \
  int qmax_solve_n##n##_f32();                                                  \
  int split_nv_n##n##_f32();                                                    \
  const char* name_solve_n##n##_f32(int variant);
HMPC_F32_LIST(HMPC_DECL)
#undef HMPC_DECL
#define HMPC_DECL(n)                                                            \
  bool launch_solve_n##n##_f32r(int variant, const SolveArgs& a, hipStream_t s); \
  int qmax_solve_n##n##_f32r();                                                  \
  int split_nv_n##n##_f32r();                                                    \
  const char* name_solve_n##n##_f32r(int variant);
HMPC_F32R_LIST(HMPC_DECL)
#undef HMPC_DECL

static bool f32_compiled(int variant, int N) {
  if (variant != 2 && variant != 3) return false;
#define HMPC_CASE(n) \
  if (N == n) return true;
  HMPC_F32_LIST(HMPC_CASE)
#undef HMPC_CASE
  return false;
}
static bool f32r_compiled(int variant, int N) {
  if (variant != 2 && variant != 3) return false;
#define HMPC_CASE(n) \
  if (N == n) return true;
  HMPC_F32R_LIST(HMPC_CASE)
#undef HMPC_CASE
  return false;
}

bool horizon_compiled(int variant, int N) {
  if (variant != 2 && variant != 3) return false;
#define HMPC_CASE(n) \
  if (N == n) return true;
  HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
  return false;
}

Kernel pick_kernel(int variant, int N, int precision) {
  if (variant == 4) return (precision == 0 && N >= 1 && N <= kCasNmax) ? Kernel::Cas : Kernel::None;
  if (variant != 2 && variant != 3 || N < 1) return Kernel::None;
  switch (precision) {
    case 1:
      if (f32_compiled(variant, N)) return Kernel::DenseF32;
      return N <= kWideNmax ? Kernel::Wide : Kernel::None;
    case 2:
    case 5:
      return N <= kWideNmax ? Kernel::Wide : Kernel::None;
    case 3:
      return N <= kRicNmax ? Kernel::Riccati : Kernel::None;
    case 6:
      return f32r_compiled(variant, N) ? Kernel::DenseF32R : Kernel::None;
    case 4:
      return horizon_compiled(variant, N) ? Kernel::Dense : Kernel::None;
    case 0:
      // the measured fastest: the one-wave dense kernel up to
      // N = 10, the Riccati kernel beyond (N = 20: 3.3 M vs 2.2 M solves/s)
      if (N <= kDenseNmax && horizon_compiled(variant, N)) return Kernel::Dense;
      if (N <= kRicNmax) return Kernel::Riccati;
      if (horizon_compiled(variant, N)) return Kernel::Dense;
      return N <= kWideNmax ? Kernel::Wide : Kernel::None;
    default:
      return Kernel::None;
  }
}

bool launch_solve_fp64_list(int variant, int N, const SolveArgs& a, hipStream_t s) {
  if (variant != 2 && variant != 3) return false;
#define HMPC_CASE(n) \
  if (N == n) return launch_list_n##n(variant, a, s);
  HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
  return false;
}

bool launch_solve(int variant, int N, const SolveArgs& a, hipStream_t s) {
  switch (pick_kernel(variant, N, a.precision)) {
    case Kernel::Dense:
#define HMPC_CASE(n) \
  if (N == n) return launch_solve_n##n(variant, a, s);
      HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
      return false;
    case Kernel::DenseF32:
#define HMPC_CASE(n) \
  if (N == n) return launch_solve_n##n##_f32(variant, a, s);
      HMPC_F32_LIST(HMPC_CASE)
#undef HMPC_CASE
      return false;
    case Kernel::DenseF32R:
#define HMPC_CASE(n) \
  if (N == n) return launch_solve_n##n##_f32r(variant, a, s);
      HMPC_F32R_LIST(HMPC_CASE)
#undef HMPC_CASE
      return false;
    case Kernel::Riccati:
      return launch_solve_ric(variant, N, a, s);
    case Kernel::Wide:
      return launch_solve_wide(variant, N, a, s);
    case Kernel::Cas:
      return launch_solve_cas(N, a, s);
    default:
      return false;
  }
}

int dense_qmax(int N, int flavor) {
  if (flavor == 2) {
#define HMPC_CASE(n) \
  if (N == n) return qmax_solve_n##n##_f32r();
    HMPC_F32R_LIST(HMPC_CASE)
#undef HMPC_CASE
    return -1;
  }
  if (flavor == 1) {
#define HMPC_CASE(n) \
  if (N == n) return qmax_solve_n##n##_f32();
    HMPC_F32_LIST(HMPC_CASE)
#undef HMPC_CASE
    return -1;
  }
#define HMPC_CASE(n) \
  if (N == n) return qmax_solve_n##n();
  HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
  return -1;
}

int dense_split_nv(int N, int flavor) {
  if (flavor == 2) {
#define HMPC_CASE(n) \
  if (N == n) return split_nv_n##n##_f32r();
    HMPC_F32R_LIST(HMPC_CASE)
#undef HMPC_CASE
    return 0;
  }
  if (flavor == 1) {
#define HMPC_CASE(n) \
  if (N == n) return split_nv_n##n##_f32();
    HMPC_F32_LIST(HMPC_CASE)
#undef HMPC_CASE
    return 0;
  }
#define HMPC_CASE(n) \
  if (N == n) return split_nv_n##n();
  HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
  return 0;
}

const char* dense_name(int variant, int N, int flavor) {
  if (flavor == 2) {
#define HMPC_CASE(n) \
  if (N == n) return name_solve_n##n##_f32r(variant);
    HMPC_F32R_LIST(HMPC_CASE)
#undef HMPC_CASE
    return "";
  }
  if (flavor == 1) {
#define HMPC_CASE(n) \
  if (N == n) return name_solve_n##n##_f32(variant);
    HMPC_F32_LIST(HMPC_CASE)
#undef HMPC_CASE
    return "";
  }
#define HMPC_CASE(n) \
  if (N == n) return name_solve_n##n(variant);
  HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
  return "";
}

bool horizon_supported(int variant, int N) {
  if (variant == 4) return N >= 1 && N <= kCasNmax;
  if (variant != 2 && variant != 3) return false;
  return horizon_compiled(variant, N) || (N >= 1 && N <= kWideNmax);
}

int supported_horizons(int variant, int* Ns, int cap) {
  if (variant != 2 && variant != 3) return 0;
  int n = 0;
#define HMPC_CASE(h)            \
  if (Ns && n < cap) Ns[n] = h; \
  ++n;
  HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
  return n;
}

}  // namespace hmpc
