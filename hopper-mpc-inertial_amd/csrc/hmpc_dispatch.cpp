// Maps (variant, N) onto the per-horizon launchers compiled from
// hmpc_kernels.hip (one object per horizon, see build.sh).
#include "hmpc_internal.h"

#ifndef HMPC_HORIZON_LIST
#define HMPC_HORIZON_LIST(X) X(5) X(10) X(20)
#endif

namespace hmpc {

#define HMPC_DECL(n) bool launch_solve_n##n(int variant, const SolveArgs& a, hipStream_t s);
HMPC_HORIZON_LIST(HMPC_DECL)
#undef HMPC_DECL

bool launch_solve(int variant, int N, const SolveArgs& a, hipStream_t s) {
  if (variant != 2 && variant != 3) return false;
  if (a.precision != 0) return launch_solve_wide(variant, N, a, s);
#define HMPC_CASE(n) \
  if (N == n) return launch_solve_n##n(variant, a, s);
  HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
  return launch_solve_wide(variant, N, a, s);
}

bool horizon_compiled(int variant, int N) {
  if (variant != 2 && variant != 3) return false;
#define HMPC_CASE(n) \
  if (N == n) return true;
  HMPC_HORIZON_LIST(HMPC_CASE)
#undef HMPC_CASE
  return false;
}

bool horizon_supported(int variant, int N) {
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
