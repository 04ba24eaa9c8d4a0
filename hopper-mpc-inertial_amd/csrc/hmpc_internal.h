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
};

// Launch the solve kernel for (variant, N).  Returns false when no kernel
// is compiled for that combination.
bool launch_solve(int variant, int N, const SolveArgs& a, hipStream_t stream);
bool horizon_supported(int variant, int N);
int supported_horizons(int variant, int* Ns, int cap);

}  // namespace hmpc
