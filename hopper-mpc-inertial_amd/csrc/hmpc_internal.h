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
  // element strides of the x_ref / pf / C views (contiguous: 12N, 12 / 3N, 3
  // / N); a batch stride of 0 shares one plan window across the batch
  int64_t xref_bs, pf_bs, C_bs;
  int xref_rs, pf_rs;
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

// Launch the solve kernel for (variant, N).  Returns false when no kernel
// is compiled for that combination.
bool launch_solve(int variant, int N, const SolveArgs& a, hipStream_t stream);
bool horizon_supported(int variant, int N);
int supported_horizons(int variant, int* Ns, int cap);

}  // namespace hmpc
