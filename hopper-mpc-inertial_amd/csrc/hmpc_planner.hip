// hmpc_planner.hip -- the Runner's reference / gait generation on the device
// (SURVEY.md 8f row 3), for B robots with their own start and goal states:
//
//   plan_scan_kernel   one thread: gait_map(T, dt, t_start, 0) over the plan's
//                      T low-level steps (the float64 time accumulation of
//                      src/robotrunner.py:174-180) and the footstep counter
//                      of path_plan_init's pf loop (:218-223)
//   plan_peaks_kernel  one thread per robot: find_peaks(-z) of the robot's
//                      height profile (:211-216; scipy's plateau rule)
//   plan_rows_kernel   one thread per (robot, row): x_ref row (linspace,
//                      --curve splines, height sine, finite-difference
//                      velocities, :188-209) and pf_ref row (:218-223)
//   gait_calls_kernel  one thread: the Runner loop's per-step contact and
//                      per-MPC-call gait_map (:92-101)
//
// Every decision (gait state, peak, footstep index) and every linspace /
// difference value follows the reference's float64 operation order exactly:
// this file is compiled without FMA contraction.  The sine and the --curve
// splines are within a few ulp of numpy/scipy (tests/test_gpu_planner.py).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "hmpc_internal.h"

#pragma clang fp contract(off)

namespace hmpc {

namespace {

constexpr int kMaxPeaks = 64;   // footstep indices per robot (a 2000-step run has 5)

// Runner.gait_scheduler (src/robotrunner.py:166-172): np.mod(x, 1), swing
// when the phase exceeds phi_switch.  np.mod follows the divisor's sign:
// fmod, then + 1 for a negative remainder (numpy's npy_divmod), so t < t0
// gives the reference's phase in [0, 1)
__device__ __forceinline__ double np_mod1(double x) {
  double r = fmod(x, 1.0);
  if (r != 0.0 && r < 0.0) r += 1.0;
  return r;
}
__device__ __forceinline__ double gait_state(double t, double t0, double t_p, double phi_switch) {
  const double ph = np_mod1((t - t0) / t_p);
  return ph > phi_switch ? 0.0 : 1.0;
}

// device error word of hmpc_plan_batch (HMPC_ERR_ARG on the host): cases in
// which the reference raises IndexError or keeps more than this kernel can
constexpr int kErrPeaks = 1;      // more footstep peaks than kMaxPeaks
constexpr int kErrPeakIdx = 2;    // peak + step_adjustment outside [-T, T)
constexpr int kErrFootIdx = 4;    // footstep counter past the end of idx_pf

// np.linspace(start, stop, num) row i, component c (numpy 2.x: when any
// component's step is zero the whole array takes the y = (i / div) * delta
// path, else y = i * step; then + start; the last row is stop itself)
__device__ __forceinline__ double lin(const double* a, const double* b, int num, int i, int c, bool anyzero) {
  if (i == num - 1) return b[c];
  const double div = (double)(num - 1);
  const double delta = b[c] - a[c];
  double y;
  if (anyzero) y = ((double)i / div) * delta;
  else y = (double)i * (delta / div);
  return y + a[c];
}

// the --curve splines: scipy CubicSpline through (0, y0), (h, y1), (2h, y2)
// with not-a-knot ends is the parabola through the three points (scipy's
// n = 3 case); evaluated in Newton form
__device__ __forceinline__ double parabola(double y0, double y1, double y2, double h, double x) {
  const double d1 = (y1 - y0) / h, d2 = (y2 - y1) / h;
  const double c2 = (d2 - d1) / (2.0 * h);
  return y0 + x * (d1 + (x - h) * c2);
}

struct PlanArgs {
  int64_t B;
  int T, N_run, t_traj;
  double dt, t_p, phi_switch, t_start;
  int step_adjustment, curve;
  const double* x_in;   // [B,12]
  const double* xf;     // [B,12]
  double* x_ref;        // [B,T,12]
  double* pf_ref;       // [B,T,3]
  double* C_map;        // [T] (optional)
  int32_t* kf;          // [T] scratch: footstep counter after step k
  int32_t* peaks;       // [B][kMaxPeaks + 2] scratch: idx_pf, count at [kMaxPeaks + 1]
  int32_t* err;         // [1] error bits (kErr*), zeroed before the launch
};

// height profile (:207): x_in[2] + amp + amp sin(2 pi / period (i dt) + phi)
__device__ __forceinline__ double height(const PlanArgs& a, const double* x0, int i) {
  const double amp = a.t_p / 4.0;
  const double arg = 2.0 * M_PI / a.t_p * ((double)i * a.dt) + M_PI * 3.0 / 2.0;
  return x0[2] + amp + amp * sin(arg);
}

__global__ void plan_scan_kernel(PlanArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  // gait_map(T, dt, t_start, 0): C[k] = scheduler(ts), ts += dt
  double ts = a.t_start;
  double cprev = 0.0;
  int kf = 0;
  for (int k = 0; k < a.T; ++k) {
    const double c = gait_state(ts, 0.0, a.t_p, a.phi_switch);
    ts = ts + a.dt;
    if (a.C_map) a.C_map[k] = c;
    // (:219-222) kf += 1 on a stance -> swing edge; the n_idx bound is
    // applied per robot in plan_rows_kernel
    if (k >= 1 && cprev == 1.0 && c == 0.0) ++kf;
    a.kf[k] = kf;
    cprev = c;
  }
}

__global__ void plan_peaks_kernel(PlanArgs a) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const double* x0 = a.x_in + 12 * b;
  int32_t* pk = a.peaks + b * (kMaxPeaks + 2);
  // scipy.signal._peak_finding_utils._local_maxima_1d on x = -z
  const int n = a.T;
  int m = 0;
  pk[m++] = 0;   // idx_pf = [0, peaks + step_adjustment, T - 1]  (:212-216)
  int i = 1;
  double xm1 = -height(a, x0, 0), xi = -height(a, x0, 1);
  while (i < n - 1) {
    if (xm1 < xi) {
      int ia = i + 1;
      double xa = -height(a, x0, ia);
      while (ia < n - 1 && xa == xi) {
        ++ia;
        xa = -height(a, x0, ia);
      }
      if (xa < xi) {
        int p = (i + (ia - 1)) / 2 + a.step_adjustment;
        if (p < 0) p += n;   // a negative numpy index counts from the end
        if (p < 0 || p >= n)   // numpy: IndexError only when x_ref[idx_pf[kf]] is read:
          p = -1 - (p < 0 ? 0 : n - 1);   // kept clamped and marked (< 0), plan_rows_kernel reports it
        if (m < kMaxPeaks) pk[m++] = p;
        else atomicOr(a.err, kErrPeaks);   // the reference keeps every peak
        i = ia;
        xm1 = -height(a, x0, i - 1);
        xi = xa;
      }
    }
    ++i;
    xm1 = -height(a, x0, i - 1);
    xi = -height(a, x0, i);
  }
  pk[m++] = n - 1;
  pk[kMaxPeaks + 1] = m;
}

// x_ref[b, i, c] before the velocity columns (:188-207)
__device__ double row_val(const PlanArgs& a, const double* x0, const double* x1, bool anyzero, int i, int c) {
  if (c == 2) return height(a, x0, i);
  if (i >= a.t_traj) return x1[c];   // np.tile(xf, (N_k + t_sit, 1))
  if (a.curve) {
    const double h = (double)a.t_traj * 0.5;
    if (c == 0)   // sic (:198): the y spline is written into column 0
      return parabola(x0[1], x1[1] * 0.9, x1[1], h, (double)i);
    if (c == 5) {
      const double s45 = sin(45.0 * M_PI / 180.0);
      return parabola(0.0, -s45 * 0.4, -s45, h, (double)i);
    }
    if (c == 11 && i < a.N_run - 1)   // (:201) the yaw-rate column differentiates itself
      return (lin(x0, x1, a.t_traj, i + 1, 11, anyzero) - lin(x0, x1, a.t_traj, i, 11, anyzero)) / a.dt;
  }
  return lin(x0, x1, a.t_traj, i, c, anyzero);
}

__global__ void plan_rows_kernel(PlanArgs a) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.B * a.T) return;
  const int64_t b = g / a.T;
  const int i = (int)(g - b * a.T);
  const double* x0 = a.x_in + 12 * b;
  const double* x1 = a.xf + 12 * b;
  bool anyzero = false;
  for (int c = 0; c < 12; ++c) anyzero |= ((x1[c] - x0[c]) / (double)(a.t_traj - 1)) == 0.0;
  double* xr = a.x_ref + (b * a.T + i) * 12;
  for (int c = 0; c < 12; ++c) {
    double v;
    if (c >= 6 && c < 9 && i < a.T - 1)   // (:209) linear velocities by forward differences
      v = (row_val(a, x0, x1, anyzero, i + 1, c - 6) - row_val(a, x0, x1, anyzero, i, c - 6)) / a.dt;
    else
      v = row_val(a, x0, x1, anyzero, i, c);
    xr[c] = v;
  }
  // pf_ref[i, 0:2] = x_ref[idx_pf[kf], 0:2]  (:217-223), row 0 and column 2 zero
  const int32_t* pk = a.peaks + b * (kMaxPeaks + 2);
  const int n_idx = pk[kMaxPeaks + 1];
  double* pf = a.pf_ref + (b * a.T + i) * 3;
  pf[2] = 0.0;
  if (i == 0) {
    pf[0] = 0.0;
    pf[1] = 0.0;
  } else {
    int kf = a.kf[i];
    if (kf > n_idx - 1) {   // the reference raises IndexError past the end of idx_pf
      atomicOr(a.err, kErrFootIdx);
      kf = n_idx - 1;
    }
    int j = pk[kf];
    if (j < 0) {   // a peak outside the plan (plan_peaks_kernel), read here: IndexError (:223)
      atomicOr(a.err, kErrPeakIdx);
      j = -1 - j;
    }
    pf[0] = row_val(a, x0, x1, anyzero, j, 0);
    pf[1] = row_val(a, x0, x1, anyzero, j, 1);
  }
}

struct GaitArgs {
  int n_steps, mpc_factor, N;
  double dt, mpc_dt, t_p, phi_switch, t_start, t0;
  double* C_calls;   // [n_calls, N]
  double* s_hist;    // [n_steps] (optional)
};

__global__ void gait_calls_kernel(GaitArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double t = a.t_start;
  int p = 0;
  for (int k = 0; k < a.n_steps; ++k) {
    t = t + a.dt;   // (:96)
    if (a.s_hist) a.s_hist[k] = gait_state(t, a.t0, a.t_p, a.phi_switch);
    if (k % a.mpc_factor == 0) {   // gait_map(N, mpc_dt, t, t0)  (:100)
      double ts = t;
      for (int j = 0; j < a.N; ++j) {
        a.C_calls[(int64_t)p * a.N + j] = gait_state(ts, a.t0, a.t_p, a.phi_switch);
        ts = ts + a.mpc_dt;
      }
      ++p;
    }
  }
}

}  // namespace

int64_t plan_scratch_bytes(int64_t B, int T) {
  return (int64_t)sizeof(int32_t) * (T + B * (kMaxPeaks + 2) + 1);   // + the error word
}

bool launch_plan(int64_t B, int N_run, int N_k, double dt, int curve, double t_p, double phi_switch,
                 double t_start, int step_adjustment, const double* x_in, const double* xf, double* x_ref,
                 double* pf_ref, double* C_map, void* scratch, hipStream_t s) {
  if (B <= 0) return true;
  PlanArgs a;
  a.B = B;
  a.N_run = N_run;
  a.t_traj = N_run;   // t_sit = 0 (:186-187)
  a.T = N_run + N_k;
  a.dt = dt;
  a.t_p = t_p;
  a.phi_switch = phi_switch;
  a.t_start = t_start;
  a.step_adjustment = step_adjustment;
  a.curve = curve;
  a.x_in = x_in;
  a.xf = xf;
  a.x_ref = x_ref;
  a.pf_ref = pf_ref;
  a.C_map = C_map;
  a.kf = static_cast<int32_t*>(scratch);
  a.peaks = a.kf + a.T;
  a.err = a.peaks + B * (kMaxPeaks + 2);
  if (hipMemsetAsync(a.err, 0, sizeof(int32_t), s) != hipSuccess) return false;
  hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(plan_peaks_kernel, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, s, a);
  const int64_t n = B * a.T;
  hipLaunchKernelGGL(plan_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return true;
}

const int32_t* plan_error_word(int64_t B, int T, const void* scratch) {
  return static_cast<const int32_t*>(scratch) + T + B * (kMaxPeaks + 2);
}

bool launch_gait(int n_steps, int mpc_factor, int N, double dt, double mpc_dt, double t_p,
                 double phi_switch, double t_start, double t0, double* C_calls, double* s_hist,
                 hipStream_t s) {
  GaitArgs a{n_steps, mpc_factor, N, dt, mpc_dt, t_p, phi_switch, t_start, t0, C_calls, s_hist};
  hipLaunchKernelGGL(gait_calls_kernel, dim3(1), dim3(64), 0, s, a);
  return true;
}

}  // namespace hmpc
