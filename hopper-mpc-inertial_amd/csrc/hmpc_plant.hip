// hmpc_plant.hip -- the Runner's plant on the device:
// batched RK4 integration of the SE(3) rigid-body dynamics between MPC
// solves, and the SE(3) -> Euler state conversion that feeds the next solve.
//
//   dynamics_ct     src/robotrunner.py:126-152
//   rk4_normalized  src/robotrunner.py:154-164
//   convert         src/robotrunner.py:19-28 (quat2euler: src/utils.py:54-62,
//                   transforms3d 'rzyx' = quat2mat + mat2euler)
//
// One thread per robot: the state (13 doubles), the held input and the
// constants live in registers; a launch integrates `n_steps` low-level steps
// (one MPC period = mpc_factor steps in the Runner) so the state never leaves
// the chip between them.  This is ~1e4 flops per robot per period: latency
// of a small launch, not throughput, is what it costs next to the solve.
#include <hip/hip_runtime.h>

#include "hmpc_internal.h"

namespace hmpc {

namespace {

struct Rot {   // body-to-world rotation H' L(q) R(q)' H  (src/utils.py:28-43)
  double r[3][3];
  __device__ explicit Rot(const double* q) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    r[0][0] = w * w + x * x - y * y - z * z;
    r[0][1] = 2.0 * (x * y - w * z);
    r[0][2] = 2.0 * (x * z + w * y);
    r[1][0] = 2.0 * (x * y + w * z);
    r[1][1] = w * w - x * x + y * y - z * z;
    r[1][2] = 2.0 * (y * z - w * x);
    r[2][0] = 2.0 * (x * z - w * y);
    r[2][1] = 2.0 * (y * z + w * x);
    r[2][2] = w * w - x * x - y * y + z * z;
  }
  __device__ void apply(const double* a, double* o) const {   // o = R a
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = r[i][0] * a[0] + r[i][1] * a[1] + r[i][2] * a[2];
  }
  __device__ void apply_t(const double* a, double* o) const {   // o = R' a
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = r[0][i] * a[0] + r[1][i] * a[1] + r[2][i] * a[2];
  }
};

__device__ inline void cross(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// dX = f(X, U, pf)   (src/robotrunner.py:126-152)
__device__ void dynamics(const PlantArgs& a, const double* X, const double* U, const double* pf,
                         double* dX) {
  const double* p = X;
  const double* q = X + 3;
  const double* v = X + 7;
  const double* w = X + 10;
  const Rot R(q);
  double fw[3] = {U[0], U[1], U[2] - a.g * a.m};   // Fgw + Fw
  double ftb[3], dpf[3], r[3], fb[3], t[3];
  R.apply_t(fw, ftb);
  for (int i = 0; i < 3; ++i) dpf[i] = pf[i] - p[i];
  R.apply_t(dpf, r);
  for (int i = 0; i < 3; ++i) r[i] += a.rh[i];
  R.apply_t(U, fb);
  cross(r, fb, t);
  double tau[3] = {U[3] + t[0], U[4] + t[1], U[5] + t[2]};
  R.apply(v, dX);   // dp
  // dq = 0.5 L(q) H w
  dX[3] = 0.5 * (-q[1] * w[0] - q[2] * w[1] - q[3] * w[2]);
  dX[4] = 0.5 * (q[0] * w[0] - q[3] * w[1] + q[2] * w[2]);
  dX[5] = 0.5 * (q[3] * w[0] + q[0] * w[1] - q[1] * w[2]);
  dX[6] = 0.5 * (-q[2] * w[0] + q[1] * w[1] + q[0] * w[2]);
  double wv[3];
  cross(w, v, wv);
  for (int i = 0; i < 3; ++i) dX[7 + i] = ftb[i] / a.m - wv[i];
  // dw = J^-1 (tau - w x J w)
  double jw[3], wjw[3], rhs[3];
  for (int i = 0; i < 3; ++i) jw[i] = a.J[3 * i] * w[0] + a.J[3 * i + 1] * w[1] + a.J[3 * i + 2] * w[2];
  cross(w, jw, wjw);
  for (int i = 0; i < 3; ++i) rhs[i] = tau[i] - wjw[i];
  for (int i = 0; i < 3; ++i)
    dX[10 + i] = a.Jinv[3 * i] * rhs[0] + a.Jinv[3 * i + 1] * rhs[1] + a.Jinv[3 * i + 2] * rhs[2];
}

// x = convert(X)   (src/robotrunner.py:19-28)
__device__ void convert_state(const double* X, double* x) {
  const double* q = X + 3;
  x[0] = X[0]; x[1] = X[1]; x[2] = X[2];
  // quat2euler: transforms3d quat2mat (s = 2/|q|^2) then mat2euler 'rzyx'
  const double w = q[0], qx = q[1], qy = q[2], qz = q[3];
  const double nq = w * w + qx * qx + qy * qy + qz * qz;
  double M[3][3];
  if (nq < 2.220446049250313e-16) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) M[i][j] = i == j ? 1.0 : 0.0;
  } else {
    const double s = 2.0 / nq;
    const double X_ = qx * s, Y = qy * s, Z = qz * s;
    const double wX = w * X_, wY = w * Y, wZ = w * Z;
    const double xX = qx * X_, xY = qx * Y, xZ = qx * Z;
    const double yY = qy * Y, yZ = qy * Z, zZ = qz * Z;
    M[0][0] = 1.0 - (yY + zZ); M[0][1] = xY - wZ; M[0][2] = xZ + wY;
    M[1][0] = xY + wZ; M[1][1] = 1.0 - (xX + zZ); M[1][2] = yZ - wX;
    M[2][0] = xZ - wY; M[2][1] = yZ + wX; M[2][2] = 1.0 - (xX + yY);
  }
  const double cy = sqrt(M[0][0] * M[0][0] + M[1][0] * M[1][0]);
  if (cy > 4.0 * 2.220446049250313e-16) {
    x[3] = atan2(M[2][1], M[2][2]);
    x[4] = atan2(-M[2][0], cy);
    x[5] = atan2(M[1][0], M[0][0]);
  } else {
    x[3] = atan2(-M[1][2], M[1][1]);
    x[4] = atan2(-M[2][0], cy);
    x[5] = 0.0;
  }
  const Rot R(q);
  R.apply(X + 7, x + 6);    // body v -> world pdot
  R.apply(X + 10, x + 9);   // body w -> world w
}

__global__ void __launch_bounds__(64) plant_kernel(PlantArgs a) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  double X[13], U[6];
  for (int i = 0; i < 13; ++i) X[i] = a.X[b * 13 + i];
  for (int i = 0; i < 6; ++i) U[i] = a.U[b * a.U_bs + i];
  const double h = a.dt;
#pragma unroll 1
  for (int s = 0; s < a.n_steps; ++s) {
    const double* pf = a.pf + b * a.pf_bs + (int64_t)s * a.pf_ss;
    double pfl[3] = {pf[0], pf[1], pf[2]};
    double f1[13], f2[13], f3[13], f4[13], Y[13];
    dynamics(a, X, U, pfl, f1);
    for (int i = 0; i < 13; ++i) Y[i] = X[i] + 0.5 * h * f1[i];
    dynamics(a, Y, U, pfl, f2);
    for (int i = 0; i < 13; ++i) Y[i] = X[i] + 0.5 * h * f2[i];
    dynamics(a, Y, U, pfl, f3);
    for (int i = 0; i < 13; ++i) Y[i] = X[i] + h * f3[i];
    dynamics(a, Y, U, pfl, f4);
    for (int i = 0; i < 13; ++i) X[i] = X[i] + (h / 6.0) * (f1[i] + 2.0 * f2[i] + 2.0 * f3[i] + f4[i]);
    const double nq = sqrt(X[3] * X[3] + X[4] * X[4] + X[5] * X[5] + X[6] * X[6]);
    for (int i = 3; i < 7; ++i) X[i] = X[i] / nq;
    if (a.X_hist)
      for (int i = 0; i < 13; ++i) a.X_hist[(b * a.n_steps + s) * 13 + i] = X[i];
  }
  for (int i = 0; i < 13; ++i) a.X[b * 13 + i] = X[i];
  if (a.x_out) {
    double x[12];
    convert_state(X, x);
    for (int i = 0; i < 12; ++i) a.x_out[b * 12 + i] = x[i];
  }
}

__global__ void __launch_bounds__(64) convert_kernel(int64_t B, const double* X, double* x) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double Xl[13], xl[12];
  for (int i = 0; i < 13; ++i) Xl[i] = X[b * 13 + i];
  convert_state(Xl, xl);
  for (int i = 0; i < 12; ++i) x[b * 12 + i] = xl[i];
}

}  // namespace

void launch_plant(const PlantArgs& a, hipStream_t s) {
  if (a.B <= 0) return;
  hipLaunchKernelGGL(plant_kernel, dim3((unsigned)((a.B + 63) / 64)), dim3(64), 0, s, a);
}

void launch_convert(int64_t B, const double* X, double* x, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(convert_kernel, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, s, B, X, x);
}

}  // namespace hmpc
