// Unit check of the half-wave primitives of hmpc_swing.hip on the GPU:
// permlane16_swap pairing, row/half broadcasts, half sums, under full and
// half-divergent exec.  Build: hipcc --offload-arch=gfx950 -O3 tools/swing_prims.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
template <int CTRL>
__device__ __forceinline__ int dpp32(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false); }
__global__ void k(double* out, int mode) {
  const int lane = threadIdx.x;
  double x = 100.0 + lane;
  double r[6] = {0, 0, 0, 0, 0, 0};
  bool run = mode == 0 || (mode == 1 ? lane >= 32 : lane < 32);
  if (run) {
    // raw permlane16_swap(x, x)
    const long long b = __double_as_longlong(x);
    auto pl = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    auto ph = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    r[0] = __longlong_as_double(((long long)(unsigned)ph[0] << 32) | (unsigned)pl[0]);
    r[1] = __longlong_as_double(((long long)(unsigned)ph[1] << 32) | (unsigned)pl[1]);
    r[2] = __builtin_amdgcn_update_dpp(0.0, x, 0x150 + 5, 0xf, 0xf, true);   // row lane 5
    r[3] = __builtin_amdgcn_update_dpp(0.0, x, 0x150 + 9, 0xf, 0xf, true);
    // half sum via 32-bit dpp of ints
    int s = lane;
    s += dpp32<0xB1>(s); s += dpp32<0x4E>(s); s += dpp32<0x141>(s); s += dpp32<0x140>(s);
    auto ps = __builtin_amdgcn_permlane16_swap((unsigned)s, (unsigned)s, false, false);
    r[4] = (double)((int)ps[0] + (int)ps[1]);
    r[5] = (double)__builtin_amdgcn_ds_bpermute((((lane >> 5) << 5) + 3) << 2, lane);
  }
  for (int i = 0; i < 6; ++i) out[(mode * 6 + i) * 64 + lane] = r[i];
}
int main() {
  double* d; hipMalloc(&d, 3 * 6 * 64 * 8);
  hipMemset(d, 0, 3 * 6 * 64 * 8);
  for (int m = 0; m < 3; ++m) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m);
  double h[3 * 6 * 64];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[6] = {"swap.even", "swap.odd", "rbc5", "rbc9", "halfsum(lane)", "bperm(h*32+3)"};
  for (int m = 0; m < 3; ++m) {
    printf("mode %d (%s)\n", m, m == 0 ? "all lanes" : m == 1 ? "upper half only" : "lower half only");
    for (int i = 0; i < 6; ++i) {
      printf("  %-14s", nm[i]);
      for (int l = 0; l < 64; l += 4) printf(" %g", h[(m * 6 + i) * 64 + l]);
      printf("\n");
    }
  }
  return 0;
}
