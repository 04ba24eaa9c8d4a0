// fp64_peak.hip -- measured vector FMA throughput of the MI355X this runs on,
// the denominator of bench.py's fp64_vector / fp32_vector roofline (VERDICT
// r02 item 6: anchor the peak on the box, not on a datasheet).
//
// Every thread runs 16 independent FMA chains (enough ILP to cover the fp64
// FMA latency at 8 waves / SIMD); 8 workgroups of 256 threads per CU.  One
// FMA = 2 flops.  Prints one JSON line:
//   {"fp64_fma_tflops": ..., "fp32_fma_tflops": ..., "fp32_pk_fma_tflops": ...,
//    "cus": ..., "clock_mhz": ...}
// Build: hipcc --offload-arch=gfx950 -O3 tools/fp64_peak.hip -o tools/fp64_peak
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int kChains = 16;

template <typename T>
__global__ void __launch_bounds__(256) fma_kernel(T* out, int iters, T a, T b) {
  T x[kChains];
#pragma unroll
  for (int j = 0; j < kChains; ++j) x[j] = (T)(threadIdx.x + j);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < kChains; ++j) x[j] = fma(x[j], a, b);
  }
  T s = 0;
#pragma unroll
  for (int j = 0; j < kChains; ++j) s += x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// packed fp32: two lanes of a float2 per v_pk_fma_f32
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) pk_fma_kernel(float* out, int iters, float a, float b) {
  f2 x[kChains];
  const f2 av = {a, a}, bv = {b, b};
#pragma unroll
  for (int j = 0; j < kChains; ++j) x[j] = (f2){(float)(threadIdx.x + j), (float)j};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < kChains; ++j) x[j] = __builtin_elementwise_fma(x[j], av, bv);
  }
  float s = 0;
#pragma unroll
  for (int j = 0; j < kChains; ++j) s += x[j].x + x[j].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename L>
double time_ms(L launch, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();   // warm (clocks, code load)
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
  const int blocks = cus * 8, threads = 256, iters = 4096, reps = 20;
  double* od;
  float* of;
  CK(hipMalloc(&od, sizeof(double) * blocks * threads));
  CK(hipMalloc(&of, sizeof(float) * blocks * threads));
  const double flops = 2.0 * kChains * (double)iters * blocks * threads;
  const double t64 = time_ms([&] { hipLaunchKernelGGL(fma_kernel<double>, dim3(blocks), dim3(threads), 0, 0, od, iters, 0.999999, 1e-7); }, reps);
  const double t32 = time_ms([&] { hipLaunchKernelGGL(fma_kernel<float>, dim3(blocks), dim3(threads), 0, 0, of, iters, 0.9999f, 1e-4f); }, reps);
  const double tpk = time_ms([&] { hipLaunchKernelGGL(pk_fma_kernel, dim3(blocks), dim3(threads), 0, 0, of, iters, 0.9999f, 1e-4f); }, reps);
  CK(hipGetLastError());
  printf("{\"fp64_fma_tflops\": %.2f, \"fp32_fma_tflops\": %.2f, \"fp32_pk_fma_tflops\": %.2f, "
         "\"cus\": %d, \"clock_mhz\": %.0f, \"threads\": %d, \"iters\": %d, \"chains\": %d}\n",
         flops / (t64 * 1e-3) / 1e12, flops / (t32 * 1e-3) / 1e12, 2.0 * flops / (tpk * 1e-3) / 1e12, cus,
         clk / 1e3, blocks * threads, iters, kChains);
  CK(hipFree(od));
  CK(hipFree(of));
  return 0;
}
