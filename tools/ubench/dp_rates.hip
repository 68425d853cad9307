// Microbenchmark: per-wave issue cost of FP64 FMA, f32<->f64 conversions and f32 FMA on gfx950.
// Used to size the faithful FFT ("FP64 budget"). Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define ITERS 4096
#define CHAINS 8
__global__ void k_fma64(double* out, double a, double b) {
  double x[CHAINS];
  for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3 + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fma(x[c], a, b);
  }
  double s = 0; for (int c = 0; c < CHAINS; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cvt(double* out, float a) {
  float x[CHAINS];
  for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) { double d = (double)x[c]; x[c] = (float)(d * 0.5 + 0.25); }
  }
  double s = 0; for (int c = 0; c < CHAINS; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma32(double* out, float a, float b) {
  float x[CHAINS];
  for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fmaf(x[c], a, b);
  }
  double s = 0; for (int c = 0; c < CHAINS; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  int blocks = 256 * 8, threads = 256;
  double* d; hipMalloc(&d, sizeof(double) * blocks * threads);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipEventRecord(e0); k_fma64<<<blocks, threads>>>(d, 0.999, 1e-3); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double ops = (double)blocks * threads * ITERS * CHAINS;
    printf("fma64: %.3f ms  %.2f Tlane-op/s  (%.1f TFLOP/s)\n", ms, ops / ms / 1e9, 2 * ops / ms / 1e9);
    hipEventRecord(e0); k_cvt<<<blocks, threads>>>(d, 0.5f); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("cvt-up+fma64+cvt-down: %.3f ms  %.2f Tlane-iter/s (3 ops each)\n", ms, ops / ms / 1e9);
    hipEventRecord(e0); k_fma32<<<blocks, threads>>>(d, 0.999f, 1e-3f); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("fma32: %.3f ms  %.2f Tlane-op/s\n", ms, ops / ms / 1e9);
  }
  return 0;
}
