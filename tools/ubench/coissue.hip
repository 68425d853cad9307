// Microbenchmark: does 32-bit VALU work issue alongside the FP64 pipe on gfx950, and how
// long is a dependent f64 chain? Per lane C independent chains; each loop step issues one
// instruction per chain of each listed kind. Reported: SIMD cycles per loop step at 2.4 GHz.
// Not part of the product. Build: hipcc --offload-arch=gfx950 -O3 -o coissue tools/ubench/coissue.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 1024

// kinds: F = v_fma_f64 on chain c, X = v_xor_b32 on int chain c, S = v_fma_f32 on float chain c,
// V = f64 -> f32 -> f64 conversion round trip on chain c (2 instructions)
template <int C, bool F, bool X, bool S, bool V>
__global__ void k(double* out, double a, float b, unsigned m) {
  double d[C], e[C];
  unsigned u[C];
  float f[C];
  for (int c = 0; c < C; ++c) {
    d[c] = threadIdx.x * 1e-3 + c;
    e[c] = threadIdx.x * 2e-3 + c;
    u[c] = threadIdx.x * 7u + c;
    f[c] = threadIdx.x * 1e-3f + c;
  }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (F) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[c]) : "v"(a));
      if (X) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[c]) : "v"(m));
      if (S) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(b));
      if (V) {
        float t;
        asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(t) : "v"(e[c]));
        asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(e[c]) : "v"(t));
      }
    }
  }
  double s = 0;
  for (int c = 0; c < C; ++c) s += d[c] + e[c] + u[c] + f[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*KF)(double*, double, float, unsigned);
int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  double* out;
  hipMalloc(&out, sizeof(double) * p.multiProcessorCount * 8 * 256);
  struct Case { const char* n; KF f; int per_simd_waves; };
  Case cs[] = {
      {"fma_f64 x8 chains             (8 w/SIMD)", k<8, true, false, false, false>, 8},
      {"xor_b32 x8                    (8 w/SIMD)", k<8, false, true, false, false>, 8},
      {"fma_f32 x8                    (8 w/SIMD)", k<8, false, false, true, false>, 8},
      {"fma_f64 + xor_b32 x8          (8 w/SIMD)", k<8, true, true, false, false>, 8},
      {"fma_f64 + fma_f32 x8          (8 w/SIMD)", k<8, true, false, true, false>, 8},
      {"cvt round trip x8             (8 w/SIMD)", k<8, false, false, false, true>, 8},
      {"fma_f64 + cvt round trip x8   (8 w/SIMD)", k<8, true, false, false, true>, 8},
      {"fma_f64 x8 chains             (4 w/SIMD)", k<8, true, false, false, false>, 4},
      {"fma_f64 x4 chains             (4 w/SIMD)", k<4, true, false, false, false>, 4},
      {"fma_f64 x2 chains             (4 w/SIMD)", k<2, true, false, false, false>, 4},
      {"fma_f64 x1 chain              (4 w/SIMD)", k<1, true, false, false, false>, 4},
      {"fma_f64 x1 chain              (1 w/SIMD)", k<1, true, false, false, false>, 1},
      {"cvt round trip x1             (1 w/SIMD)", k<1, false, false, false, true>, 1},
      {"fma_f64 + xor_b32 x2          (4 w/SIMD)", k<2, true, true, false, false>, 4},
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    for (auto& c : cs) {
      // one workgroup of 64 * w threads per CU... w waves per SIMD: 4 w waves per CU
      const int threads = 256, blocks = p.multiProcessorCount * c.per_simd_waves;
      hipLaunchKernelGGL(c.f, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001, 0.999999f, 0x5555u);
      hipEventRecord(e0);
      hipLaunchKernelGGL(c.f, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001, 0.999999f, 0x5555u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1)
        printf("%s  %.3f ms  %.2f SIMD cycles per loop step\n", c.n, ms,
               ms * 1e-3 * 2.4e9 / ((double)ITERS * c.per_simd_waves));
    }
  return 0;
}
