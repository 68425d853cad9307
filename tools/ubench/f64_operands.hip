// Microbenchmark: issue cost of f64 VALU instructions by operand kind (VGPR / SGPR /
// inline constant sources), 8 waves per SIMD, 8 independent chains per lane. Question: is
// the measured ~5 cycles per v_fma_f64 (4 expected from the FP64 peak) an operand-fetch
// cost that SGPR operands avoid? Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -o f64_operands tools/ubench/f64_operands.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define K(name, ASM, ...)                                                                 \
  __global__ void name(double* out, double a, double b) {                                 \
    double x[8];                                                                          \
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3 + c;                            \
    double va = a + threadIdx.x, vb = b - threadIdx.x;                                    \
    for (int i = 0; i < ITERS; ++i) {                                                     \
      _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                     \
        _Pragma("unroll") for (int c = 0; c < 8; ++c) asm volatile(ASM : "+v"(x[c]) : __VA_ARGS__); \
      }                                                                                   \
    }                                                                                     \
    double s = 0;                                                                         \
    for (int c = 0; c < 8; ++c) s += x[c];                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + va + vb;                             \
  }

K(k_fma_vvv, "v_fma_f64 %0, %0, %1, %2", "v"(va), "v"(vb))
K(k_fma_vsv, "v_fma_f64 %0, %0, %1, %2", "s"(a), "v"(vb))
K(k_fma_vss, "v_fma_f64 %0, %0, %1, %1", "s"(a), "s"(a))
K(k_fma_vvk, "v_fma_f64 %0, %0, %1, 0.5", "v"(va), "v"(vb))
K(k_mul_vv, "v_mul_f64 %0, %0, %1", "v"(va), "v"(vb))
K(k_mul_vs, "v_mul_f64 %0, %0, %1", "s"(a), "v"(vb))
K(k_add_vv, "v_add_f64 %0, %0, %1", "v"(va), "v"(vb))
K(k_add_vk, "v_add_f64 %0, %0, 1.0", "v"(va), "v"(vb))
K(k_fmac_vv, "v_fmac_f64 %0, %1, %2", "v"(va), "v"(vb))

__global__ void k_cvt_n(double* out, double a, double b) {
  double x[8];
  float y[8];
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3 + c + a + b;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(y[c]) : "v"(x[c]));
    }
  }
  float s = 0;
  for (int c = 0; c < 8; ++c) s += y[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cvt_w(double* out, double a, double b) {
  double x[8];
  float y[8];
  for (int c = 0; c < 8; ++c) y[c] = threadIdx.x * 1e-3f + c + (float)a;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(x[c]) : "v"(y[c]));
    }
  }
  double s = b;
  for (int c = 0; c < 8; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*KF)(double*, double, double);
int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount, waves_per_simd = 8, blocks = cus * waves_per_simd, threads = 256;
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  // clock: s_memrealtime is 100 MHz; the shader clock from a long f64 chain is not needed:
  // report cycles at the nominal 2.4 GHz (the clock holds 2.40 GHz under load)
  struct { const char* n; KF f; } ks[] = {
      {"v_fma_f64 v,v,v", k_fma_vvv}, {"v_fma_f64 v,s,v", k_fma_vsv}, {"v_fma_f64 v,s,s", k_fma_vss},
      {"v_fma_f64 v,v,const", k_fma_vvk}, {"v_fmac_f64 v,v", k_fmac_vv}, {"v_mul_f64 v,v", k_mul_vv},
      {"v_mul_f64 v,s", k_mul_vs}, {"v_add_f64 v,v", k_add_vv}, {"v_add_f64 v,const", k_add_vk},
      {"v_cvt_f32_f64", k_cvt_n}, {"v_cvt_f64_f32", k_cvt_w}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001, 0.999999);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001, 0.999999);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // per SIMD: waves_per_simd waves x ITERS x 32 instructions
      const double instr = (double)waves_per_simd * ITERS * 32;
      if (rep) printf("%-24s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", k.n, ms,
                      ms * 1e-3 * 2.4e9 / instr);
    }
  return 0;
}
