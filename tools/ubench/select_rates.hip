// Microbenchmark: issue cost of per-lane selects on gfx950 (8 waves per SIMD, 8 independent
// chains per lane): v_cndmask_b32 with the lane mask in an SGPR pair (e64) or in VCC (e32),
// v_bfi_b32 with the mask in a VGPR, v_perm_b32, and v_fma_f32 / v_xor_b32 / v_and_or_b32 for
// reference. Not part of the product. Build: hipcc --offload-arch=gfx950 -O3 -o select_rates tools/ubench/select_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define K(name, SETUP, ASM, ...)                                                          \
  __global__ void name(double* out, float a, float b) {                                   \
    float x[8];                                                                           \
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3f + c;                           \
    const unsigned long long m = __ballot(threadIdx.x & 1);                               \
    const unsigned vm = (threadIdx.x & 1) ? 0xFFFFFFFFu : 0u;                             \
    (void)m; (void)vm;                                                                    \
    SETUP;                                                                                \
    for (int i = 0; i < ITERS; ++i) {                                                     \
      _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                     \
        _Pragma("unroll") for (int c = 0; c < 8; ++c) asm volatile(ASM : "+v"(x[c]) : __VA_ARGS__); \
      }                                                                                   \
    }                                                                                     \
    float s = b;                                                                          \
    for (int c = 0; c < 8; ++c) s += x[c];                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                       \
  }

K(k_cnd_e64, , "v_cndmask_b32_e64 %0, %0, %1, %2", "v"(a), "s"(m))
K(k_cnd_e32, asm volatile("s_mov_b64 vcc, %0" ::"s"(m) : "vcc"), "v_cndmask_b32_e32 %0, %0, %1, vcc", "v"(a))
K(k_bfi, , "v_bfi_b32 %0, %1, %0, %2", "v"(vm), "v"(a))
K(k_perm, , "v_perm_b32 %0, %0, %1, %2", "v"(a), "v"(vm))
K(k_fma32, , "v_fma_f32 %0, %0, %1, %2", "v"(a), "v"(b))
K(k_xor, , "v_xor_b32 %0, %0, %1", "v"(vm))
K(k_andor, , "v_and_or_b32 %0, %0, %1, %2", "v"(vm), "v"(a))
K(k_bitop3, , "v_bitop3_b32 %0, %1, %0, %2 bitop3:0xd8", "v"(vm), "v"(a))
K(k_cnd_e64vcc, asm volatile("s_mov_b64 vcc, %0" ::"s"(m) : "vcc"), "v_cndmask_b32_e64 %0, %0, %1, vcc", "v"(a))
// the compiler's pattern: a compare writes the mask, a select reads it (2 instructions per chain step)
K(k_cmp_cnd_vcc, , "v_cmp_gt_f32_e32 vcc, %0, %1\n v_cndmask_b32_e32 %0, %0, %1, vcc", "v"(a))
K(k_cmp_cnd_sgpr, , "v_cmp_gt_f32_e64 s[40:41], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[40:41]", "v"(a))

typedef void (*KF)(double*, float, float);
int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8, threads = 256;
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  struct { const char* n; KF f; } ks[] = {{"v_cndmask_b32_e64 (sgpr)", k_cnd_e64}, {"v_cndmask_b32_e32 (vcc)", k_cnd_e32},
      {"v_bfi_b32 (vgpr mask)", k_bfi}, {"v_perm_b32", k_perm}, {"v_fma_f32", k_fma32}, {"v_xor_b32", k_xor},
      {"v_and_or_b32", k_andor}, {"v_bitop3_b32", k_bitop3}, {"v_cndmask_b32_e64 (vcc)", k_cnd_e64vcc},
      {"cmp+cndmask via vcc (x2 instr)", k_cmp_cnd_vcc}, {"cmp+cndmask via sgpr (x2 instr)", k_cmp_cnd_sgpr}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001f, 0.999999f);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001f, 0.999999f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr = 8.0 * ITERS * 32;  // per SIMD: 8 waves x ITERS x 32
      if (rep) printf("%-26s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", k.n, ms, ms * 1e-3 * 2.4e9 / instr);
    }
  return 0;
}
