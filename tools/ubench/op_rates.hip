// Microbenchmark: issue cost (SIMD cycles per wave64 instruction) of the VALU operations the
// faithful FFT and the feature reductions are built from, on gfx950. 8 waves per SIMD, 8
// independent chains per lane, instructions pinned by inline asm. Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -o op_rates tools/ubench/op_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

// f64 -> f64 ops, one operand chained
#define K64(name, ASM)                                                              \
  __global__ void name(double* out, double a, double b) {                           \
    double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, \
           x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                   \
    for (int i = 0; i < ITERS; ++i) {                                               \
      _Pragma("unroll") for (int u = 0; u < 4; ++u) {                               \
        asm volatile(ASM : "+v"(x0) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x1) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x2) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x3) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x4) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x5) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x6) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x7) : "v"(a), "v"(b));                              \
      }                                                                             \
    }                                                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7; \
  }
#define K32(name, ASM)                                                              \
  __global__ void name(double* out, float a, float b) {                             \
    float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, \
          x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                    \
    for (int i = 0; i < ITERS; ++i) {                                               \
      _Pragma("unroll") for (int u = 0; u < 4; ++u) {                               \
        asm volatile(ASM : "+v"(x0) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x1) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x2) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x3) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x4) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x5) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x6) : "v"(a), "v"(b));                              \
        asm volatile(ASM : "+v"(x7) : "v"(a), "v"(b));                              \
      }                                                                             \
    }                                                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7; \
  }
typedef float f2 __attribute__((ext_vector_type(2)));
#define KPK(name, ASM)                                                              \
  __global__ void name(double* out, float a, float b) {                             \
    f2 x0 = {threadIdx.x * 1e-3f, 1}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, \
       x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                       \
    f2 av = {a, a}, bv = {b, b};                                                    \
    for (int i = 0; i < ITERS; ++i) {                                               \
      _Pragma("unroll") for (int u = 0; u < 4; ++u) {                               \
        asm volatile(ASM : "+v"(x0) : "v"(av), "v"(bv));                            \
        asm volatile(ASM : "+v"(x1) : "v"(av), "v"(bv));                            \
        asm volatile(ASM : "+v"(x2) : "v"(av), "v"(bv));                            \
        asm volatile(ASM : "+v"(x3) : "v"(av), "v"(bv));                            \
        asm volatile(ASM : "+v"(x4) : "v"(av), "v"(bv));                            \
        asm volatile(ASM : "+v"(x5) : "v"(av), "v"(bv));                            \
        asm volatile(ASM : "+v"(x6) : "v"(av), "v"(bv));                            \
        asm volatile(ASM : "+v"(x7) : "v"(av), "v"(bv));                            \
      }                                                                             \
    }                                                                               \
    f2 s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;                         \
  }

K64(k_fma64, "v_fma_f64 %0, %0, %1, %2")
K64(k_mul64, "v_mul_f64 %0, %0, %1")
K64(k_add64, "v_add_f64 %0, %0, %1")
K64(k_rsq64, "v_rsq_f64 %0, %0")
K64(k_sqrt64, "v_sqrt_f64 %0, %0")
K64(k_rcp64, "v_rcp_f64 %0, %0")
K32(k_fma32, "v_fma_f32 %0, %0, %1, %2")
K32(k_add32, "v_add_f32 %0, %0, %1")
K32(k_rsq32, "v_rsq_f32 %0, %0")
K32(k_log32, "v_log_f32 %0, %0")
K32(k_cnd, "v_cndmask_b32 %0, %0, %1, vcc")
K32(k_dpp, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
KPK(k_pkfma, "v_pk_fma_f32 %0, %0, %1, %2")
KPK(k_pkmul, "v_pk_mul_f32 %0, %0, %1")

// f64 -> f32 -> f64 round trip (the per-stage float32 store of the faithful FFT): 2 instructions
__global__ void k_cvt_rt(double* out, double a, double b) {
  double x[8];
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3 + c + a + b;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float t;
        asm volatile("v_cvt_f32_f64 %1, %0\n v_cvt_f64_f32 %0, %1" : "+v"(x[c]), "=&v"(t));
      }
    }
  }
  double s = 0;
  for (int c = 0; c < 8; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_cndmask_b32_e64 with the lane mask in an SGPR pair from a ballot (the kernel's form)
__global__ void k_cnd64(double* out, float a, float b) {
  float x[8];
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3f + c;
  const unsigned long long m = __ballot(threadIdx.x & 1);
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "s"(m));
    }
  }
  float s = b;
  for (int c = 0; c < 8; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Mixed streams: an f64 FMA followed by an f32 FMA on independent chains (can f32 work
// fill f64 issue gaps?)
__global__ void k_mix(double* out, double a, double b) {
  double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  float y0 = threadIdx.x * 1e-3f, y1 = y0 + 1, y2 = y0 + 2, y3 = y0 + 3;
  float af = (float)a, bf = (float)b;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x0) : "v"(a), "v"(b));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(y0) : "v"(af), "v"(bf));
      asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x1) : "v"(a), "v"(b));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(y1) : "v"(af), "v"(bf));
      asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x2) : "v"(a), "v"(b));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(y2) : "v"(af), "v"(bf));
      asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x3) : "v"(a), "v"(b));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(y3) : "v"(af), "v"(bf));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + y0 + y1 + y2 + y3;
}


// Matrix-core f64: issue cost of v_mfma_f64_16x16x4_f64 / v_mfma_f64_4x4x4_4b_f64 (4
// independent accumulators), and whether f64 MFMA work overlaps VALU f64 FMAs: MODE 0 =
// MFMA only, 1 = VALU only, 2 = both interleaved in each wave, 3 = half the waves each.
typedef double d4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ void k_mm(double* out, double a, double b) {
  d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
         x6 = x0 + 6, x7 = x0 + 7;
  const double av = a + threadIdx.x * 1e-9;
  const bool mm = MODE == 0 || MODE == 2 || (MODE == 3 && (threadIdx.x & 64));
  const bool vv = MODE == 1 || MODE == 2 || (MODE == 3 && !(threadIdx.x & 64));
  for (int i = 0; i < ITERS; ++i) {
    if (mm) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b, acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b, acc3, 0, 0, 0);
    }
    if (vv) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x0) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x1) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x2) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x3) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x4) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x5) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x6) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x7) : "v"(a), "v"(b));
      }
    }
  }
  const d4 s = acc0 + acc1 + acc2 + acc3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + s.z + s.w + x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}
__global__ void k_mm4(double* out, double a, double b) {
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const double av = a + threadIdx.x * 1e-9;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(av, b, acc[u], 0, 0, 0);
  }
  double s = 0;
  for (int u = 0; u < 8; ++u) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Clock: s_memtime ticks per s_memrealtime tick (100 MHz) over a long spin.
__global__ void k_clock(unsigned long long* out) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double x = threadIdx.x;
  for (int i = 0; i < 200000; ++i) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(x));
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
  if (x == 12345.0) out[0] = 0;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8, threads = 256;  // 32 waves per CU = 8 per SIMD
  double* d;
  hipMalloc(&d, sizeof(double) * blocks * threads);
  unsigned long long* c;
  hipMalloc(&c, sizeof(unsigned long long) * 2 * cus);
  hipLaunchKernelGGL(k_clock, dim3(cus), dim3(64), 0, 0, c);
  hipDeviceSynchronize();
  unsigned long long hc[2];
  hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
  const double ghz = (double)hc[0] / (double)hc[1] * 0.1;
  printf("CUs %d, shader clock (memtime/realtime) %.3f GHz\n", cus, ghz);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct T { const char* n; void (*k64)(double*, double, double); void (*k32)(double*, float, float); int per; };
  T ts[] = {
      {"v_fma_f64", k_fma64, nullptr, 1},   {"v_mul_f64", k_mul64, nullptr, 1},
      {"v_add_f64", k_add64, nullptr, 1},   {"v_rsq_f64", k_rsq64, nullptr, 1},
      {"v_sqrt_f64", k_sqrt64, nullptr, 1}, {"v_rcp_f64", k_rcp64, nullptr, 1},
      {"cvt f64->f32->f64 (2 instr)", k_cvt_rt, nullptr, 2},
      {"mix f64 fma + f32 fma (2 instr)", k_mix, nullptr, 2},
      {"v_fma_f32", nullptr, k_fma32, 1},   {"v_add_f32", nullptr, k_add32, 1},
      {"v_rsq_f32", nullptr, k_rsq32, 1},   {"v_log_f32", nullptr, k_log32, 1},
      {"v_cndmask_b32 (vcc)", nullptr, k_cnd, 1}, {"v_cndmask_b32_e64 (sgpr mask)", nullptr, k_cnd64, 1},
      {"v_mov_b32_dpp", nullptr, k_dpp, 1},
      {"v_pk_fma_f32", nullptr, k_pkfma, 1}, {"v_pk_mul_f32", nullptr, k_pkmul, 1},
  };
  for (int rep = 0; rep < 2; ++rep) {
    for (auto& t : ts) {
      hipEventRecord(e0);
      if (t.k64) hipLaunchKernelGGL(t.k64, dim3(blocks), dim3(threads), 0, 0, d, 0.999, 1e-3);
      else hipLaunchKernelGGL(t.k32, dim3(blocks), dim3(threads), 0, 0, d, 0.999f, 1e-3f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // wave-instructions per SIMD
      const double wi = (double)blocks * threads / 64 * ITERS * 32 / (cus * 4.0);
      const double cyc = ms * 1e-3 * ghz * 1e9 / (wi * t.per);
      if (rep == 1) printf("%-34s %8.3f ms  %6.2f cycles per wave-instruction per SIMD\n", t.n, ms, cyc);
    }
  }
  {
    const double wpsimd = (double)blocks * threads / 64 / (cus * 4.0);  // waves per SIMD
    struct M { const char* n; void (*k)(double*, double, double); double mf, va; };
    // per wave: MFMA count, VALU f64 FMA count (MODE 3: half the waves each)
    M ms[] = {{"mfma16 only (4/iter)", k_mm<0>, 4, 0}, {"fma64 only (32/iter)", k_mm<1>, 0, 32},
              {"mfma16 + fma64 in each wave", k_mm<2>, 4, 32}, {"half waves mfma16, half fma64", k_mm<3>, 2, 16},
              {"mfma_f64_4x4x4 only (8/iter)", k_mm4, 8, 0}};
    for (int rep = 0; rep < 2; ++rep) {
      for (auto& t : ms) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(t.k, dim3(blocks), dim3(threads), 0, 0, d, 0.999, 1e-3);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float msv;
        hipEventElapsedTime(&msv, e0, e1);
        const double cyc = msv * 1e-3 * ghz * 1e9;  // per SIMD
        if (rep == 1)
          printf("%-34s %8.3f ms  %9.0f cycles per SIMD; %.2f cycles per MFMA if alone, %.2f per fma64 if alone\n",
                 t.n, msv, cyc, t.mf ? cyc / (wpsimd * ITERS * t.mf) : 0.0, t.va ? cyc / (wpsimd * ITERS * t.va) : 0.0);
      }
    }
  }
  return 0;
}
