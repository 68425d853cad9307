// Lane layout of v_mfma_f32_4x4x1_16b_f32 (__builtin_amdgcn_mfma_f32_4x4x1f32), measured with
// one-hot operands: for each probe lane p, A = e_p with B[l] = l + 1, and B = e_p with
// A[l] = l + 1; C = 0. D has 4 VGPRs per lane; prints (lane, vgpr) = value of the nonzero outputs,
// and a chained check that C accumulates: D2 = A x B + D1.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void probe(float* outA, float* outB, float* outC) {
  const int l = threadIdx.x;
  for (int p = 0; p < 64; ++p) {
    const v4f z = {0.f, 0.f, 0.f, 0.f};
    v4f d = __builtin_amdgcn_mfma_f32_4x4x1f32((l == p) ? 1.0f : 0.0f, l + 1.0f, z, 0, 0, 0);
    for (int r = 0; r < 4; ++r) outA[(p * 64 + l) * 4 + r] = d[r];
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(l + 1.0f, (l == p) ? 1.0f : 0.0f, z, 0, 0, 0);
    for (int r = 0; r < 4; ++r) outB[(p * 64 + l) * 4 + r] = d[r];
  }
  const v4f z = {0.f, 0.f, 0.f, 0.f};
  v4f d = __builtin_amdgcn_mfma_f32_4x4x1f32(1.0f, l + 1.0f, z, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_4x4x1f32(2.0f, l + 1.0f, d, 0, 0, 0);
  for (int r = 0; r < 4; ++r) outC[l * 4 + r] = d[r];
}

int main() {
  float *a, *b, *c;
  hipMalloc(&a, 64 * 64 * 4 * 4);
  hipMalloc(&b, 64 * 64 * 4 * 4);
  hipMalloc(&c, 64 * 4 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, a, b, c);
  static float ha[64 * 64 * 4], hb[64 * 64 * 4], hc[64 * 4];
  hipMemcpy(ha, a, sizeof ha, hipMemcpyDeviceToHost);
  hipMemcpy(hb, b, sizeof hb, hipMemcpyDeviceToHost);
  hipMemcpy(hc, c, sizeof hc, hipMemcpyDeviceToHost);
  for (int p = 0; p < 64; ++p) {
    printf("A-onehot lane %2d ->", p);
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r)
        if (ha[(p * 64 + l) * 4 + r] != 0) printf(" D[l%d,v%d]=%g", l, r, ha[(p * 64 + l) * 4 + r]);
    printf("\n");
  }
  for (int p = 0; p < 64; ++p) {
    printf("B-onehot lane %2d ->", p);
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r)
        if (hb[(p * 64 + l) * 4 + r] != 0) printf(" D[l%d,v%d]=%g", l, r, hb[(p * 64 + l) * 4 + r]);
    printf("\n");
  }
  printf("accumulate (A=1 then A=2, B=l+1):");
  for (int l = 0; l < 8; ++l) printf(" l%d:(%g %g %g %g)", l, hc[l * 4], hc[l * 4 + 1], hc[l * 4 + 2], hc[l * 4 + 3]);
  printf("\n");
  return 0;
}
