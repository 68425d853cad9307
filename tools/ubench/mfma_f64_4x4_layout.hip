// Lane layout of v_mfma_f64_4x4x4_4b_f64 (__builtin_amdgcn_mfma_f64_4x4x4f64), measured with
// one-hot operands: for each probe p, A = e_p (lane p holds 1) with B[l] = l + 1, and
// B = e_p with A[l] = l + 1; D = A x B, C = 0. Prints the nonzero outputs of every probe.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double* outA, double* outB) {
  const int l = threadIdx.x;
  for (int p = 0; p < 64; ++p) {
    double a = (l == p) ? 1.0 : 0.0, b = l + 1.0;
    outA[p * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    a = l + 1.0;
    b = (l == p) ? 1.0 : 0.0;
    outB[p * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  }
}

int main() {
  double *a, *b;
  hipMalloc(&a, 64 * 64 * 8);
  hipMalloc(&b, 64 * 64 * 8);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, a, b);
  static double ha[4096], hb[4096];
  hipMemcpy(ha, a, sizeof ha, hipMemcpyDeviceToHost);
  hipMemcpy(hb, b, sizeof hb, hipMemcpyDeviceToHost);
  for (int p = 0; p < 64; ++p) {
    printf("A-onehot lane %2d ->", p);
    for (int l = 0; l < 64; ++l) if (ha[p * 64 + l] != 0) printf(" D[%d]=%g", l, ha[p * 64 + l]);
    printf("\n");
  }
  for (int p = 0; p < 64; ++p) {
    printf("B-onehot lane %2d ->", p);
    for (int l = 0; l < 64; ++l) if (hb[p * 64 + l] != 0) printf(" D[%d]=%g", l, hb[p * 64 + l]);
    printf("\n");
  }
  return 0;
}
