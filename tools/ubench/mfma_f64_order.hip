// In what order does v_mfma_f64_4x4x4_4b_f64 sum its four products? mfcc.js:85-93 sums the DCT as a sequential
// double chain (v += dct[n] * lm[n], n ascending; a product of two floats is exact in double, so each step is one
// FMA). If the matrix core adds the k = 0..3 products to C one FMA after another in k order, a chain of MFMA steps
// over ascending band quartets IS the reference's sequential sum, and the reference-order MFCC can use the matrix
// cores for its DCT. Random operands with cancellation (products of two floats, as in the DCT), STEPS chained
// instructions; each output compared bit for bit with host emulations of candidate orders.
// Lane layout (tools/ubench/mfma_f64_4x4_layout.hip): A[i][k] of block g at lane 16k + 4g + i, B[k][j] at
// 16k + 4g + j, D[i][j] at 16i + 4g + j.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>

constexpr int STEPS = 8, TRIALS = 2000;

__global__ void chain(const double* a, const double* b, double* d) {
  const int l = threadIdx.x;
  double acc = 0.0;
  for (int s = 0; s < STEPS; ++s) acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a[s * 64 + l], b[s * 64 + l], acc, 0, 0, 0);
  d[l] = acc;
}

static uint64_t st = 0x9E3779B97F4A7C15ull;
static double rnd() {  // a float32 value in [-4, 4) with a random sign and exponent spread
  st ^= st << 13; st ^= st >> 7; st ^= st << 17;
  const float m = (float)((st >> 40) & 0xFFFFFF) * 0x1p-24f;
  return (double)(((st >> 8) & 1) ? -m : m) * std::ldexp(1.0, (int)((st >> 16) % 8) - 4);
}

int main() {
  double *da, *db, *dd;
  hipMalloc(&da, STEPS * 64 * 8);
  hipMalloc(&db, STEPS * 64 * 8);
  hipMalloc(&dd, 64 * 8);
  static double ha[STEPS * 64], hb[STEPS * 64], hd[64];
  long n = 0, seq = 0, rev = 0, pair = 0;
  for (int t = 0; t < TRIALS; ++t) {
    for (int i = 0; i < STEPS * 64; ++i) { ha[i] = rnd(); hb[i] = rnd(); }
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, da, db, dd);
    hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
    for (int g = 0; g < 4; ++g)
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          double s1 = 0, s2 = 0, s3 = 0;
          for (int s = 0; s < STEPS; ++s) {
            double p[4];
            for (int k = 0; k < 4; ++k) p[k] = ha[s * 64 + 16 * k + 4 * g + i] * hb[s * 64 + 16 * k + 4 * g + j];  // exact
            for (int k = 0; k < 4; ++k) s1 = s1 + p[k];            // sequential, k ascending (the reference's order)
            for (int k = 3; k >= 0; --k) s2 = s2 + p[k];           // k descending
            s3 = s3 + ((p[0] + p[1]) + (p[2] + p[3]));             // pairwise tree, then C
          }
          const double got = hd[16 * i + 4 * g + j];
          ++n;
          seq += got == s1;
          rev += got == s2;
          pair += got == s3;
        }
  }
  printf("%ld outputs of %d chained MFMAs: equal to k-ascending sequential %ld, k-descending %ld, pairwise tree %ld\n", n,
         STEPS, seq, rev, pair);
  return 0;
}
