/* Emulates the MFMA mel path: E_j = fmaf chain over ascending k of (float)w_jk * p_k,
 * lm_j = (float)log(E_j), mfcc = (float)(sum_j dct * lm / 13) (double, sequential). */
#include <math.h>
#include <stdint.h>
void oracle_mel_bins(int n, double sr, int nfilt, int32_t* bins, float* mv, float* mf);
void oracle_dct(int nfilt, float* dct);
static double wt(const int32_t* b, int j, int i) {
  if (i >= b[j] && i < b[j + 1]) return (double)(i - b[j]) / (b[j + 1] - b[j]);
  if (i >= b[j + 1] && i < b[j + 2]) return (double)(b[j + 2] - i) / (b[j + 2] - b[j + 1]);
  return 0.0;
}
void emu_mfcc_mfma(const float* amp, long F, int n, int nfilt, float* out) {
  int32_t b[70]; float dct[13 * 64];
  oracle_mel_bins(n, 44100.0, nfilt, b, 0, 0);
  oracle_dct(nfilt, dct);
  int L = n / 2;
  for (long f = 0; f < F; f++) {
    const float* a = amp + f * L;
    float lm[64];
    for (int j = 0; j < nfilt; j++) {
      float acc = 0.0f;
      for (int k = 0; k < L; k++) { float p = a[k] * a[k]; acc = fmaf((float)wt(b, j, k), p, acc); }
      lm[j] = (float)log((double)acc);
    }
    for (int c = 0; c < 13; c++) {
      double v = 0; for (int j = 0; j < nfilt; j++) v += (double)dct[c + j * 13] * lm[j];
      out[f * 13 + c] = (float)(v / 13);
    }
  }
}
