/*
 * meyda_oracle.c — CPU restatement of the meyda per-frame hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The
 * product path (libmeyda_gpu.so) never links or calls it.
 *
 * It restates, in plain C with JavaScript number semantics (IEEE double, no FMA
 * contraction: built with -ffp-contract=off), the reference algorithm:
 *   window        src/meyda.js:158-168      (+ tables :116-138)
 *   FFT           lib/jsfft/fft.js:123-208  (radix-2 DIT, bit reversal, f64
 *                 butterflies, Float32Array storage between stages,
 *                 lib/jsfft/complex_array.js:7,22-36)
 *   amplitude     src/meyda.js:104-114
 *   bark scale    src/meyda.js:170-182
 *   extractors    src/extractors/NAME.js (file:line at each function below)
 * Parity of this restatement is pinned by tests/golden/ (generated from the
 * reference itself by tools/gen_golden.js; see tests/test_oracle_golden.py).
 *
 * Transcendentals come from glibc (V8 uses fdlibm ports); the golden tests
 * check every host table bit-for-bit, and the feature tolerances absorb the
 * rare last-ulp differences in pow/log/exp.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_NUM_SCALARS 13
#define ORACLE_NUM_BARK 24
#define ORACLE_NUM_COEFFS 13

enum { OR_RMS, OR_ENERGY, OR_ZCR, OR_CENTROID, OR_FLATNESS, OR_SLOPE, OR_ROLLOFF,
       OR_SPREAD, OR_SKEWNESS, OR_KURTOSIS, OR_LOUDNESS_TOTAL, OR_PSPREAD, OR_PSHARP };

static const double JS_PI = 3.141592653589793;        /* Math.PI */
static const double JS_SQRT1_2 = 0.7071067811865476;  /* Math.SQRT1_2 */

/* src/utils.js:13-19 */
int oracle_is_power_of_two(double num) {
  while (fmod(num, 2.0) == 0.0 && num > 1) num /= 2;
  return num == 1;
}

/* src/meyda.js:128-138 (symmetric hann, note the N-1) */
void oracle_hanning(int n, float* out) {
  for (int i = 0; i < n; i++) out[i] = (float)(0.5 - 0.5 * cos(2 * JS_PI * i / (n - 1)));
}

/* src/meyda.js:116-126 (the "- 1" is kept literally) */
void oracle_hamming(int n, float* out) {
  for (int i = 0; i < n; i++) out[i] = (float)(0.54 - 0.46 * cos(2 * JS_PI * ((double)i / n - 1)));
}

/* src/meyda.js:170-182: the frequency is stored to a Float32Array and read back. */
void oracle_bark_scale(int n, double sr, float* out) {
  for (int i = 0; i < n; i++) {
    float f = (float)((double)i * sr / n);
    double q = (double)f / 7518;
    out[i] = (float)(13 * atan((double)f / 1315.8) + 3.5 * atan(q * q));
  }
}

/* src/extractors/loudness.js:24-45 */
void oracle_bark_band_limits(const float* bark, int spec_len, int nbands, int32_t* lim) {
  double band_end = (double)bark[spec_len - 1] / nbands;
  int band = 1;
  for (int i = 0; i <= nbands; i++) lim[i] = 0;
  for (int i = 0; i < spec_len; i++) {
    while ((double)bark[i] > band_end) {
      if (band <= nbands) lim[band] = i; /* typed-array write out of range is a no-op in JS */
      band++;
      band_end = (double)band * bark[spec_len - 1] / nbands;
    }
  }
  lim[nbands] = spec_len - 1;
}

/* src/extractors/mfcc.js:7-38: mel edges stored to Float32Arrays, then bins. */
void oracle_mel_bins(int n, double sr, int nfilt, int32_t* bins, float* mel_values, float* mel_freq) {
  double lo = 1125 * log(1 + (0.0 / 700));
  double hi = 1125 * log(1 + ((sr / 2) / 700));
  double step = (hi - lo) / (nfilt + 1);
  for (int i = 0; i < nfilt + 2; i++) {
    float mv = (float)(i * step);
    float mf = (float)(700 * (exp((double)mv / 1125) - 1));
    if (mel_values) mel_values[i] = mv;
    if (mel_freq) mel_freq[i] = mf;
    bins[i] = (int32_t)floor((double)(n + 1) * mf / sr);
  }
}

/* src/extractors/mfcc.js:67-83: dct[i + j*13] */
void oracle_dct(int nfilt, float* dct) {
  double k = JS_PI / nfilt, w1 = 1.0 / sqrt((double)nfilt), w2 = sqrt(2.0 / nfilt);
  for (int i = 0; i < ORACLE_NUM_COEFFS; i++)
    for (int j = 0; j < nfilt; j++)
      dct[i + j * ORACLE_NUM_COEFFS] = (float)((i == 0 ? w1 : w2) * cos(k * (i + 1) * (j + 0.5)));
}

/* src/extractors/mfcc.js:40-51: weight of filter j at bin i (0 outside). */
static double mel_weight(const int32_t* b, int j, int i) {
  if (i >= b[j] && i < b[j + 1]) return (double)(i - b[j]) / (b[j + 1] - b[j]);
  if (i >= b[j + 1] && i < b[j + 2]) return (double)(b[j + 2] - i) / (b[j + 2] - b[j + 1]);
  return 0.0;
}

/* lib/jsfft/fft.js:173-183 */
static int bit_reverse(int index, int n) {
  int r = 0;
  while (n > 1) { r = (r << 1) + (index & 1); index >>= 1; n >>= 1; }
  return r;
}

/* jsfft: del_f per stage (fft.js:144-145), exposed for the host-table test. */
void oracle_twiddle_seeds(int n, double* out) {
  int s = 0;
  for (int w = 1; w < n; w <<= 1, s++) { out[2 * s] = cos(JS_PI / w); out[2 * s + 1] = sin(JS_PI / w); }
}

/* lib/jsfft/fft.js:123-171 + :185-208, in place on Float32 storage. */
void oracle_jsfft(float* re, float* im, int n) {
  for (int i = 0; i < n; i++) {               /* BitReverseComplexArray: each pair swapped once */
    int r = bit_reverse(i, n);
    if (r > i) {
      float t = re[r]; re[r] = re[i]; re[i] = t;
      t = im[r]; im[r] = im[i]; im[i] = t;
    }
  }
  for (int width = 1; width < n; width <<= 1) {
    double del_r = cos(JS_PI / width), del_i = sin(JS_PI / width);
    for (int i = 0; i < n / (2 * width); i++) {
      double f_r = 1, f_i = 0;
      for (int j = 0; j < width; j++) {
        int l = 2 * i * width + j, r = l + width;
        double left_r = re[l], left_i = im[l];
        double right_r = f_r * re[r] - f_i * im[r];
        double right_i = f_i * re[r] + f_r * im[r];
        re[l] = (float)(JS_SQRT1_2 * (left_r + right_r));
        im[l] = (float)(JS_SQRT1_2 * (left_i + right_i));
        re[r] = (float)(JS_SQRT1_2 * (left_r - right_r));
        im[r] = (float)(JS_SQRT1_2 * (left_i - right_i));
        double temp = f_r * del_r - f_i * del_i;
        f_i = f_r * del_i + f_i * del_r;
        f_r = temp;
      }
    }
  }
}

/* src/utils.js:1-11 (k^p is exact in double for the sizes used) */
static double mu(int p, const float* a, int len) {
  double num = 0, den = 0;
  for (int k = 0; k < len; k++) {
    double kp = 1;
    for (int q = 0; q < p; q++) kp *= k;
    num += kp * fabs((double)a[k]);
    den += a[k];
  }
  return num / den;
}

typedef struct {
  int n, nfilt;
  double sr;
  const float* window;   /* n */
  const int32_t* bblim;  /* 25 */
  const int32_t* melb;   /* nfilt + 2 */
  const float* dct;      /* 13 * nfilt */
  double sharp_tail[ORACLE_NUM_BARK];
} oracle_ctx;

/* One frame. Any output pointer may be NULL. */
static void oracle_frame(const oracle_ctx* c, const float* x, int literal, float* amp_out,
                         float* cre, float* cim, double* sc, float* loud_spec, float* mfcc_out,
                         float* work, const float* amp_in) {
  const int n = c->n, L = n / 2;
  float* re = work;          /* n */
  float* im = work + n;      /* n */
  float* amp = work + 2 * n; /* L */
  if (amp_in) {
    memcpy(amp, amp_in, sizeof(float) * L); /* features of a given spectrum (test helper) */
  } else {
    /* src/meyda.js:158-168: windowed[i] = sig[i] * w[i] stored to Float32Array */
    for (int i = 0; i < n; i++) { re[i] = (float)((double)x[i] * c->window[i]); im[i] = 0.0f; }
    if (!literal) oracle_jsfft(re, im, n); /* literal: the snapshot never transforms per buffer */
    /* src/meyda.js:104-114 */
    for (int i = 0; i < L; i++) {
      double r = re[i], q = im[i];
      amp[i] = (float)sqrt(r * r + q * q);
    }
    if (amp_out) memcpy(amp_out, amp, sizeof(float) * L);
    if (cre) memcpy(cre, re, sizeof(float) * n);
    if (cim) memcpy(cim, im, sizeof(float) * n);
  }
  if (!sc && !loud_spec && !mfcc_out) return;

  double s[ORACLE_NUM_SCALARS];
  /* rms.js:1-11 and energy.js:1-7 (Math.pow(v,2) == v*v in V8/fdlibm) */
  double e = 0;
  for (int i = 0; i < n; i++) e += (double)x[i] * x[i];
  s[OR_ENERGY] = e;
  s[OR_RMS] = sqrt(e / n);
  /* zcr.js:1-9: signal[n] is undefined, so the last pair never counts; -0 >= 0 */
  int z = 0;
  for (int i = 0; i + 1 < n; i++)
    if ((x[i] >= 0 && x[i + 1] < 0) || (x[i] < 0 && x[i + 1] >= 0)) z++;
  s[OR_ZCR] = z;
  /* spectralCentroid.js:1-3, spectralSpread.js:1-4, spectralSkewness.js:1-9, spectralKurtosis.js:1-10 */
  double m1 = mu(1, amp, L), m2 = mu(2, amp, L), m3 = mu(3, amp, L), m4 = mu(4, amp, L);
  s[OR_CENTROID] = m1;
  s[OR_SPREAD] = sqrt(m2 - m1 * m1);
  s[OR_SKEWNESS] = (2 * pow(m1, 3) - 3 * m1 * m2 + m3) / pow(sqrt(m2 - m1 * m1), 3);
  s[OR_KURTOSIS] = (-3 * pow(m1, 4) + 6 * m1 * m2 - 4 * m1 * m3 + m4) / pow(sqrt(m2 - m1 * m1), 4);
  /* spectralFlatness.js:1-10 */
  double ln = 0, den = 0;
  for (int i = 0; i < L; i++) { ln += log((double)amp[i]); den += amp[i]; }
  s[OR_FLATNESS] = exp(ln / L) * L / den;
  /* spectralSlope.js:1-18 (denominator as written, without the L factor) */
  double ampSum = 0, freqSum = 0, powFreqSum = 0, ampFreqSum = 0;
  for (int i = 0; i < L; i++) {
    ampSum += amp[i];
    double f = (double)i * c->sr / n;
    powFreqSum += f * f;
    freqSum += f;
    ampFreqSum += f * amp[i];
  }
  s[OR_SLOPE] = (L * ampFreqSum - freqSum * ampSum) / (ampSum * (powFreqSum - freqSum * freqSum));
  /* spectralRolloff.js:1-16 */
  double nyq = c->sr / (2.0 * (L - 1));
  double ec = 0;
  for (int i = 0; i < L; i++) ec += amp[i];
  double thr = 0.99 * ec;
  int k = L - 1;
  while (ec > thr && k >= 0) { ec -= amp[k]; --k; }
  s[OR_ROLLOFF] = (k + 1) * nyq;
  /* loudness.js:47-96 */
  float spec[ORACLE_NUM_BARK];
  for (int b = 0; b < ORACLE_NUM_BARK; b++) {
    double sum = 0;
    for (int j = c->bblim[b]; j < c->bblim[b + 1]; j++) sum += amp[j];
    spec[b] = (float)pow(sum, 0.23);
  }
  double total = 0;
  for (int b = 0; b < ORACLE_NUM_BARK; b++) total += spec[b];
  s[OR_LOUDNESS_TOTAL] = total;
  if (loud_spec) memcpy(loud_spec, spec, sizeof spec);
  /* perceptualSpread.js:1-14 */
  double mx = 0;
  for (int b = 0; b < ORACLE_NUM_BARK; b++) if (spec[b] > mx) mx = spec[b];
  double ps = (total - mx) / total;
  s[OR_PSPREAD] = ps * ps;
  /* perceptualSharpness.js:1-16 (spec[i+1] off-by-one and constant tail as written) */
  double out = 0;
  for (int i = 0; i < ORACLE_NUM_BARK; i++) out += (i < 15) ? (i + 1) * (double)spec[i + 1] : c->sharp_tail[i];
  out *= 0.11 / total;
  s[OR_PSHARP] = out;
  if (sc) memcpy(sc, s, sizeof s);

  if (mfcc_out) {
    /* mfcc.js:53-65: Float32Array accumulator, double products, ascending bins */
    float lm[64];
    for (int b = 0; b < c->nfilt; b++) {
      float acc = 0.0f;
      for (int j = 0; j < L; j++) {
        float p = (float)((double)amp[j] * amp[j]); /* powerSpectrum.js:1-7 */
        double w = mel_weight(c->melb, b, j);
        acc = (float)((double)acc + w * p);
      }
      lm[b] = (float)log((double)acc);
    }
    /* mfcc.js:85-93 */
    for (int q = 0; q < ORACLE_NUM_COEFFS; q++) {
      double v = 0;
      for (int b = 0; b < c->nfilt; b++) v += (double)c->dct[q + b * ORACLE_NUM_COEFFS] * lm[b];
      mfcc_out[q] = (float)(v / ORACLE_NUM_COEFFS);
    }
  }
}

/*
 * Batch entry point. frames: F x n (row-major). window: 0 = hanning, 1 = hamming.
 * Outputs (each may be NULL): amp F x n/2, cre/cim F x n, scalars F x 13 (record
 * order above), loud_spec F x 24, mfcc F x 13. literal != 0 reproduces the
 * snapshot's onaudioprocess (no per-buffer FFT). Returns 0, or -1 on bad input.
 * Thread-safe: callers may run disjoint frame ranges concurrently. amp_in (optional, F x n/2)
 * replaces the window+FFT+amplitude steps (used to isolate feature parity in tests).
 */
int oracle_extract_ex(const float* frames, const float* amp_in, long nframes, int n, double sr,
                      int window, int nfilt, int literal, float* amp, float* cre, float* cim,
                      double* scalars, float* loud_spec, float* mfcc) {
  if (!oracle_is_power_of_two(n) || n < 4 || nfilt < 1 || nfilt > 64) return -1;
  const int L = n / 2;
  float* win = malloc(sizeof(float) * n);
  float* bark = malloc(sizeof(float) * n);
  float* dct = malloc(sizeof(float) * ORACLE_NUM_COEFFS * nfilt);
  float* work = malloc(sizeof(float) * (2 * n + L));
  int32_t bbl[ORACLE_NUM_BARK + 1], melb[66];
  if (!win || !bark || !dct || !work) { free(win); free(bark); free(dct); free(work); return -1; }
  if (window == 1) oracle_hamming(n, win); else oracle_hanning(n, win);
  oracle_bark_scale(n, sr, bark);
  oracle_bark_band_limits(bark, L, ORACLE_NUM_BARK, bbl);
  oracle_mel_bins(n, sr, nfilt, melb, NULL, NULL);
  oracle_dct(nfilt, dct);
  oracle_ctx c = { .n = n, .nfilt = nfilt, .sr = sr, .window = win, .bblim = bbl, .melb = melb, .dct = dct };
  for (int i = 0; i < ORACLE_NUM_BARK; i++) c.sharp_tail[i] = 0.066 * exp(0.171 * (i + 1));
  for (long f = 0; f < nframes; f++) {
    oracle_frame(&c, frames + f * n, literal,
                 amp ? amp + f * L : NULL, cre ? cre + f * n : NULL, cim ? cim + f * n : NULL,
                 scalars ? scalars + f * ORACLE_NUM_SCALARS : NULL,
                 loud_spec ? loud_spec + f * ORACLE_NUM_BARK : NULL,
                 mfcc ? mfcc + f * ORACLE_NUM_COEFFS : NULL, work, amp_in ? amp_in + f * L : NULL);
  }
  free(win); free(bark); free(dct); free(work);
  return 0;
}

int oracle_extract(const float* frames, long nframes, int n, double sr, int window, int nfilt,
                   int literal, float* amp, float* cre, float* cim, double* scalars,
                   float* loud_spec, float* mfcc) {
  return oracle_extract_ex(frames, NULL, nframes, n, sr, window, nfilt, literal, amp, cre, cim,
                           scalars, loud_spec, mfcc);
}

/* Features of given amplitude spectra (frames still supply rms/energy/zcr). */
int oracle_features_from_amp(const float* frames, const float* amp_in, long nframes, int n,
                             double sr, int nfilt, double* scalars, float* loud_spec, float* mfcc) {
  return oracle_extract_ex(frames, amp_in, nframes, n, sr, 0, nfilt, 0, NULL, NULL, NULL, scalars,
                           loud_spec, mfcc);
}

/* Synthetic PCM: splitmix64 output for state seed advanced
 * (i+1) times, top 24 bits -> exact f32 in [-1, 1). i = first_index + t. */
void oracle_synth(uint64_t seed, uint64_t first_index, long count, float* out) {
  for (long t = 0; t < count; t++) {
    uint64_t z = seed + (first_index + (uint64_t)t + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    out[t] = (float)((double)(z >> 40) * (1.0 / 8388608.0) - 1.0);
  }
}
