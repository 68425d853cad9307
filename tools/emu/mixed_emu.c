/*
 * CPU emulation of the kernel's faithful FFT arithmetic per pass layout (design validation
 * only, not shipped): which slot pairs run which butterfly form depends on the register
 * geometry (R slots per lane), exactly as kernels.hip run_stage decides it:
 *   pass 0 (stages q < RB): block-start pairs are static -> bfly_special; others generic;
 *   pass P >= 1 (q0 = P*RB): pairs whose register-part location bits [q0, q) are zero are
 *     "mixed" (block-start on the lanes whose low q0 bits are zero, generic elsewhere);
 *     the rest generic.
 * Forms:
 *   generic (fused):  Ar = fma(cx, Rr, -cy Ri), Ai = fma(cx, Ri, cy Rr), c = S f;
 *                     lo = (fma(S, Lr, Ar), fma(S, Li, Ai)), hi = (fma(S, Lr, -Ar), fma(-S, Li, Ai))
 *   special:          lo = (S (L0 + R0), S (L0 - R0)), hi = (fma(S, Lh, Sfx Rh), Sfy Rh)
 *   mode 1 mixed-generic lanes (unscaled f, b = fx, c0 = S fy):
 *                     t1 = fma(b, Rr, Lr), t3 = fma(-b, Rr, Lr), t2 = fma(b, Ri, Li), t4 = fma(-b, Ri, Li)
 *                     lo = (fma(S, t1, -c0 Ri), fma(S, t2, c0 Rr)), hi = (fma(S, t3, c0 Ri), fma(-S, t4, c0 Rr))
 *   mode 1 mixed-special lanes: lo = (S (L0 + R0), S (L0 - R0)) (fma(S, fma(1, R0, L0), 0)),
 *                     hi = (S fma(fx', Rh, Lh), Sfy' Rh)
 * Counts bit-exact amplitude bins against the oracle's jsfft restatement.
 * Build: gcc -O2 -ffp-contract=off mixed_emu.c ../../oracle/meyda_oracle.c -lm -o /tmp/mixed_emu
 * Run:   /tmp/mixed_emu N FRAMES MODE   (MODE 0 = current kernel, 1 = unfused mixed form)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

void oracle_jsfft(float* re, float* im, int n);
void oracle_hanning(int n, float* out);
void oracle_synth(uint64_t seed, uint64_t first_index, long count, float* out);

static const double S = 0.7071067811865476, PI = 3.141592653589793;

static int rev(int x, int bits) { int r = 0; for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; } return r; }
static void build_klist(int m, int* k) {
  if (m == 2) { k[0] = 0; return; }
  int w = m / 2, h = w / 2;
  int* sub = malloc(sizeof(int) * h);
  build_klist(w, sub);
  k[0] = 0; k[h] = w / 2;
  for (int a = 1; a < h; a++) { k[a] = sub[a]; k[h + a] = w - sub[a]; }
  free(sub);
}

/* per stage s (q = s - 1): f_k(a) unscaled for a > 0, f_{w/2} at a = 0 */
static double (*g_f)[2];
static int g_off[32];
static void setup(int n) {
  int B = 0; while ((1 << B) < n) B++;
  g_f = calloc(n, sizeof *g_f);
  int off = 0;
  for (int s = 1; s < B; s++) {
    int w = 1 << s, h = w / 2;
    g_off[s] = off;
    double dr = cos(PI / w), di = sin(PI / w), fr = 1, fi = 0;
    double (*f)[2] = malloc(sizeof(double[2]) * w);
    for (int j = 0; j < w; j++) { f[j][0] = fr; f[j][1] = fi; double t = fr * dr - fi * di; fi = fr * di + fi * dr; fr = t; }
    int* kl = malloc(sizeof(int) * h);
    build_klist(w, kl);
    for (int a = 0; a < h; a++) { int k = a == 0 ? w / 2 : kl[a]; g_f[off + a][0] = f[k][0]; g_f[off + a][1] = f[k][1]; }
    off += h; free(f); free(kl);
  }
}

static void half_fft(const float* xw, int n, int rb, int mode, float* sre, float* sim) {
  int L = n / 2, B = 0; while ((1 << B) < n) B++;
  for (int j = 0; j < L; j++) {
    int e = rev(j, B - 1);
    double a = xw[e], b = xw[e + L];
    sre[j] = (float)(S * (a + b)); sim[j] = (float)(S * (a - b));
  }
  for (int s = 1; s < B; s++) {
    int q = s - 1, h = 1 << q, q0 = (q / rb) * rb;
    const double* fw = g_f[g_off[s]];  /* f_{w/2} */
    const double sfx = S * fw[0], sfy = S * fw[1];
    for (int blk = 0; blk < L; blk += 2 * h) {
      for (int a = 0; a < h; a++) {
        int lo = blk + a, hi = lo + h;
        double Lr = sre[lo], Li = sim[lo], Rr = sre[hi], Ri = sim[hi];
        int mixed = q0 > 0 && ((a >> q0) & ((1 << (q - q0)) - 1)) == 0;
        if (a == 0 && !(mode == 1 && mixed)) {
          sre[lo] = (float)(S * (Lr + Rr)); sim[lo] = (float)(S * (Lr - Rr));
          sre[hi] = (float)fma(S, Li, sfx * Ri); sim[hi] = (float)(sfy * Ri);
        } else if (a == 0) {
          sre[lo] = (float)fma(S, fma(1.0, Rr, Lr), 0.0); sim[lo] = (float)fma(S, fma(-1.0, Rr, Lr), 0.0);
          sre[hi] = (float)fma(S, fma(fw[0], Ri, Li), 0.0); sim[hi] = (float)(sfy * Ri);
        } else if (mode == 1 && mixed) {
          const double* f = g_f[g_off[s] + a];
          double b = f[0], c0 = S * f[1];
          double t1 = fma(b, Rr, Lr), t3 = fma(-b, Rr, Lr), t2 = fma(b, Ri, Li), t4 = fma(-b, Ri, Li);
          double ui = c0 * Ri, ur = c0 * Rr;
          sre[lo] = (float)fma(S, t1, -ui); sim[lo] = (float)fma(S, t2, ur);
          sre[hi] = (float)fma(S, t3, ui); sim[hi] = (float)fma(-S, t4, ur);
        } else {
          const double* f = g_f[g_off[s] + a];
          double cx = S * f[0], cy = S * f[1];
          double Ar = fma(cx, Rr, -(cy * Ri)), Ai = fma(cx, Ri, cy * Rr);
          sre[lo] = (float)fma(S, Lr, Ar); sim[lo] = (float)fma(S, Li, Ai);
          sre[hi] = (float)fma(S, Lr, -Ar); sim[hi] = (float)fma(-S, Li, Ai);
        }
      }
    }
  }
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 1024;
  int frames = argc > 2 ? atoi(argv[2]) : 2000;
  int mode = argc > 3 ? atoi(argv[3]) : 0;
  int L = n / 2, B = 0; while ((1 << B) < n) B++;
  int R = L / 64, rb = 0; while ((1 << rb) < R) rb++;
  setup(n);
  int* klN = malloc(sizeof(int) * L);
  build_klist(n, klN);
  float *x = malloc(sizeof(float) * n), *w = malloc(sizeof(float) * n), *xw = malloc(sizeof(float) * n);
  float *re = malloc(sizeof(float) * n), *im = malloc(sizeof(float) * n);
  float *sre = malloc(sizeof(float) * L), *sim = malloc(sizeof(float) * L);
  oracle_hanning(n, w);
  long exact = 0, total = 0, cat_exact[3] = {0}, cat_tot[3] = {0}, cat_bins[3] = {0}, cat_bexact[3] = {0};
  for (int f = 0; f < frames; f++) {
    int cat = f % 3;
    oracle_synth(0x6D657964, (uint64_t)f * n, n, x);
    if (cat == 1) for (int i = 0; i < n; i++) x[i] = (float)(0.6 * sin(2 * PI * (50 + f) * i / n) + 1e-3 * x[i]);
    if (cat == 2) for (int i = 0; i < n; i++) x[i] = (float)(0.5 * sin(2 * PI * 440.0 * (i + f * n) / 44100.0 * (1 + 1e-4 * f)));
    for (int i = 0; i < n; i++) { xw[i] = x[i] * w[i]; re[i] = xw[i]; im[i] = 0; }
    oracle_jsfft(re, im, n);
    half_fft(xw, n, rb, mode, sre, sim);
    int fe = 1;
    for (int j = 0; j < L; j++) {
      int k = klN[j];
      float gr = sre[j], gi = j == 0 ? 0.0f : sim[j];
      float ar = (float)sqrt((double)gr * gr + (double)gi * gi);
      float br = (float)sqrt((double)re[k] * re[k] + (double)im[k] * im[k]);
      total++; cat_bins[cat]++;
      if (ar == br) { exact++; cat_bexact[cat]++; } else fe = 0;
    }
    cat_tot[cat]++; cat_exact[cat] += fe;
  }
  printf("N=%d R=%d mode=%d: amp bit-exact %.6f; bins exact noise/tone+noise/tone %.6f %.6f %.6f; frames fully exact %ld/%ld %ld/%ld %ld/%ld\n",
         n, R, mode, (double)exact / total, (double)cat_bexact[0] / cat_bins[0], (double)cat_bexact[1] / cat_bins[1],
         (double)cat_bexact[2] / cat_bins[2], cat_exact[0], cat_tot[0], cat_exact[1], cat_tot[1], cat_exact[2], cat_tot[2]);
  return 0;
}
