/*
 * CPU emulation of the GPU FFT design (design validation only, not shipped).
 *
 * The frame is real, so every jsfft stage output block is Hermitian. The GPU
 * keeps only the half spectrum of each block in N/2 complex "slots" laid out so
 * that each stage is an in-place radix-2 network over slot locations:
 *   stage 0 (load): slot j = (s(x_a + x_b), s(x_a - x_b)), x_a = xw[rev(j)], x_b = xw[rev(j)+N/2]
 *   stage s >= 1 (h = 2^(s-1)): pairs (a, a+h) in each 2h block;
 *       a == 0 : special  (L0,Lh),(R0,Rh) -> (s(L0+R0), s(L0-R0)), s(Lh + f_{w/2} Rh)
 *       a  > 0 : generic  L,R -> s L + c R  and  conj(s L - c R),  c = s f_k(a)
 * and compares against the oracle (the jsfft restatement), counting bit-exact bins.
 * Build: gcc -O2 -ffp-contract=off half_fft_emu.c ../../oracle/meyda_oracle.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_jsfft(float* re, float* im, int n);
void oracle_hanning(int n, float* out);
void oracle_synth(uint64_t seed, uint64_t first_index, long count, float* out);

static const double S = 0.7071067811865476, PI = 3.141592653589793;

static int rev(int x, int bits) { int r = 0; for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; } return r; }

/* klist[m][a]: logical Hermitian index stored at slot location a of a size-m block. */
static void build_klist(int m, int* k) {
  if (m == 2) { k[0] = 0; return; }
  int w = m / 2, h = w / 2;
  int* sub = malloc(sizeof(int) * h);
  build_klist(w, sub);
  k[0] = 0; k[h] = w / 2;
  for (int a = 1; a < h; a++) { k[a] = sub[a]; k[h + a] = w - sub[a]; }
  free(sub);
}

static int g_fma = 1;
static double fm(double a, double b, double c) { return g_fma ? fma(a, b, c) : a * b + c; }

static void half_fft(const float* xw, int n, float* sre, float* sim, double (*tw)[2], const int* twoff) {
  int L = n / 2, B = 0; while ((1 << B) < n) B++;
  for (int j = 0; j < L; j++) {
    int e = rev(j, B - 1);
    double a = xw[e], b = xw[e + L];
    sre[j] = (float)(S * (a + b)); sim[j] = (float)(S * (a - b));
  }
  for (int s = 1; s < B; s++) {
    int h = 1 << (s - 1);
    for (int blk = 0; blk < L; blk += 2 * h) {
      for (int a = 0; a < h; a++) {
        int lo = blk + a, hi = blk + a + h;
        double Lr = sre[lo], Li = sim[lo], Rr = sre[hi], Ri = sim[hi];
        const double* c = tw[twoff[s] + a];
        if (a == 0) {
          /* exact reference ops: f = f_{w/2} (unscaled) */
          sre[lo] = (float)(S * (Lr + Rr)); sim[lo] = (float)(S * (Lr - Rr));
          sre[hi] = (float)(S * (Li + c[0] * Ri)); sim[hi] = (float)(S * (c[1] * Ri));
        } else {
          double Ar = fm(c[0], Rr, -(c[1] * Ri));
          double Ai = fm(c[0], Ri, c[1] * Rr);
          sre[lo] = (float)fm(S, Lr, Ar); sim[lo] = (float)fm(S, Li, Ai);
          sre[hi] = (float)fm(S, Lr, -Ar); sim[hi] = (float)(-fm(S, Li, -Ai));
        }
      }
    }
  }
}

static double (*g_tw)[2]; static int g_twoff[32]; static int g_n;
static void setup(int n) {
  if (g_n == n) return;
  g_n = n;
  int B = 0; while ((1 << B) < n) B++;
  free(g_tw); g_tw = calloc(n, sizeof *g_tw);
  int off = 0;
  for (int s = 1; s < B; s++) {
    int w = 1 << s, h = w / 2;
    g_twoff[s] = off;
    double dr = cos(PI / w), di = sin(PI / w), fr = 1, fi = 0;
    double (*f)[2] = malloc(sizeof(double[2]) * w);
    for (int j = 0; j < w; j++) { f[j][0] = fr; f[j][1] = fi; double t = fr * dr - fi * di; fi = fr * di + fi * dr; fr = t; }
    int* kl = malloc(sizeof(int) * h);
    build_klist(w, kl);
    for (int a = 0; a < h; a++) {
      int k = a == 0 ? w / 2 : kl[a];
      double sc = a == 0 ? 1.0 : S;
      g_tw[off + a][0] = sc * f[k][0]; g_tw[off + a][1] = sc * f[k][1];
    }
    off += h; free(f); free(kl);
  }
}
void emu_half_amp(const float* frames, long F, int n, const float* win, float* amp) {
  setup(n);
  int L = n / 2;
  int* klN = malloc(sizeof(int) * L); build_klist(n, klN);
  float *xw = malloc(sizeof(float) * n), *sre = malloc(sizeof(float) * L), *sim = malloc(sizeof(float) * L);
  for (long f = 0; f < F; f++) {
    for (int i = 0; i < n; i++) xw[i] = frames[f * n + i] * win[i];
    half_fft(xw, n, sre, sim, g_tw, g_twoff);
    for (int j = 0; j < L; j++) {
      float gr = sre[j], gi = j == 0 ? 0.0f : sim[j];
      amp[f * L + klN[j]] = (float)sqrt((double)gr * gr + (double)gi * gi);
    }
  }
  free(klN); free(xw); free(sre); free(sim);
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 1024;
  int frames = argc > 2 ? atoi(argv[2]) : 2000;
  g_fma = argc > 3 ? atoi(argv[3]) : 1;
  int L = n / 2, B = 0; while ((1 << B) < n) B++;
  /* twiddles: jsfft recurrence per stage, located by klist of the input block */
  double (*tw)[2] = calloc(n, sizeof *tw);
  int twoff[32];
  int off = 0;
  for (int s = 1; s < B; s++) {
    int w = 1 << s, h = w / 2;
    twoff[s] = off;
    double dr = cos(PI / w), di = sin(PI / w), fr = 1, fi = 0;
    double (*f)[2] = malloc(sizeof(double[2]) * w);
    for (int j = 0; j < w; j++) { f[j][0] = fr; f[j][1] = fi; double t = fr * dr - fi * di; fi = fr * di + fi * dr; fr = t; }
    int* kl = malloc(sizeof(int) * h);
    build_klist(w, kl);
    for (int a = 0; a < h; a++) {
      int k = a == 0 ? w / 2 : kl[a];
      double sc = a == 0 ? 1.0 : S;
      tw[off + a][0] = sc * f[k][0]; tw[off + a][1] = sc * f[k][1];
    }
    off += h;
    free(f); free(kl);
  }
  int* klN = malloc(sizeof(int) * L);
  build_klist(n, klN);
  float *x = malloc(sizeof(float) * n), *w = malloc(sizeof(float) * n), *xw = malloc(sizeof(float) * n);
  float *re = malloc(sizeof(float) * n), *im = malloc(sizeof(float) * n);
  float *sre = malloc(sizeof(float) * L), *sim = malloc(sizeof(float) * L);
  oracle_hanning(n, w);
  long exact = 0, total = 0, cexact = 0, ctotal = 0, frames_exact = 0, cat_exact[3]={0}, cat_tot[3]={0};
  double maxrel = 0;
  for (int f = 0; f < frames; f++) {
    oracle_synth(0x6D657964, (uint64_t)f * n, n, x);
    if (f % 3 == 1) for (int i = 0; i < n; i++) x[i] = (float)(0.6 * sin(2 * PI * (50 + f) * i / n) + 1e-3 * x[i]);
    if (f % 3 == 2) for (int i = 0; i < n; i++) x[i] = (float)(0.5 * sin(2 * PI * 440.0 * (i + f * n) / 44100.0 * (1 + 1e-4 * f)));
    for (int i = 0; i < n; i++) { xw[i] = x[i] * w[i]; re[i] = xw[i]; im[i] = 0; }
    oracle_jsfft(re, im, n);
    half_fft(xw, n, sre, sim, tw, twoff);
    int fe = 1;
    for (int j = 0; j < L; j++) {
      int k = klN[j];
      float gr = sre[j], gi = j == 0 ? 0.0f : sim[j];
      float ar = (float)sqrt((double)gr * gr + (double)gi * gi);
      float br = (float)sqrt((double)re[k] * re[k] + (double)im[k] * im[k]);
      total++; if (ar == br) exact++; else fe = 0;
      double d = fabs((double)ar - br) / (br > 0 ? br : 1e-30);
      if (d > maxrel) maxrel = d;
      ctotal += 2; cexact += (gr == re[k]) + (gi == im[k]);
      if (j == 0) { ctotal += 1; cexact += (sim[0] == re[L]); }
    }
    frames_exact += fe; cat_tot[f%3]++; cat_exact[f%3]+=fe;
  }
  printf("N=%d frames=%d fma=%d: amp bit-exact %.8f (%ld/%ld), complex comps exact %.8f, frames fully exact %.5f, max rel amp err %.3g\n",
         n, frames, g_fma, (double)exact / total, exact, total, (double)cexact / ctotal, (double)frames_exact / frames, maxrel);
  printf("  per category fully-exact frames: %ld/%ld %ld/%ld %ld/%ld\n", cat_exact[0],cat_tot[0],cat_exact[1],cat_tot[1],cat_exact[2],cat_tot[2]);
  return 0;
}
