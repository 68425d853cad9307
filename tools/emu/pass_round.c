/*
 * Per-pass rounding study (design validation only, not shipped; tools/pass_rounding.py drives it).
 *
 * jsfft's FFT_2_Iterative (lib/jsfft/fft.js:123-171) computes every butterfly in double and stores every
 * stage to Float32Array (lib/jsfft/complex_array.js:7,31-32). The kernel's faithful mode reproduces that:
 * 2 conversions per value and stage, 394 of its 1,161 VALU per frame. A "per-pass" precision
 * would keep double through the register stages of a pass and round to float32 only where the kernel's
 * passes meet (its LDS exchanges) and at the end. This restates jsfft with that rounding schedule:
 *   stage s (width 2^s, s = 0 .. B-1) is rounded to float32 iff bit s of round_mask is set.
 * round_mask = all ones is jsfft itself (the oracle's oracle_jsfft); the kernel's pass boundaries at
 * R = N/128 slots per lane (RB = log2 R) are s = RB, 2 RB, ... and s = B - 1 (stage 0 joins pass 0).
 * Build: gcc -O2 -shared -fPIC -ffp-contract=off pass_round.c -lm -o /tmp/libpass_round.so
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

static const double JS_PI = 3.141592653589793, JS_SQRT1_2 = 0.7071067811865476;

static int bit_reverse(int index, int n) {
  int r = 0;
  while (n > 1) { r = (r << 1) + (index & 1); index >>= 1; n >>= 1; }
  return r;
}

/* xw: the windowed frame (float32, n); out: amplitude f32(sqrt(re^2 + im^2)) of bins 0 .. n/2 - 1
 * (src/meyda.js:104-114), from the float32 values of the last stage (the last stage is always rounded:
 * the amplitude reads Float32Array storage). */
void pr_amp(const float* xw, int n, uint32_t round_mask, float* amp) {
  double* re = malloc(sizeof(double) * n);
  double* im = malloc(sizeof(double) * n);
  for (int i = 0; i < n; i++) { re[bit_reverse(i, n)] = xw[i]; im[i] = 0.0; }
  int s = 0;
  for (int width = 1; width < n; width <<= 1, s++) {
    const double del_r = cos(JS_PI / width), del_i = sin(JS_PI / width);
    const int rnd = (round_mask >> s) & 1;
    for (int i = 0; i < n / (2 * width); i++) {
      double f_r = 1, f_i = 0;
      for (int j = 0; j < width; j++) {
        const int l = 2 * i * width + j, r = l + width;
        const double left_r = re[l], left_i = im[l];
        const double right_r = f_r * re[r] - f_i * im[r];
        const double right_i = f_i * re[r] + f_r * im[r];
        double a = JS_SQRT1_2 * (left_r + right_r), b = JS_SQRT1_2 * (left_i + right_i);
        double c = JS_SQRT1_2 * (left_r - right_r), d = JS_SQRT1_2 * (left_i - right_i);
        if (rnd) { a = (float)a; b = (float)b; c = (float)c; d = (float)d; }
        re[l] = a; im[l] = b; re[r] = c; im[r] = d;
        const double temp = f_r * del_r - f_i * del_i;
        f_i = f_r * del_i + f_i * del_r;
        f_r = temp;
      }
    }
  }
  for (int k = 0; k < n / 2; k++) {
    const double xr = (float)re[k], xi = (float)im[k];
    amp[k] = (float)sqrt(xr * xr + xi * xi);
  }
  free(re);
  free(im);
}
