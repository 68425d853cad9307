// Fused per-frame feature extraction for gfx950 (MI355X).
//
// One launch processes a batch of frames. Each 256-thread workgroup loops over
// batches of FB frames:
//
//  Phase 1 (one wave per frame, FB/4 frames per wave):
//    load + rms/energy/zcr      src/extractors/rms.js, energy.js, zcr.js
//    window                     src/meyda.js:158-168
//    FFT                        lib/jsfft/fft.js:123-208, restated as a Hermitian
//                               half-spectrum radix-2 network: the
//                               frame is real, so each stage output block is kept as
//                               N/2 complex "slots"; every stage is rounded to
//                               float32 exactly where jsfft stores to Float32Array,
//                               with float64 butterflies.
//    amplitude                  src/meyda.js:104-114 -> LDS batch buffer
//    per-frame reductions       moments (src/utils.js:1-11), log sum
//                               (spectralFlatness.js), prefix sums (spectralRolloff.js,
//                               loudness band sums loudness.js:47-66)
//  Phase 2 (whole workgroup, frames x bands in parallel):
//    specific loudness          loudness.js:55-63 (pow 0.23, float32 store)
//    mel filterbank + log       mfcc.js:53-65 (sequential float32 accumulation, as written)
//    DCT                        mfcc.js:85-93
//    scalar features            spectral*.js, perceptual*.js
//
// Compiled with -ffp-contract=off: every fused multiply-add below is explicit.
#include "mgx_internal.h"

namespace mgx {
namespace {

constexpr double kS = 0.7071067811865476;  // Math.SQRT1_2 (lib/jsfft/fft.js:10)
constexpr float kSf = 0.70710677f;
constexpr double kLn2 = 0.6931471805599453;

constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v >> 1); }
constexpr int rev_bits(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r = (r << 1) | ((x >> i) & 1);
  return r;
}

template <int N>
struct Geo {
  static constexpr int L = N / 2;           // slots per frame == amplitude bins
  static constexpr int R = L / 64;          // slots per lane
  static constexpr int SB = ilog2c(L);      // slot-location bits
  static constexpr int RB = ilog2c(R);      // register bits
  static constexpr int NPASS = (SB + RB - 1) / RB;
  static constexpr int CH = N / 64;         // 64-sample input chunks per frame
  static constexpr int FB = N >= 2048 ? 8 : 16;  // frames per workgroup batch
  static constexpr int AMP_STRIDE = L + 1;  // odd float stride between frames in LDS
  static constexpr int SLOT_PHYS = L + (L >> 4) + 2;
  static_assert(R >= 2 && (R & (R - 1)) == 0, "N must be a power of two in [256, 2048]");
};

// Location bits of pass p: register bits [0, m) drive location bits [q0, q0+m); the
// six lane bits take the lowest remaining location bits; leftover register bits
// take the rest. Pass 0 is fixed by the load: location = rev6(lane)*R + r.
template <int N>
struct PassGeo {
  using G = Geo<N>;
  static constexpr int q0(int p) { return p * G::RB; }
  static constexpr int m(int p) { return (G::SB - q0(p)) < G::RB ? (G::SB - q0(p)) : G::RB; }
  static constexpr int free_bit(int p, int idx) {
    int cnt = 0;
    for (int b = 0; b < G::SB; ++b) {
      if (b >= q0(p) && b < q0(p) + m(p)) continue;
      if (cnt == idx) return b;
      ++cnt;
    }
    return -1;
  }
  static constexpr int rpart(int p, int r) {
    int loc = 0;
    for (int i = 0; i < G::RB; ++i) {
      const int pos = i < m(p) ? q0(p) + i : free_bit(p, 6 + (i - m(p)));
      loc |= ((r >> i) & 1) << pos;
    }
    return loc;
  }
  static __device__ int lanepart(int p, int lane) {
    if (p == 0) return rev_bits(lane, 6) << G::RB;
    int loc = 0;
    for (int i = 0; i < 6; ++i) loc |= ((lane >> i) & 1) << free_bit(p, i);
    return loc;
  }
};

__device__ __forceinline__ int phys(int loc) { return loc + (loc >> 4); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// ---------------------------------------------------------------- butterflies
// Generic slot pair (location a > 0 in its block), c = SQRT1_2 * f_k:
//   lo <- s L + c R,  hi <- conj(s L - c R)
template <bool FAITH>
__device__ __forceinline__ void bfly_generic(float2& lo, float2& hi, const double2* tw, const float2* twf, int idx) {
  if constexpr (FAITH) {
    const double2 c = tw[idx];
    const double Lr = lo.x, Li = lo.y, Rr = hi.x, Ri = hi.y;
    const double Ar = __builtin_fma(c.x, Rr, -(c.y * Ri));
    const double Ai = __builtin_fma(c.x, Ri, c.y * Rr);
    lo.x = (float)__builtin_fma(kS, Lr, Ar);
    lo.y = (float)__builtin_fma(kS, Li, Ai);
    hi.x = (float)__builtin_fma(kS, Lr, -Ar);
    hi.y = (float)__builtin_fma(-kS, Li, Ai);
  } else {
    const float2 c = twf[idx];
    const float Ar = __builtin_fmaf(c.x, hi.x, -(c.y * hi.y));
    const float Ai = __builtin_fmaf(c.x, hi.y, c.y * hi.x);
    const float Lr = lo.x, Li = lo.y;
    lo.x = __builtin_fmaf(kSf, Lr, Ar);
    lo.y = __builtin_fmaf(kSf, Li, Ai);
    hi.x = __builtin_fmaf(kSf, Lr, -Ar);
    hi.y = __builtin_fmaf(-kSf, Li, Ai);
  }
}

// Block-start pair (location 0): the packed reals (X[0], X[w/2]) of both halves.
// Exactly jsfft's operations for j = 0 and j = w/2 (f_0 = 1, f = f_{w/2} unscaled).
template <bool FAITH>
__device__ __forceinline__ void bfly_special(float2& lo, float2& hi, const double2* tw, const float2* twf, int idx) {
  if constexpr (FAITH) {
    const double2 f = tw[idx];
    const double L0 = lo.x, Lh = lo.y, R0 = hi.x, Rh = hi.y;
    lo.x = (float)(kS * (L0 + R0));
    lo.y = (float)(kS * (L0 - R0));
    hi.x = (float)(kS * (Lh + f.x * Rh));
    hi.y = (float)(kS * (f.y * Rh));
  } else {
    const float2 f = twf[idx];
    const float L0 = lo.x, Lh = lo.y, R0 = hi.x, Rh = hi.y;
    lo.x = kSf * (L0 + R0);
    lo.y = kSf * (L0 - R0);
    hi.x = kSf * __builtin_fmaf(f.x, Rh, Lh);
    hi.y = kSf * (f.y * Rh);
  }
}

// One radix-2 stage on location bit q = q0(P) + I, entirely in registers.
template <int N, int P, int I, bool FAITH>
__device__ __forceinline__ void run_stage(float2 (&v)[Geo<N>::R], int lp, const DevTables& t) {
  using G = Geo<N>;
  using PG = PassGeo<N>;
  constexpr int q = PG::q0(P) + I;
  constexpr int mask = (1 << q) - 1;
  const int la = lp & mask;  // 0 in pass 0
#pragma unroll
  for (int r = 0; r < G::R; ++r) {
    if (r & (1 << I)) continue;
    const int rp = PG::rpart(P, r) & mask;
    const int hi = r | (1 << I);
    if constexpr (P == 0) {
      if (rp == 0) bfly_special<FAITH>(v[r], v[hi], t.tw, t.twf, mask);
      else bfly_generic<FAITH>(v[r], v[hi], t.tw, t.twf, mask + rp);
    } else {
      const int a = la | rp;
      if (a == 0) bfly_special<FAITH>(v[r], v[hi], t.tw, t.twf, mask);
      else bfly_generic<FAITH>(v[r], v[hi], t.tw, t.twf, mask + a);
    }
  }
}

template <int N, int P, int I, bool FAITH>
__device__ __forceinline__ void run_stages(float2 (&v)[Geo<N>::R], int lp, const DevTables& t) {
  if constexpr (I < PassGeo<N>::m(P)) {
    run_stage<N, P, I, FAITH>(v, lp, t);
    run_stages<N, P, I + 1, FAITH>(v, lp, t);
  }
}

// Move the slots from pass P-1's lane/register layout to pass P's through LDS.
template <int N, int P>
__device__ __forceinline__ void exchange(float2 (&v)[Geo<N>::R], int lp_prev, int lp_cur, float2* buf) {
  using G = Geo<N>;
  using PG = PassGeo<N>;
  const int bprev = phys(lp_prev), bcur = phys(lp_cur);
  wave_sync();
#pragma unroll
  for (int r = 0; r < G::R; ++r) buf[bprev + phys(PG::rpart(P - 1, r))] = v[r];
  wave_sync();
#pragma unroll
  for (int r = 0; r < G::R; ++r) v[r] = buf[bcur + phys(PG::rpart(P, r))];
}

template <int N, int P, bool FAITH>
__device__ __forceinline__ void run_passes(float2 (&v)[Geo<N>::R], const int (&lp)[Geo<N>::NPASS],
                                           float2* buf, const DevTables& t) {
  if constexpr (P < Geo<N>::NPASS) {
    if constexpr (P > 0) exchange<N, P>(v, lp[P - 1], lp[P], buf);
    run_stages<N, P, 0, FAITH>(v, lp[P], t);
    run_passes<N, P + 1, FAITH>(v, lp, buf, t);
  }
}

struct FrameRec {
  double S[5];      // sum_k k^p a_k, p = 0..4
  double ln2sum;    // sum_k log2 a_k
  double energy;    // sum x^2
  double band[kBark];
  float spec[kBark];
  float lm[kMaxMel];
  int zcr;
  int roll_m;
};

template <typename T>
__device__ __forceinline__ void put_scalar(const KernelArgs& a, int i, uint64_t f, double v) {
  if (a.out.scalars[i]) static_cast<T*>(a.out.scalars[i])[f] = (T)v;
}

template <int N, bool FAITH, bool LITERAL>
__global__ __launch_bounds__(kThreads) void extract_kernel(KernelArgs a) {
  using G = Geo<N>;
  using PG = PassGeo<N>;
  constexpr int L = G::L, R = G::R, CH = G::CH, FB = G::FB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* amp_all = reinterpret_cast<float*>(smem);
  constexpr size_t amp_bytes = ((size_t)FB * G::AMP_STRIDE * 4 + 15) / 16 * 16;
  float2* slot_all = reinterpret_cast<float2*>(smem + amp_bytes);
  FrameRec* recs = reinterpret_cast<FrameRec*>(smem + amp_bytes + (size_t)4 * G::SLOT_PHYS * 8);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float2* buf = slot_all + wave * G::SLOT_PHYS;
  double* pbuf = reinterpret_cast<double*>(buf);
  int lp[G::NPASS];
#pragma unroll
  for (int p = 0; p < G::NPASS; ++p) lp[p] = PG::lanepart(p, lane);

  const DevTables& t = a.t;
  const uint64_t nb = (a.num_frames + FB - 1) / FB;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint64_t f0 = b * FB;
    // ------------------------------------------------------------- phase 1
    for (int j = 0; j < FB / 4; ++j) {
      const int fb = j * 4 + wave;
      const uint64_t f = f0 + fb;
      const bool valid = f < a.num_frames;
      const float* xin = a.frames + f * (uint64_t)N;
      float* amp = amp_all + fb * G::AMP_STRIDE;
      float x[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) x[c] = valid ? xin[c * 64 + lane] : 0.0f;

      // rms.js / energy.js: sum of squares (double); zcr.js: sign changes of adjacent
      // samples, `x >= 0` vs `x < 0` (so -0 is non-negative and NaN never counts).
      double e = 0.0;
      int z = 0;
      uint64_t pge = 0, plt = 0;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const double xd = x[c];
        e = __builtin_fma(xd, xd, e);
        const uint64_t g = __ballot(x[c] >= 0.0f), l = __ballot(x[c] < 0.0f);
        z += __popcll(((g & (l >> 1)) | (l & (g >> 1))) & 0x7FFFFFFFFFFFFFFFull);
        if (c > 0) z += (int)((((pge >> 63) & l) | ((plt >> 63) & g)) & 1ull);
        pge = g;
        plt = l;
      }
      e = wave_sum(e);

      // src/meyda.js:158-168: windowed[i] = sig[i] * w[i], stored to Float32Array
      // (the exact double product rounded once == a float32 multiply).
#pragma unroll
      for (int c = 0; c < CH; ++c) x[c] *= t.window[c * 64 + lane];

      if (a.need_spectrum) {
        if constexpr (LITERAL) {
          // The snapshot never transforms per buffer: |w x| is the "spectrum".
#pragma unroll
          for (int c = 0; c < R; ++c) amp[c * 64 + lane] = fabsf(x[c]);
        } else {
          // Stage 0 (jsfft width 1) at load: slot j = rev(e) pairs x[e] with x[e + N/2].
          float2 v[R];
#pragma unroll
          for (int c = 0; c < R; ++c) {
            const int r = rev_bits(c, G::RB);
            if constexpr (FAITH) {
              const double xa = x[c], xb = x[c + R];
              v[r].x = (float)(kS * (xa + xb));
              v[r].y = (float)(kS * (xa - xb));
            } else {
              v[r].x = kSf * (x[c] + x[c + R]);
              v[r].y = kSf * (x[c] - x[c + R]);
            }
          }
          run_passes<N, 0, FAITH>(v, lp, buf, t);

          // src/meyda.js:104-114: |X_k| for k < N/2, rounded to float32.
          const int lpl = lp[G::NPASS - 1];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int rp = PG::rpart(G::NPASS - 1, r);
            const int loc = lpl | rp;
            const int k = t.klist[loc];
            const bool dc = (rp == 0) && (lpl == 0);
            float av;
            if constexpr (FAITH) {
              const double xr = v[r].x, xi = v[r].y;
              av = (float)sqrt(__builtin_fma(xr, xr, xi * xi));
            } else {
              av = sqrtf(__builtin_fmaf(v[r].x, v[r].x, v[r].y * v[r].y));
            }
            if (dc) av = fabsf(v[r].x);  // slot 0 packs (X[0], X[N/2]), both real
            amp[k] = av;
            if (valid && a.out.complex_real) {
              float* cr = a.out.complex_real + f * (uint64_t)N;
              float* ci = a.out.complex_imag + f * (uint64_t)N;
              if (dc) {
                cr[0] = v[r].x; ci[0] = 0.0f;
                cr[L] = v[r].y; ci[L] = 0.0f;
              } else {
                cr[k] = v[r].x; ci[k] = v[r].y;
                cr[N - k] = v[r].x; ci[N - k] = -v[r].y;
              }
            }
          }
        }
        wave_sync();

        if (valid && a.out.amplitude_spectrum) {
#pragma unroll
          for (int c = 0; c < R; ++c)
            a.out.amplitude_spectrum[f * (uint64_t)L + c * 64 + lane] = amp[c * 64 + lane];
        }
        if (valid && a.out.power_spectrum) {
#pragma unroll
          for (int c = 0; c < R; ++c) {
            const float av = amp[c * 64 + lane];
            a.out.power_spectrum[f * (uint64_t)L + c * 64 + lane] = av * av;  // powerSpectrum.js
          }
        }

        // Per-frame reductions, lane t owns bins [R t, R t + R).
        double T0 = 0, T1 = 0, T2 = 0, T3 = 0, T4 = 0, l2 = 0;
        double pl[R];
#pragma unroll
        for (int jj = 0; jj < R; ++jj) {
          const float av = amp[R * lane + jj];
          const double ad = av;
          pl[jj] = T0;
          T0 += ad;
          T1 = __builtin_fma((double)jj, ad, T1);
          T2 = __builtin_fma((double)(jj * jj), ad, T2);
          T3 = __builtin_fma((double)(jj * jj * jj), ad, T3);
          T4 = __builtin_fma((double)(jj * jj * jj * jj), ad, T4);
          l2 += (double)log2f(av);
        }
        // exclusive scan of the lane totals -> prefix P(k) = sum_{i<k} a_i
        double incl = T0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const double y = __shfl_up(incl, d);
          if (lane >= d) incl += y;
        }
        double excl = __shfl_up(incl, 1);
        if (lane == 0) excl = 0.0;
        const double total = __shfl(incl, 63);
        // spectralRolloff.js:6-15: the largest m with P(m) <= 0.99 total (P(0) = 0).
        const double thr = 0.99 * total;
        int cnt = 0;
        wave_sync();  // the slot buffer is reused as the prefix scratch
#pragma unroll
        for (int jj = 0; jj < R; ++jj) {
          const double pk = excl + pl[jj];
          pbuf[R * lane + jj] = pk;
          cnt += __popcll(__ballot(pk <= thr));
        }
        const int roll_m = (total > thr) ? cnt - 1 : L;
        const double bb = (double)(R * lane), b2 = bb * bb, b3 = b2 * bb, b4 = b3 * bb;
        double S1 = __builtin_fma(bb, T0, T1);
        double S2 = T2 + 2.0 * bb * T1 + b2 * T0;
        double S3 = T3 + 3.0 * bb * T2 + 3.0 * b2 * T1 + b3 * T0;
        double S4 = T4 + 4.0 * bb * T3 + 6.0 * b2 * T2 + 4.0 * b3 * T1 + b4 * T0;
        S1 = wave_sum(S1);
        S2 = wave_sum(S2);
        S3 = wave_sum(S3);
        S4 = wave_sum(S4);
        l2 = wave_sum(l2);
        wave_sync();
        FrameRec& rec = recs[fb];
        if (lane < kBark) rec.band[lane] = pbuf[t.bblim[lane + 1]] - pbuf[t.bblim[lane]];
        if (lane == 0) {
          rec.S[0] = total; rec.S[1] = S1; rec.S[2] = S2; rec.S[3] = S3; rec.S[4] = S4;
          rec.ln2sum = l2;
          rec.roll_m = roll_m;
        }
      }
      if (lane == 0) {
        recs[fb].energy = e;
        recs[fb].zcr = z;
      }
    }
    __syncthreads();

    // ------------------------------------------------------------- phase 2
    const int tid = threadIdx.x;
    if (a.need_spectrum && a.need_loudness) {
      for (int i = tid; i < FB * kBark; i += kThreads) {
        const int bnd = i / FB, fb = i % FB;
        const float s = (float)pow(recs[fb].band[bnd], 0.23);  // loudness.js:62
        recs[fb].spec[bnd] = s;
        const uint64_t f = f0 + fb;
        if (f < a.num_frames && a.out.loudness_specific) a.out.loudness_specific[f * kBark + bnd] = s;
      }
    }
    if (a.need_spectrum && a.need_mfcc) {
      // mfcc.js:53-65: Float32Array accumulator, double products, ascending bins.
      for (int i = tid; i < FB * a.nfilt; i += kThreads) {
        const int flt = i / FB, fb = i % FB;
        const float* amp = amp_all + fb * G::AMP_STRIDE;
        const int k0 = t.mel_start[flt], cnt = t.mel_cnt[flt];
        const double* w = t.mel_w + t.mel_off[flt];
        float acc = 0.0f;
        for (int q = 0; q < cnt; ++q) {
          const float av = amp[k0 + q];
          const float pw = av * av;  // powerSpectrum.js: Math.pow(a, 2) stored to Float32Array
          acc = (float)((double)acc + w[q] * (double)pw);
        }
        recs[fb].lm[flt] = (float)log((double)acc);
      }
    }
    __syncthreads();
    if (a.need_spectrum && a.need_mfcc) {
      for (int i = tid; i < FB * a.ncoef; i += kThreads) {
        const int c = i / FB, fb = i % FB;
        const uint64_t f = f0 + fb;
        double v = 0.0;
        for (int n = 0; n < a.nfilt; ++n) v += (double)t.dct[c + n * a.ncoef] * (double)recs[fb].lm[n];
        if (f < a.num_frames && a.out.mfcc) a.out.mfcc[f * a.ncoef + c] = (float)(v / a.ncoef);
      }
    }
    if (tid < FB && f0 + tid < a.num_frames) {
      const FrameRec& rc = recs[tid];
      const uint64_t f = f0 + tid;
      double sv[MGX_NUM_SCALARS];
      sv[MGX_ENERGY] = rc.energy;
      sv[MGX_RMS] = sqrt(rc.energy / N);
      sv[MGX_ZCR] = (double)rc.zcr;
      if (a.need_spectrum) {
        const double S0 = rc.S[0];
        const double m1 = rc.S[1] / S0, m2 = rc.S[2] / S0, m3 = rc.S[3] / S0, m4 = rc.S[4] / S0;
        const double var = m2 - m1 * m1, sd = sqrt(var);
        sv[MGX_SPECTRAL_CENTROID] = m1;
        sv[MGX_SPECTRAL_SPREAD] = sd;
        sv[MGX_SPECTRAL_SKEWNESS] = (2.0 * m1 * m1 * m1 - 3.0 * m1 * m2 + m3) / (sd * sd * sd);
        sv[MGX_SPECTRAL_KURTOSIS] = (-3.0 * m1 * m1 * m1 * m1 + 6.0 * m1 * m2 - 4.0 * m1 * m3 + m4) / (sd * sd * sd * sd);
        sv[MGX_SPECTRAL_FLATNESS] = exp(rc.ln2sum * kLn2 / L) * L / S0;
        const double afs = (a.sample_rate / N) * rc.S[1];
        sv[MGX_SPECTRAL_SLOPE] = (L * afs - a.freq_sum * S0) / (S0 * (a.pow_freq_sum - a.freq_sum * a.freq_sum));
        sv[MGX_SPECTRAL_ROLLOFF] = (double)rc.roll_m * a.nyq_bin;
        if (a.need_loudness) {
          double total = 0.0, mx = 0.0, sh = 0.0;
          for (int i = 0; i < kBark; ++i) {
            total += rc.spec[i];
            if (rc.spec[i] > mx) mx = rc.spec[i];
          }
          for (int i = 0; i < kBark; ++i) sh += (i < 15) ? (i + 1) * (double)rc.spec[i + 1] : t.sharp_tail[i];
          const double ps = (total - mx) / total;
          sv[MGX_LOUDNESS_TOTAL] = total;
          sv[MGX_PERCEPTUAL_SPREAD] = ps * ps;
          sv[MGX_PERCEPTUAL_SHARPNESS] = sh * (0.11 / total);
        } else {
          sv[MGX_LOUDNESS_TOTAL] = sv[MGX_PERCEPTUAL_SPREAD] = sv[MGX_PERCEPTUAL_SHARPNESS] = 0.0;
        }
      } else {
        for (int i = MGX_SPECTRAL_CENTROID; i < MGX_NUM_SCALARS; ++i) sv[i] = 0.0;
      }
      for (int i = 0; i < MGX_NUM_SCALARS; ++i) {
        if (a.scalar_f64) put_scalar<double>(a, i, f, sv[i]);
        else put_scalar<float>(a, i, f, sv[i]);
      }
    }
    __syncthreads();
  }
}

__global__ void synth_kernel(float* __restrict__ out, uint64_t count, uint64_t seed, uint64_t first) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < count; i += stride) {
    float r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint64_t z = seed + (first + i + u + 1) * 0x9E3779B97F4A7C15ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      r[u] = (float)(uint32_t)(z >> 40) * 0x1p-23f - 1.0f;
    }
    if (i + 3 < count && ((reinterpret_cast<uintptr_t>(out + i) & 15) == 0)) {
      *reinterpret_cast<float4*>(out + i) = make_float4(r[0], r[1], r[2], r[3]);
    } else {
      for (int u = 0; u < 4 && i + u < count; ++u) out[i + u] = r[u];
    }
  }
}

template <int N>
size_t lds_bytes() {
  using G = Geo<N>;
  const size_t amp_bytes = ((size_t)G::FB * G::AMP_STRIDE * 4 + 15) / 16 * 16;
  return amp_bytes + (size_t)4 * G::SLOT_PHYS * 8 + (size_t)G::FB * sizeof(FrameRec);
}

template <int N, bool FAITH, bool LITERAL>
hipError_t launch_n(const KernelArgs& a, int grid, hipStream_t stream) {
  const size_t lds = lds_bytes<N>();
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&extract_kernel<N, FAITH, LITERAL>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((extract_kernel<N, FAITH, LITERAL>), dim3(grid), dim3(kThreads), lds, stream, a);
  return hipGetLastError();
}

template <int N>
hipError_t launch_prec(int precision, int mode, const KernelArgs& a, int grid, hipStream_t stream) {
  if (mode == MGX_MODE_LITERAL) return launch_n<N, true, true>(a, grid, stream);
  if (precision == MGX_PRECISION_FAST) return launch_n<N, false, false>(a, grid, stream);
  return launch_n<N, true, false>(a, grid, stream);
}

}  // namespace

size_t extract_lds_bytes(int n) {
  switch (n) {
    case 256: return lds_bytes<256>();
    case 512: return lds_bytes<512>();
    case 1024: return lds_bytes<1024>();
    case 2048: return lds_bytes<2048>();
    default: return 0;
  }
}

int frames_per_batch(int n) {
  switch (n) {
    case 256: return Geo<256>::FB;
    case 512: return Geo<512>::FB;
    case 1024: return Geo<1024>::FB;
    case 2048: return Geo<2048>::FB;
    default: return 0;
  }
}

hipError_t launch_extract(int n, int precision, int mode, const KernelArgs& a, int grid,
                          hipStream_t stream) {
  switch (n) {
    case 256: return launch_prec<256>(precision, mode, a, grid, stream);
    case 512: return launch_prec<512>(precision, mode, a, grid, stream);
    case 1024: return launch_prec<1024>(precision, mode, a, grid, stream);
    case 2048: return launch_prec<2048>(precision, mode, a, grid, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_synth(float* out, uint64_t count, uint64_t seed, uint64_t first_index,
                        hipStream_t stream) {
  const uint64_t threads = (count + 3) / 4;
  uint64_t blocks = (threads + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, out, count, seed, first_index);
  return hipGetLastError();
}

}  // namespace mgx
