// Host side of the C ABI (include/meyda_gpu.h): plan construction, host tables,
// device residency, launches and error reporting.
//
// Host tables follow the reference formulas evaluated in IEEE double exactly as
// the JavaScript does (this file is compiled with -ffp-contract=off); the
// golden tests compare them bit-for-bit with the reference's own tables
// (tests/test_capi_host.py).
#include <hip/hip_runtime.h>
#include <emmintrin.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mgx_internal.h"

namespace {
thread_local std::string g_last_error;
}  // namespace

namespace mgx {
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  const int code = (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? MGX_E_OUT_OF_MEMORY : MGX_E_DEVICE;
  return fail(code, "%s: %s", what, hipGetErrorString(e));
}
}  // namespace mgx

namespace {
using mgx::fail;
using mgx::hip_fail;

const uint64_t kHostChunk = 65536;              // frames per host-staging chunk
// Host batches of at most this many frames (a real-time buffer, or a streaming batch of K
// buffers) skip the device staging: the frames are copied into plan-owned pinned host memory
// that the kernel reads over PCIe itself, and it writes the features back there (no DMA copies,
// no cross-stream events: one launch and one stream synchronisation per call). Overridden by
// $MGX_SMALL_BATCH_FRAMES at plan creation (0: always the staged path).
const uint64_t kSmallBatchFrames = 512;
// How long the small path spins on its completion word before it blocks on the stream (a
// 512-frame batch takes ~0.1 ms; a longer wait is a busy device, where blocking frees the core).
const int kSmallSpinUs = 2000;
// Resident launches (MGX_FLAG_RESIDENT) started and not yet seen to end, per device: each holds one workgroup
// slot of one CU, so the persistent grid of any other launch on the device is that much smaller (a grid of
// exactly the resident workgroups would leave one workgroup -- its whole share of the launch -- waiting for a
// slot until the others finish: twice the launch time).
constexpr int kMaxDevices = 64;
std::atomic<int> g_resident_live[kMaxDevices];
const double kJsPi = 3.141592653589793;        // Math.PI
const double kJsSqrt1_2 = 0.7071067811865476;  // Math.SQRT1_2

const char* const kNames[MGX_NUM_FEATURES] = {
    "rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope",
    "spectralRolloff", "spectralSpread", "spectralSkewness", "spectralKurtosis",
    "loudness.total", "perceptualSpread", "perceptualSharpness", "loudness", "mfcc",
    "amplitudeSpectrum", "powerSpectrum", "complexSpectrum", "buffer"};

// src/feature-info.js:1-65
const int kInfo[MGX_NUM_FEATURES] = {
    MGX_TYPE_NUMBER, MGX_TYPE_NUMBER, MGX_TYPE_NUMBER, MGX_TYPE_NUMBER, MGX_TYPE_NUMBER,
    MGX_TYPE_NUMBER, MGX_TYPE_NUMBER, MGX_TYPE_NUMBER, MGX_TYPE_NUMBER, MGX_TYPE_NUMBER,
    MGX_TYPE_NUMBER, MGX_TYPE_NUMBER, MGX_TYPE_NUMBER, MGX_TYPE_MULTIPLE_ARRAYS, MGX_TYPE_ARRAY,
    MGX_TYPE_ARRAY, MGX_TYPE_ARRAY, MGX_TYPE_MULTIPLE_ARRAYS, MGX_TYPE_ARRAY};

// --------------------------------------------------------------- host tables
// src/meyda.js:128-138
void hanning(int n, float* out) {
  for (int i = 0; i < n; i++) out[i] = (float)(0.5 - 0.5 * cos(2 * kJsPi * i / (n - 1)));
}
// src/meyda.js:116-126
void hamming(int n, float* out) {
  for (int i = 0; i < n; i++) out[i] = (float)(0.54 - 0.46 * cos(2 * kJsPi * ((double)i / n - 1)));
}
// src/meyda.js:170-182 (the frequency is stored to a Float32Array, then read back)
void bark_scale(int n, double sr, float* out) {
  for (int i = 0; i < n; i++) {
    const float f = (float)((double)i * sr / n);
    const double q = (double)f / 7518;
    out[i] = (float)(13 * atan((double)f / 1315.8) + 3.5 * atan(q * q));
  }
}
// src/extractors/loudness.js:24-45. len = N/2 is 0 for bufferSize 1 (a power of two the
// reference accepts): barkScale[-1] is undefined there, so bandEnd is NaN, no limit moves
// and the last one is length - 1 = -1.
void bark_limits(const float* bark, int len, int nb, int32_t* lim) {
  if (len <= 0) {
    for (int i = 0; i < nb; i++) lim[i] = 0;
    lim[nb] = len - 1;
    return;
  }
  double end = (double)bark[len - 1] / nb;
  int band = 1;
  for (int i = 0; i <= nb; i++) lim[i] = 0;
  for (int i = 0; i < len; i++) {
    while ((double)bark[i] > end) {
      if (band <= nb) lim[band] = i;
      band++;
      end = (double)band * bark[len - 1] / nb;
    }
  }
  lim[nb] = len - 1;
}
// src/extractors/mfcc.js:7-38
void mel_bins(int n, double sr, int nf, int32_t* bins) {
  const double lo = 1125 * log(1 + (0.0 / 700));
  const double hi = 1125 * log(1 + ((sr / 2) / 700));
  const double step = (hi - lo) / (nf + 1);
  for (int i = 0; i < nf + 2; i++) {
    const float mv = (float)(i * step);
    const float mf = (float)(700 * (exp((double)mv / 1125) - 1));
    bins[i] = (int32_t)floor((double)(n + 1) * mf / sr);
  }
}
// src/extractors/mfcc.js:67-83
void dct_table(int nf, int nc, float* dct) {
  const double k = kJsPi / nf, w1 = 1.0 / sqrt((double)nf), w2 = sqrt(2.0 / nf);
  for (int i = 0; i < nc; i++)
    for (int j = 0; j < nf; j++) dct[i + j * nc] = (float)((i == 0 ? w1 : w2) * cos(k * (i + 1) * (j + 0.5)));
}
// Logical Hermitian index stored at each slot location of a size-m block.
void klist(int m, std::vector<int>& k) {
  k.assign(m / 2, 0);
  if (m == 2) return;
  std::vector<int> sub;
  klist(m / 2, sub);
  const int w = m / 2, h = w / 2;
  k[0] = 0;
  k[h] = w / 2;
  for (int a = 1; a < h; a++) {
    k[a] = sub[a];
    k[h + a] = w - sub[a];
  }
}
// lib/jsfft/fft.js:140-165: per stage, f_j by the recurrence from (cos pi/w, sin pi/w).
// Entry a of stage q (input blocks of w = 2^(q+1) samples, offset 2^q - 1) holds
// SQRT1_2 * f_{k(a)} (a = 0: SQRT1_2 * f_0); entry N/2 - 1 + q holds SQRT1_2 * f_{w/2}
// (the block-start pair, kernels.hip bfly_special / bfly_mixed).
void twiddles(int n, std::vector<double>& tw) {
  const int L = n / 2;
  int stages = 0;
  for (int w = 2; w <= L; w <<= 1) ++stages;
  tw.assign(2 * (size_t)(L - 1 + stages), 0.0);
  size_t off = 0;
  for (int w = 2; w <= L; w <<= 1) {
    const int h = w / 2;
    const double dr = cos(kJsPi / w), di = sin(kJsPi / w);
    std::vector<double> fr(w), fi(w);
    double r = 1, i = 0;
    for (int j = 0; j < w; j++) {
      fr[j] = r;
      fi[j] = i;
      const double t = r * dr - i * di;
      i = r * di + i * dr;
      r = t;
    }
    std::vector<int> kl;
    klist(w, kl);
    for (int a = 0; a < h; a++) {
      const int k = a == 0 ? 0 : kl[a];
      tw[2 * (off + a)] = kJsSqrt1_2 * fr[k];
      tw[2 * (off + a) + 1] = kJsSqrt1_2 * fi[k];
    }
    // SQRT1_2 * f_{w/2} (block-start pair) after the stage entries
    const size_t fq = (size_t)(L - 1) + (size_t)(__builtin_ctz((unsigned)w) - 1);
    tw[2 * fq] = kJsSqrt1_2 * fr[w / 2];
    tw[2 * fq + 1] = kJsSqrt1_2 * fi[w / 2];
    off += h;
  }
}

// Coefficients of the mixed butterflies (kernels.hip bfly_mixed_tame), same indexing as
// twiddles(): entry a > 0 of stage q holds (f_x, SQRT1_2 f_y) with f = f_{k(a)} unscaled;
// entry 0 (the block-start pair) holds (1, 0), so that fma(b, R, L) is exactly jsfft's
// left + right there; entry N/2 - 1 + q holds (f_{w/2,x}, SQRT1_2 f_{w/2,y}) (lane-uniform).
void mixed_coeffs(int n, std::vector<double>& tm) {
  const int L = n / 2;
  int stages = 0;
  for (int w = 2; w <= L; w <<= 1) ++stages;
  // 4 doubles per entry: (b, c0, t4, kL) (kernels.hip bfly_mixed_tame)
  tm.assign(4 * (size_t)(L - 1 + stages), 0.0);
  size_t off = 0;
  for (int w = 2; w <= L; w <<= 1) {
    const int h = w / 2;
    const double dr = cos(kJsPi / w), di = sin(kJsPi / w);
    std::vector<double> fr(w), fi(w);
    double r = 1, i = 0;
    for (int j = 0; j < w; j++) {
      fr[j] = r;
      fi[j] = i;
      const double t = r * dr - i * di;
      i = r * di + i * dr;
      r = t;
    }
    std::vector<int> kl;
    klist(w, kl);
    // block start: b = 1, c0 = 0, t4 = S f_y(w/2), kL = 0
    tm[4 * off] = 1.0;
    tm[4 * off + 2] = kJsSqrt1_2 * fi[w / 2];
    for (int a = 1; a < h; a++) {
      tm[4 * (off + a)] = fr[kl[a]];
      tm[4 * (off + a) + 1] = kJsSqrt1_2 * fi[kl[a]];
      tm[4 * (off + a) + 2] = kJsSqrt1_2 * fr[kl[a]];
      tm[4 * (off + a) + 3] = -kJsSqrt1_2;
    }
    const size_t fq = (size_t)(L - 1) + (size_t)(__builtin_ctz((unsigned)w) - 1);
    tm[4 * fq] = fr[w / 2];
    tm[4 * fq + 1] = kJsSqrt1_2 * fi[w / 2];
    off += h;
  }
}

// Mel filterbank as per-bin segment tables (kernels.hip mel_energies): bin k lies in
// segment m with b_m <= k < b_{m+1}, m in [0, nf]; band j rises over segment j and falls
// over segment j + 1 (mfcc.js:43-50). Bins at or past b_{nf+1} belong to no band.
void mel_segments(const int32_t* b, int nf, int L, std::vector<float>& wud, std::vector<uint8_t>& seg) {
  wud.assign(2 * (size_t)L, 0.0f);
  seg.assign(L, (uint8_t)(nf + 1));
  for (int k = 0; k < L; ++k) {
    int m = -1;
    for (int j = 0; j <= nf; ++j)
      if (b[j] <= k && k < b[j + 1]) m = j;
    if (m < 0) continue;
    seg[k] = (uint8_t)m;
    wud[2 * k] = (float)((double)(k - b[m]) / (b[m + 1] - b[m]));
    wud[2 * k + 1] = (float)((double)(b[m + 1] - k) / (b[m + 1] - b[m]));
  }
}

// Per-lane form of the segment tables for kernels.hip mel_energies (lane t owns bins
// [R t, R t + R), R = L / 64), one record of mgx::mel_rec_words(R) dwords per lane:
//   weights       per bin the rising weight and, up to R = 8, the falling one 1 - rising in
//                 float32 as a pair (the kernel forms it itself above)
//   R bytes       keep (1, or 0 where a segment starts: the sums restart)
//   8 bytes       keeps (0/1) of the 6 segmented-scan steps
//   2 words       the assembly offsets of band t (below)
// Dense layout of the wave's slot buffer (float2 (U, D) entries): lane t stores its running sums
// before bin jj >= 1 at entry (jj - 1) * 64 + t (fixed offsets, no per-bin address), the segmented
// scan's carry into it at (R - 1) * 64 + t, lane 63 the segment still open at the last bin at
// R * 64 and lane 0 a zero at R * 64 + 1. Segment m's total is carry-or-zero + entry: the running
// sum before the bin that starts the next segment (or the zero when that bin opens a lane), plus
// the carry into that lane when m began in an earlier lane; lane 63's inclusive scan value when m
// is open at the last bin; 0 when m has no bin. Band j (lane j < nf) sums U_j and D_{j+1} from the
// byte offsets (cU | dU << 16, cD | dD << 16). The scan keeps replay the flag logic of a
// Hillis-Steele segmented scan over the kernel's DPP steps (row_shr 1, 2, 4, 8; row_bcast 15 on
// rows 1, 3; row_bcast 31 on rows 2, 3), which depends only on which lanes hold a segment start.
void mel_lane_tables(const std::vector<uint8_t>& seg, const std::vector<float>& wud, int nf, int L,
                     std::vector<uint32_t>& rec) {
  const int R = L / 64, sink = nf + 1, W = mgx::mel_rec_words(R), B = (R + 3) / 4, WW = mgx::mel_weight_words(R);
  rec.assign((size_t)W * 64, 0u);
  const uint32_t zero = 8u * (uint32_t)(R * 64 + 1), tail = 8u * (uint32_t)(R * 64);
  bool seen[64];
  for (int t = 0; t < 64; ++t) {
    uint32_t* r = &rec[(size_t)W * t];
    uint8_t* keeps = reinterpret_cast<uint8_t*>(r + WW);
    seen[t] = false;
    for (int jj = 0; jj < R; ++jj) {
      const int k = R * t + jj;
      const int prevseg = k == 0 ? sink : seg[k - 1];
      const bool start = seg[k] != prevseg;
      if (start) seen[t] = true;
      keeps[jj] = start ? 0 : 1;
      if (WW == 2 * R) {  // (rise, 1 - rise): the falling weight the kernel would form, in float32
        const float up = wud[2 * k], dn = 1.0f - up;
        memcpy(&r[2 * jj], &up, 4);
        memcpy(&r[2 * jj + 1], &dn, 4);
      } else {
        memcpy(&r[jj], &wud[2 * k], 4);
      }
    }
  }
  // (carry-or-zero, entry) byte offsets of segment m's total
  auto total = [&](int m, uint32_t& c, uint32_t& d) {
    int first = -1, last = -1;
    for (int k = 0; k < L; ++k)
      if (seg[k] == m) {
        if (first < 0) first = k;
        last = k;
      }
    c = d = zero;
    if (first < 0) return;           // an empty segment: 0
    const int next = last + 1;
    if (next == L) {                 // open at the last bin: lane 63's inclusive scan value
      d = tail;
      return;
    }
    const int e = next / R, pos = next % R;
    if (first < e * R) c = 8u * (uint32_t)((R - 1) * 64 + e);  // started in an earlier lane: + its carry
    if (pos > 0) d = 8u * (uint32_t)((pos - 1) * 64 + e);       // the running sum before the next start
  };
  for (int j = 0; j < 64; ++j) {
    uint32_t cU = zero, dU = zero, cD = zero, dD = zero;
    if (j < nf) {
      total(j, cU, dU);
      total(j + 1, cD, dD);
    }
    uint32_t* r = &rec[(size_t)W * j];
    r[WW + B + 2] = cU | dU << 16;
    r[WW + B + 3] = cD | dD << 16;
  }
  bool f[64];
  for (int t = 0; t < 64; ++t) f[t] = seen[t];
  for (int s = 0; s < 6; ++s) {
    bool g[64];
    for (int t = 0; t < 64; ++t) {
      const int row = t / 16;
      int src = -1;
      if (s < 4) src = (t % 16) >= (1 << s) ? t - (1 << s) : -1;
      else if (s == 4) src = (row == 1 || row == 3) ? row * 16 - 1 : -1;
      else src = (row == 2 || row == 3) ? 31 : -1;
      uint8_t* lane8 = reinterpret_cast<uint8_t*>(&rec[(size_t)W * t + WW + B]);
      // 0 also where the step has no source for this lane: the kernel's row broadcasts write
      // every row (no row mask), so a row outside the step's rows must not add what it receives
      lane8[s] = (f[t] || src < 0) ? 0 : 1;
      g[t] = f[t] || (src >= 0 && f[src]);
    }
    memcpy(f, g, sizeof f);
  }
}

// MGX_FLAG_MFCC_REFERENCE: the mel band sums of mfcc.js:53-62 in the reference's
// own order, as serial chains (kernels.hip mel_chains). Band j's chain walks its bins
// [b_j, b_{j+2}) (clamped to the reference's j < N/2) in ascending order with the weights of
// mfcc.js:43-50 -- (k - b_j) / (b_{j+1} - b_j) rising, (b_{j+2} - k) / (b_{j+2} - b_{j+1}) falling,
// IEEE double quotients as JavaScript forms them -- and the float32 accumulator (every other bin
// adds an exact +0 in the reference for a finite spectrum). F frames x nf such chains run together
// (F = 8: two consecutive batches of a wave, when nf <= kChainPairMaxMel; else the batch's 4).
// A chain runs in whole groups of 8 steps from its first bin rounded down to 4 (16-byte row loads),
// or earlier if it would run past N/2, with leading zero weights (a zero weight times a finite
// power adds +0); a band without bins (low bands of many-band plans) has one group of zero
// weights, so its energy is the reference's 0.
// Packed tracks: the 64 lanes are 64 / F tracks x the F frames (lane = track * F + frame). The
// bands are dealt to the tracks longest first, each to the least loaded track, and a track runs its
// bands' chains back to back, so the lanes stay busy for ngroups = the largest track load (N = 1024,
// 26 bands: 18 groups instead of the 24 of phases whose length is the phase's longest chain).
//   ctl[g * 64 + lane], g < ngroups (the lane's row and what happens at the group's start):
//     bits 0-12 the row offset in floats (frame * L + bin), bit 25 a chain starts here (its first
//     step adds to 0), bit 26 the finished chain before it is
//     stored at bits 13-24 (a byte offset into the wave's frame records: FrameRec::lm of its frame
//     and band); without bit 26 the store goes to the lane's scratch word.
//   ctl[ngroups * 64 + lane]: the store of the lane's last chain (bit 26 and bits 13-24 only).
//   w[track * ngroups * 8 + s]: the weight of the track's step s (0 past its last chain).
struct ChainSched {
  int ngroups = 0;
  std::vector<uint32_t> ctl;
  std::vector<double> w;
};
// (the control word's fields hold every plan: 8 frames' rows at N = kChainMaxN, the last record's lm[63])
static_assert(8 * (mgx::kChainMaxN / 2) - 1 <= 0x1FFF, "row offsets fit bits 0-12");
static_assert(3 * mgx::kRecBytes + mgx::kRecLmOff + 4 * (mgx::kMaxMel - 1) <= 0xFFF, "record offsets fit bits 13-24");
void chain_schedule(const int32_t* b, int nf, int L, int F, ChainSched& cs) {
  const int ntr = 64 / F;
  std::vector<int> lo(nf), len(nf), order;
  for (int j = 0; j < nf; ++j) {
    const int first = std::min<int>(b[j], L), end = std::min<int>(b[j + 2], L);
    lo[j] = first / 4 * 4;
    len[j] = std::max(8, (std::max(0, end - lo[j]) + 7) / 8 * 8);
    if (lo[j] + len[j] > L) lo[j] = L - len[j];  // (L and len multiples of 8)
    order.push_back(j);
  }
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return len[x] > len[y]; });
  std::vector<std::vector<int>> track(ntr);
  std::vector<int> load(ntr, 0);
  for (int j : order) {
    int t = 0;
    for (int u = 1; u < ntr; ++u)
      if (load[u] < load[t]) t = u;
    track[t].push_back(j);
    load[t] += len[j];
  }
  const int ng = *std::max_element(load.begin(), load.end()) / 8;
  cs.ngroups = ng;
  cs.ctl.assign((size_t)(ng + 1) * 64, 0u);
  cs.w.assign((size_t)ntr * ng * 8, 0.0);
  auto target = [&](int j, int f) {  // byte offset of FrameRec::lm[band (+32: a pair's first batch)]
    const int lmo = (F == 8 && f < 4) ? 32 : 0;
    return (uint32_t)((f & 3) * mgx::kRecBytes + mgx::kRecLmOff + 4 * (j + lmo)) << 13 | 1u << 26;
  };
  for (int t = 0; t < ntr; ++t) {
    double* w = cs.w.data() + (size_t)t * ng * 8;
    int g0 = 0;
    for (size_t c = 0; c < track[t].size(); ++c) {
      const int j = track[t][c];
      for (int s = 0; s < len[j]; ++s) {
        const int k = lo[j] + s;
        double v = 0.0;
        if (k >= b[j] && k < b[j + 1] && k < L) v = (double)(k - b[j]) / (double)(b[j + 1] - b[j]);
        else if (k >= b[j + 1] && k < b[j + 2] && k < L) v = (double)(b[j + 2] - k) / (double)(b[j + 2] - b[j + 1]);
        w[g0 * 8 + s] = v;
      }
      for (int f = 0; f < F; ++f) {
        const int lane = t * F + f;
        for (int g = g0; g < g0 + len[j] / 8; ++g) {
          uint32_t c32 = (uint32_t)(f * L + lo[j] + 8 * (g - g0));
          if (g == g0) c32 |= 1u << 25 | (c > 0 ? target(track[t][c - 1], f) : 0u);
          cs.ctl[(size_t)g * 64 + lane] = c32;
        }
      }
      g0 += len[j] / 8;
    }
    for (int f = 0; f < F; ++f) {
      const int lane = t * F + f;
      // past the track's last chain: bin 0 of the frame with zero weights (adds +0); no reset
      for (int g = g0; g < ng; ++g) cs.ctl[(size_t)g * 64 + lane] = (uint32_t)(f * L);
      cs.ctl[(size_t)ng * 64 + lane] = track[t].empty() ? 0u : target(track[t].back(), f);
    }
  }
}

int validate(const mgx_plan_desc* d) {
  if (!d) return fail(MGX_E_INVALID_ARGUMENT, "plan descriptor is NULL");
  if (d->struct_size != sizeof(mgx_plan_desc))
    return fail(MGX_E_INVALID_ARGUMENT, "mgx_plan_desc.struct_size is %u, expected %zu", d->struct_size, sizeof(mgx_plan_desc));
  if (!mgx_is_power_of_two((double)d->buffer_size))
    return fail(MGX_E_NOT_POWER_OF_TWO, "Buffer size is not a power of two: Meyda will not run.");
  if (!(d->sample_rate > 0) || !std::isfinite(d->sample_rate))
    return fail(MGX_E_INVALID_ARGUMENT, "sample_rate must be positive and finite");
  if (d->window > MGX_WINDOW_HAMMING) return fail(MGX_E_INVALID_ARGUMENT, "unknown window %u", d->window);
  if (d->precision > MGX_PRECISION_FAST) return fail(MGX_E_INVALID_ARGUMENT, "unknown precision %u", d->precision);
  if (d->mode > MGX_MODE_LITERAL) return fail(MGX_E_INVALID_ARGUMENT, "unknown mode %u", d->mode);
  if (d->num_bark_bands != mgx::kBark) return fail(MGX_E_UNSUPPORTED, "num_bark_bands must be 24 (loudness.js)");
  if (d->num_mel_bands < 1 || d->num_mel_bands > (uint32_t)mgx::kMaxMel)
    return fail(MGX_E_UNSUPPORTED, "num_mel_bands must be in [1, %d]", mgx::kMaxMel);
  if (d->num_mfcc_coeffs < 1 || d->num_mfcc_coeffs > (uint32_t)mgx::kMaxCoeffs)
    return fail(MGX_E_UNSUPPORTED, "num_mfcc_coeffs must be in [1, %d]", mgx::kMaxCoeffs);
  if (d->flags & ~(MGX_FLAG_DCT_SEQUENTIAL | MGX_FLAG_MFCC_REFERENCE | MGX_FLAG_RESIDENT)) return fail(MGX_E_INVALID_ARGUMENT, "unknown plan flags 0x%x", d->flags);
  return MGX_OK;
}

template <typename T>
size_t carve(size_t& off, size_t count) {
  off = (off + 255) / 256 * 256;
  const size_t at = off;
  off += count * sizeof(T);
  return at;
}

}  // namespace

struct mgx_plan {
  mgx_plan_desc d;
  int n = 0, L = 0;
  unsigned char* dev = nullptr;
  void* lds_image = nullptr;  // DevTables::lds_image (its own allocation)
  mgx::DevTables t{};
  double freq_sum = 0, pow_freq_sum = 0, nyq = 0, sharp_tail = 0;
  int grid_cap = 1;
  int cus = 0;  // compute units of the plan's device
  int chain_groups = 0;  // MGX_FLAG_MFCC_REFERENCE: 8-step groups of the mel chains (chain_schedule)
  int chain_pair = 0;  // ... over two consecutive batches of a wave (8 frames)
  // Per-stream device scratch, one set per stream a launch used (the launches of one stream run
  // in order, those of two streams may overlap): the scalar windows (kernels.hip scalar_pass) and,
  // for the reference-order MFCC, the mel chains' power rows (mel_chains). Each set's event is
  // recorded after every launch that uses it, so destroy waits for exactly those launches (the
  // stream itself may be gone by then).
  struct ChainRing {
    void* stream;
    uint64_t* scal;
    float* rows;  // null until a reference-order MFCC launch on the stream
    hipEvent_t done;
    uint64_t* pool_ctr = nullptr;  // the tail pool's ticket counter (KernelArgs::pool_ctr; N = 2048 plans)
  };
  std::vector<ChainRing> chain_rings;
  // two device slots for mgx_extract_host (copy of chunk i+1 beside the extraction of chunk i)
  float* s_frames[2] = {nullptr, nullptr};
  unsigned char* s_out[2] = {nullptr, nullptr};
  size_t s_out_bytes = 0;
  uint64_t s_chunk = 0;
  unsigned char* s_pcm[2] = {nullptr, nullptr};  // raw PCM slots for mgx_extract_host_pcm
  uint64_t s_pcm_bytes = 0;
  hipStream_t s_copy = nullptr, s_comp = nullptr;
  hipEvent_t ev_loaded[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr}, ev_back[2] = {nullptr, nullptr};
  // small host batches (kSmallBatchFrames): pinned, device-mapped, coherent host buffers
  uint64_t small_max = kSmallBatchFrames;
  int pool_pct = 15;  // the N = 2048 tail pool's share of the groups, percent (MGX_POOL_PCT overrides; 0: off)
  // a launch whose frames exceed this many bytes reads them with non-temporal loads (KernelArgs::nt_frames):
  // the MALL's 256 MiB (MGX_NT_MIN_MB overrides, in MiB)
  uint64_t nt_min_bytes = 256ull << 20;
  // the small path's completion word (KernelArgs::done_flag): a mapped host word, the device
  // counter of finished waves and the launch sequence number
  uint32_t* h_done = nullptr;
  // the device addresses of h_in, h_out and h_done (looked up once per allocation, not per call)
  void* d_in_map = nullptr;
  void* d_out_map = nullptr;
  uint32_t* d_done_map = nullptr;
  uint32_t* d_done_count = nullptr;
  uint32_t done_seq = 0;
  float* h_in = nullptr;
  unsigned char* h_out = nullptr;
  size_t h_in_bytes = 0, h_out_bytes = 0;
  // MGX_FLAG_RESIDENT: one-frame host calls served by a launch that stays on the device (resident_request)
  bool resident = false;
  uint32_t res_idle_ms = 20;   // its idle timeout (MGX_RESIDENT_IDLE_MS overrides)
  bool res_light = false;      // MGX_RESIDENT_POLL=light: the launch polls the first word only (kernels.hip res_wait)
  hipStream_t s_res = nullptr; // its own stream: nothing else is queued behind it
  uint64_t* h_mail = nullptr;  // pinned, mapped: N request words (KernelArgs::res_mail), then the exit word
  uint64_t* d_mail = nullptr;  // the device address of h_mail
  bool res_live = false;       // a resident launch was started and has not been seen to end
  uint32_t res_key = 0;        // the outputs it writes (bit k: output k of mgx_outputs requested)
  uint32_t res_next = 0;       // the request number it waits for next
};

namespace {
// resident: the launch is the plan's resident server (MGX_FLAG_RESIDENT), serving requests seq, seq + 1, ...
struct ResidentLaunch {
  uint32_t seq;
};
int extract_device_impl(mgx_plan* p, const float* frames, uint64_t nframes, const mgx_outputs* o, void* stream,
                        const uint32_t* done, const float* inline_frame = nullptr, const ResidentLaunch* res = nullptr);
void resident_stop(mgx_plan* p);
}  // namespace

extern "C" {

int mgx_abi_version(void) { return MGX_ABI_VERSION; }
const char* mgx_last_error(void) { return g_last_error.c_str(); }

// src/utils.js:13-19
int mgx_is_power_of_two(double num) {
  while (fmod(num, 2.0) == 0.0 && num > 1) num /= 2;
  return num == 1;
}

int mgx_feature_index(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < MGX_NUM_FEATURES; ++i)
    if (strcmp(name, kNames[i]) == 0) return i;
  return -1;
}
const char* mgx_feature_name(int f) { return (f >= 0 && f < MGX_NUM_FEATURES) ? kNames[f] : nullptr; }
int mgx_feature_info(int f) { return (f >= 0 && f < MGX_NUM_FEATURES) ? kInfo[f] : -1; }

void mgx_plan_desc_init(mgx_plan_desc* d) {
  if (!d) return;
  memset(d, 0, sizeof *d);
  d->struct_size = sizeof *d;
  d->buffer_size = 512;
  d->sample_rate = 44100.0;
  d->window = MGX_WINDOW_HANNING;
  d->precision = MGX_PRECISION_FAITHFUL;
  d->mode = MGX_MODE_PER_BUFFER_FFT;
  d->num_bark_bands = 24;
  d->num_mel_bands = 26;
  d->num_mfcc_coeffs = 13;
  d->scalar_f64 = 0;
  d->device = 0;
}

int mgx_device_count(int* count) {
  if (!count) return fail(MGX_E_INVALID_ARGUMENT, "count is NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *count = c;
  return MGX_OK;
}

int mgx_get_host_tables(const mgx_plan_desc* d, const mgx_host_tables* out) {
  int rc = validate(d);
  if (rc) return rc;
  if (!out) return fail(MGX_E_INVALID_ARGUMENT, "tables is NULL");
  const int n = (int)d->buffer_size, nf = (int)d->num_mel_bands, nc = (int)d->num_mfcc_coeffs;
  std::vector<float> han(n), ham(n), bark(n);
  hanning(n, han.data());
  hamming(n, ham.data());
  bark_scale(n, d->sample_rate, bark.data());
  if (out->hanning) memcpy(out->hanning, han.data(), n * sizeof(float));
  if (out->hamming) memcpy(out->hamming, ham.data(), n * sizeof(float));
  if (out->window) memcpy(out->window, d->window == MGX_WINDOW_HAMMING ? ham.data() : han.data(), n * sizeof(float));
  if (out->bark_scale) memcpy(out->bark_scale, bark.data(), n * sizeof(float));
  if (out->bark_limits) bark_limits(bark.data(), n / 2, mgx::kBark, out->bark_limits);
  if (out->mel_bins) mel_bins(n, d->sample_rate, nf, out->mel_bins);
  if (out->dct) dct_table(nf, nc, out->dct);
  return MGX_OK;
}

int mgx_plan_create(const mgx_plan_desc* d, mgx_plan** out) {
  if (!out) return fail(MGX_E_INVALID_ARGUMENT, "out_plan is NULL");
  *out = nullptr;
  int rc = validate(d);
  if (rc) return rc;
  const int n = (int)d->buffer_size;
  if (n < 256 || n > 2048)
    return fail(MGX_E_UNSUPPORTED, "buffer_size %d: the GPU path supports 256..2048", n);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MGX_E_NO_DEVICE, "no HIP device available");
  if (d->device < 0 || d->device >= ndev) return fail(MGX_E_INVALID_ARGUMENT, "device %d out of range (%d devices)", d->device, ndev);
  hipError_t e = hipSetDevice(d->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, d->device);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(MGX_E_NO_DEVICE, "device %d is %s; this build targets gfx950 (MI355X)", d->device, prop.gcnArchName);

  const int L = n / 2, nf = (int)d->num_mel_bands, nc = (int)d->num_mfcc_coeffs;
  std::vector<float> han(n), ham(n), bark(n), dct((size_t)nc * nf);
  hanning(n, han.data());
  hamming(n, ham.data());
  bark_scale(n, d->sample_rate, bark.data());
  int32_t lim[mgx::kBark + 1];
  bark_limits(bark.data(), L, mgx::kBark, lim);
  std::vector<int32_t> bins(nf + 2);
  mel_bins(n, d->sample_rate, nf, bins.data());
  dct_table(nf, nc, dct.data());
  std::vector<double> tw;
  twiddles(n, tw);
  std::vector<double> twm;
  mixed_coeffs(n, twm);
  std::vector<float> twf(tw.size());
  for (size_t i = 0; i < tw.size(); ++i) twf[i] = (float)tw[i];
  std::vector<int> kl;
  klist(n, kl);
  std::vector<float> mwud;
  std::vector<uint8_t> mseg;
  mel_segments(bins.data(), nf, L, mwud, mseg);
  std::vector<uint32_t> mrec;
  mel_lane_tables(mseg, mwud, nf, L, mrec);
  const bool chain = (d->flags & MGX_FLAG_MFCC_REFERENCE) && d->mode == MGX_MODE_PER_BUFFER_FFT &&
                     d->precision == MGX_PRECISION_FAITHFUL && n <= mgx::kChainMaxN;
  ChainSched cs;
  const bool pair = chain && nf <= mgx::kChainPairMaxMel;
  if (chain) chain_schedule(bins.data(), nf, L, pair ? 8 : 4, cs);

  if ((d->flags & MGX_FLAG_RESIDENT) && (d->precision != MGX_PRECISION_FAITHFUL || d->mode != MGX_MODE_PER_BUFFER_FFT || chain))
    return fail(MGX_E_UNSUPPORTED, "MGX_FLAG_RESIDENT: faithful per-buffer plans without MGX_FLAG_MFCC_REFERENCE only");

  auto* p = new mgx_plan();
  p->d = *d;
  p->resident = (d->flags & MGX_FLAG_RESIDENT) != 0;
  p->n = n;
  p->L = L;
  // spectralSlope.js:9-16 input-independent sums, in the reference's order
  for (int i = 0; i < L; i++) {
    const double f = (double)i * d->sample_rate / n;
    p->pow_freq_sum += f * f;
    p->freq_sum += f;
  }
  p->nyq = d->sample_rate / (2.0 * (L - 1));  // spectralRolloff.js:4
  for (int i = 15; i < mgx::kBark; ++i) p->sharp_tail += 0.066 * exp(0.171 * (i + 1));  // perceptualSharpness.js:10
  // persistent grid: exactly the workgroups that are resident at once
  p->grid_cap = prop.multiProcessorCount * std::max(1, mgx::extract_blocks_per_cu(n, (int)d->precision, (int)d->mode, (int)d->num_mfcc_coeffs, (int)d->num_mel_bands, chain));
  p->chain_groups = cs.ngroups;
  p->chain_pair = pair;
  p->cus = prop.multiProcessorCount;
  // (tuning knob: MGX_GRID_CAP overrides the persistent grid's size; MGX_GRID_CAP=print reports it)
  if (const char* gc = getenv("MGX_GRID_CAP")) {
    if (strcmp(gc, "print") == 0) fprintf(stderr, "mgx: grid_cap %d (%d CUs)\n", p->grid_cap, prop.multiProcessorCount);
    else if (atoi(gc) > 0) p->grid_cap = atoi(gc);
  }
  if (const char* sb = getenv("MGX_SMALL_BATCH_FRAMES")) p->small_max = (uint64_t)std::max(0, atoi(sb));
  if (const char* pp = getenv("MGX_POOL_PCT")) p->pool_pct = std::min(50, std::max(0, atoi(pp)));
  if (const char* nm = getenv("MGX_NT_MIN_MB")) p->nt_min_bytes = (uint64_t)std::max(0, atoi(nm)) << 20;
  if (const char* ri = getenv("MGX_RESIDENT_IDLE_MS")) p->res_idle_ms = (uint32_t)std::min(10000, std::max(1, atoi(ri)));
  if (const char* rp = getenv("MGX_RESIDENT_POLL")) p->res_light = strcmp(rp, "light") == 0;

  size_t off = 0;
  const size_t o_win = carve<float>(off, n), o_tw = carve<double>(off, tw.size()),
               o_twf = carve<float>(off, twf.size()), o_twm = carve<double>(off, twm.size()),
               o_kl = carve<int>(off, L),
               o_lim = carve<int>(off, mgx::kBark + 1), o_mw = carve<uint32_t>(off, mrec.size()), o_dct = carve<float>(off, dct.size()),
               o_mb = carve<int32_t>(off, bins.size()), o_cl = carve<uint32_t>(off, cs.ctl.size()),
               o_cw = carve<double>(off, cs.w.size()), o_lt = carve<double>(off, 2 * 64);
  std::vector<unsigned char> host(off, 0);
  auto put = [&](size_t at, const void* src, size_t bytes) { if (bytes) memcpy(host.data() + at, src, bytes); };
  put(o_win, d->window == MGX_WINDOW_HAMMING ? ham.data() : han.data(), n * sizeof(float));
  put(o_tw, tw.data(), tw.size() * sizeof(double));
  put(o_twf, twf.data(), twf.size() * sizeof(float));
  put(o_twm, twm.data(), twm.size() * sizeof(double));
  put(o_kl, kl.data(), L * sizeof(int));
  put(o_lim, lim, sizeof lim);
  put(o_mw, mrec.data(), mrec.size() * sizeof(uint32_t));
  put(o_mb, bins.data(), bins.size() * sizeof(int32_t));
  put(o_dct, dct.data(), dct.size() * sizeof(float));
  put(o_cl, cs.ctl.data(), cs.ctl.size() * sizeof(uint32_t));
  put(o_cw, cs.w.data(), cs.w.size() * sizeof(double));
  {
    // the reference-order MFCC's natural log (kernels.hip ref_ln): per 1/64 of the mantissa range its centre's
    // reciprocal, rounded, and the negated log of that reciprocal, from the 64-bit-mantissa long double log
    double lt[2 * 64];
    for (int k = 0; k < 64; ++k) {
      const double inv = (double)(1.0L / (1.0L + (long double)(2 * k + 1) / 128.0L));
      lt[2 * k] = inv;
      lt[2 * k + 1] = (double)(-logl((long double)inv));
    }
    put(o_lt, lt, sizeof lt);
  }
  e = hipMalloc(reinterpret_cast<void**>(&p->dev), off);
  if (e != hipSuccess) { delete p; return hip_fail(e, "hipMalloc(plan tables)"); }
  e = hipMemcpy(p->dev, host.data(), off, hipMemcpyHostToDevice);
  if (e != hipSuccess) { (void)hipFree(p->dev); delete p; return hip_fail(e, "hipMemcpy(plan tables)"); }
  unsigned char* b = p->dev;
  p->t.window = reinterpret_cast<const float*>(b + o_win);
  p->t.tw = reinterpret_cast<const double2*>(b + o_tw);
  p->t.twf = reinterpret_cast<const float2*>(b + o_twf);
  p->t.twm = reinterpret_cast<const double2*>(b + o_twm);
  p->t.klist = reinterpret_cast<const int*>(b + o_kl);
  p->t.bblim = reinterpret_cast<const int*>(b + o_lim);
  p->t.mel_rec = reinterpret_cast<const uint32_t*>(b + o_mw);
  p->t.mel_bins = reinterpret_cast<const int*>(b + o_mb);
  p->t.dct = reinterpret_cast<const float*>(b + o_dct);
  p->t.chain_ctl = reinterpret_cast<const uint32_t*>(b + o_cl);
  p->t.chain_w = reinterpret_cast<const double*>(b + o_cw);
  p->t.log_tab = reinterpret_cast<const double2*>(b + o_lt);
  // the workgroup's LDS tables as one image (kernels.hip lds_image_kernel), built here once
  {
    const size_t ib = mgx::lds_image_bytes(n, nc, nf);
    mgx::KernelArgs ia{};
    ia.t = p->t;
    ia.nfilt = nf;
    ia.ncoef = nc;
    e = hipMalloc(&p->lds_image, ib);
    if (e == hipSuccess) e = hipMemset(p->lds_image, 0, ib);
    if (e == hipSuccess) e = mgx::launch_lds_image(n, (int)d->precision, (int)d->mode, ia, p->lds_image, nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) {
      if (p->lds_image) (void)hipFree(p->lds_image);
      (void)hipFree(p->dev);
      delete p;
      return hip_fail(e, "plan LDS image");
    }
    p->t.lds_image = p->lds_image;
    p->t.lds_image_chunks = (uint32_t)(ib / 16);
  }
  if (p->resident) {
    // The resident path's one-time set-up here instead of in the first real-time call, where it took ~13 ms
    // (the pinned buffers, the CU-masked stream's hardware queue; profiles/r06_resident.txt): one call on a
    // silent frame with every output (the largest layout), then the launch is ended.
    std::vector<float> z((size_t)n, 0.0f);
    std::vector<double> sc(MGX_NUM_SCALARS);
    std::vector<float> ls(mgx::kBark), mc(nc), am(L), pw(L), cr(n), ci(n);
    mgx_outputs o{};
    for (int i = 0; i < MGX_NUM_SCALARS; ++i) o.scalars[i] = &sc[i];  // (8 bytes each: room for either width)
    o.loudness_specific = ls.data();
    o.mfcc = mc.data();
    o.amplitude_spectrum = am.data();
    o.power_spectrum = pw.data();
    o.complex_real = cr.data();
    o.complex_imag = ci.data();
    int rc = mgx_extract_host(p, z.data(), 1, &o);
    resident_stop(p);
    if (rc) {
      const std::string why = g_last_error;
      mgx_plan_destroy(p);
      return fail(rc, "MGX_FLAG_RESIDENT set-up: %s", why.c_str());
    }
  }
  *out = p;
  return MGX_OK;
}

int mgx_plan_destroy(mgx_plan* p) {
  if (!p) return MGX_OK;
  (void)hipSetDevice(p->d.device);
  // the resident launch ends first (its stop word, then its stream)
  resident_stop(p);
  // every launch that used the plan's memory is done first: the plan's own streams, then the
  // caller streams' scratch events (launches on s_comp record none)
  if (p->s_copy) (void)hipStreamSynchronize(p->s_copy);
  if (p->s_comp) (void)hipStreamSynchronize(p->s_comp);
  for (auto& r : p->chain_rings) (void)hipEventSynchronize(r.done);
  if (p->dev) (void)hipFree(p->dev);
  if (p->lds_image) (void)hipFree(p->lds_image);
  for (auto& r : p->chain_rings) {
    (void)hipEventDestroy(r.done);
    if (r.scal) (void)hipFree(r.scal);
    if (r.rows) (void)hipFree(r.rows);
    if (r.pool_ctr) (void)hipFree(r.pool_ctr);
  }
  for (int i = 0; i < 2; ++i) {
    if (p->s_frames[i]) (void)hipFree(p->s_frames[i]);
    if (p->s_out[i]) (void)hipFree(p->s_out[i]);
    if (p->s_pcm[i]) (void)hipFree(p->s_pcm[i]);
    for (hipEvent_t ev : {p->ev_loaded[i], p->ev_done[i], p->ev_back[i]})
      if (ev) (void)hipEventDestroy(ev);
  }
  if (p->s_copy) (void)hipStreamDestroy(p->s_copy);
  if (p->s_comp) (void)hipStreamDestroy(p->s_comp);
  if (p->s_res) (void)hipStreamDestroy(p->s_res);
  if (p->h_mail) (void)hipHostFree(p->h_mail);
  if (p->h_in) (void)hipHostFree(p->h_in);
  if (p->h_out) (void)hipHostFree(p->h_out);
  if (p->h_done) (void)hipHostFree(p->h_done);
  if (p->d_done_count) (void)hipFree(p->d_done_count);
  delete p;
  return MGX_OK;
}

int mgx_plan_get_desc(const mgx_plan* p, mgx_plan_desc* out) {
  if (!p || !out) return fail(MGX_E_INVALID_ARGUMENT, "NULL argument");
  *out = p->d;
  return MGX_OK;
}

int mgx_extract_device(mgx_plan* p, const float* frames, uint64_t nframes, const mgx_outputs* o, void* stream) {
  return extract_device_impl(p, frames, nframes, o, stream, nullptr);
}

}  // extern "C"

namespace {

// A stream's scratch set (mgx_plan::ChainRing), the whole set at once: the scalar windows (kScalWords words
// for each wave of the largest grid), the reference-order MFCC's power-row ring (2 FPW x N/2 floats per wave;
// MGX_FLAG_MFCC_REFERENCE plans) and the tail pool's ticket counter (N = 2048 plans), zeroed in stream order
// before the first launch. On failure nothing is kept and the next call on the stream tries again.
int add_stream_scratch(mgx_plan* p, void* stream) {
  mgx_plan::ChainRing r{};
  r.stream = stream;
  auto undo = [&r]() {
    if (r.done) (void)hipEventDestroy(r.done);
    if (r.scal) (void)hipFree(r.scal);
    if (r.rows) (void)hipFree(r.rows);
    if (r.pool_ctr) (void)hipFree(r.pool_ctr);
  };
  hipError_t e = hipEventCreateWithFlags(&r.done, hipEventDisableTiming);
  if (e != hipSuccess) { r.done = nullptr; return hip_fail(e, "hipEventCreate(stream scratch)"); }
  e = hipMalloc(reinterpret_cast<void**>(&r.scal), (size_t)p->grid_cap * 4 * mgx::kScalWords * sizeof(uint64_t));
  if (e != hipSuccess) { r.scal = nullptr; undo(); return hip_fail(e, "hipMalloc(scalar windows)"); }
  if (p->chain_groups > 0) {
    const size_t fpw = (size_t)mgx::frames_per_batch(p->n) / 4;
    e = hipMalloc(reinterpret_cast<void**>(&r.rows), (size_t)p->grid_cap * 4 * 2 * fpw * (size_t)p->L * sizeof(float));
    if (e != hipSuccess) { r.rows = nullptr; undo(); return hip_fail(e, "hipMalloc(mel chain rows)"); }
  }
  if (p->n == 2048) {
    e = hipMalloc(reinterpret_cast<void**>(&r.pool_ctr), sizeof(uint64_t));
    if (e != hipSuccess) r.pool_ctr = nullptr;
    else e = hipMemsetAsync(r.pool_ctr, 0, sizeof(uint64_t), (hipStream_t)stream);
    if (e != hipSuccess) { undo(); return hip_fail(e, "tail pool counter"); }
  }
  p->chain_rings.push_back(r);
  return MGX_OK;
}

// mgx_extract_device, and with `done` (the small host path) the launch's completion word; inline_frame
// (the small path's one frame in host memory) goes into the kernel arguments where the kernel takes it
// (mgx::launch_extract); res: the plan's resident launch (resident_request). Any other launch ends the
// plan's resident one first, so the plan's own work never waits behind it or shares the device with it.
int extract_device_impl(mgx_plan* p, const float* frames, uint64_t nframes, const mgx_outputs* o, void* stream,
                        const uint32_t* done, const float* inline_frame, const ResidentLaunch* res) {
  if (!p || !o) return fail(MGX_E_INVALID_ARGUMENT, "NULL plan or outputs");
  if (nframes == 0) return MGX_OK;
  if (!frames) return fail(MGX_E_INVALID_ARGUMENT, "frames is NULL");
  if ((o->complex_real == nullptr) != (o->complex_imag == nullptr))
    return fail(MGX_E_INVALID_ARGUMENT, "complex_real and complex_imag must be given together");
  if (!res) resident_stop(p);
  mgx::KernelArgs a{};
  a.frames = frames;
  a.num_frames = nframes;
  a.t = p->t;
  a.out = *o;
  a.sample_rate = p->d.sample_rate;
  a.freq_sum = p->freq_sum;
  a.pow_freq_sum = p->pow_freq_sum;
  a.nyq_bin = p->nyq;
  a.sharp_tail_sum = p->sharp_tail;
  a.rcp_ncoef = 1.0 / (double)p->d.num_mfcc_coeffs;
  a.nfilt = (int)p->d.num_mel_bands;
  a.ncoef = (int)p->d.num_mfcc_coeffs;
  a.scalar_f64 = (int)p->d.scalar_f64;
  a.dct_sequential = (p->d.flags & MGX_FLAG_DCT_SEQUENTIAL) ? 1 : 0;
  a.chain_groups = p->chain_groups;
  a.chain_pair = p->chain_pair;
  bool spec = o->loudness_specific || o->mfcc || o->amplitude_spectrum || o->power_spectrum || o->complex_real;
  for (int i = MGX_SPECTRAL_CENTROID; i < MGX_NUM_SCALARS; ++i) spec = spec || o->scalars[i];
  a.need_spectrum = spec;
  a.need_loudness = o->loudness_specific || o->scalars[MGX_LOUDNESS_TOTAL] || o->scalars[MGX_PERCEPTUAL_SPREAD] ||
                    o->scalars[MGX_PERCEPTUAL_SHARPNESS];
  a.need_mfcc = o->mfcc != nullptr;
  // moment sums: 2 = S1..S4 and sum log2 a, 1 = S1 only, 0 = none
  a.need_mom = (o->scalars[MGX_SPECTRAL_FLATNESS] || o->scalars[MGX_SPECTRAL_SPREAD] ||
                o->scalars[MGX_SPECTRAL_SKEWNESS] || o->scalars[MGX_SPECTRAL_KURTOSIS]) ? 2
               : (o->scalars[MGX_SPECTRAL_CENTROID] || o->scalars[MGX_SPECTRAL_SLOPE]) ? 1 : 0;
  a.need_prefix = a.need_loudness || o->scalars[MGX_SPECTRAL_ROLLOFF];
  a.need_energy = o->scalars[MGX_RMS] || o->scalars[MGX_ENERGY];
  a.need_zcr = o->scalars[MGX_ZCR] != nullptr;
  bool any_scalar = false;
  for (int i = 0; i < MGX_NUM_SCALARS; ++i) any_scalar = any_scalar || o->scalars[i];
  const uint64_t fb = (uint64_t)mgx::frames_per_batch(p->n);
  const uint64_t nb = (nframes + fb - 1) / fb;
  const int dev_slot = p->d.device >= 0 && p->d.device < kMaxDevices ? p->d.device : 0;
  const int cap = std::max(1, p->grid_cap - (res ? 0 : g_resident_live[dev_slot].load(std::memory_order_relaxed)));
  const int grid = (int)std::min<uint64_t>(nb, (uint64_t)cap);
  a.wg_ranks = grid == p->grid_cap && p->cus > 0 ? p->grid_cap / p->cus : 1;
  // The scalars run once per window of a wave's batches (kernels.hip scalar_pass) when the launch
  // computes a spectrum (VALU-bound there: 0.7-1.9 % faster by N, outputs identical) and its waves
  // get at least 8 batches each on average. A time-only launch is HBM-bound, and the windows' late,
  // per-wave output writes lost it 18 %; with a few batches per wave (C2's 65,536 frames: 3) the
  // one pass at the end of each wave lengthens the launch's tail (+1.6 %). Those, and launches
  // without a scalar output, keep the per-batch form.
  a.scal_defer = a.need_spectrum && any_scalar && nb >= (uint64_t)grid * 8;
  // A batch larger than the MALL is read past the caches: it cannot stay resident between launches, and
  // its lines would evict the ones the launch reads back (the scalar windows); N = 1024 all features
  // -1.2 % per launch, the HBM-bound time-only set -12 % (profiles/r05_prologue_ab.txt, r06_nt_frames.txt).
  // A smaller one keeps plain loads: launches over the same frames then find them in the MALL (C2).
  a.nt_frames = nframes * (uint64_t)p->n * sizeof(float) > p->nt_min_bytes;
  hipError_t e = hipSetDevice(p->d.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  if (res) {
    // the resident launch: one frame per request from the mailbox (the frame pointer only feeds the kernel's
    // ignored prefetch: a valid table), no stream scratch (one frame: no windows, no pool, no chains)
    a.frames = p->t.window;
    a.res_mail = p->d_mail;
    a.res_exit = reinterpret_cast<uint32_t*>(p->d_mail + p->n);
    a.res_seq = res->seq;
    a.res_idle = p->res_idle_ms * 100000u;  // the 100 MHz real-time clock
    a.res_light = p->res_light ? 1 : 0;
    a.done_flag = const_cast<uint32_t*>(done);
    e = mgx::launch_extract(p->n, (int)p->d.precision, (int)p->d.mode, a, 1, (hipStream_t)stream, nullptr, true);
    return e == hipSuccess ? MGX_OK : hip_fail(e, "resident launch");
  }
  // the stream's scratch set: allocated whole by the first launch on the stream, whatever its shape, so one
  // untimed call per stream sets the stream up for every later call (include/meyda_gpu.h)
  mgx_plan::ChainRing* ring = nullptr;
  for (auto& r : p->chain_rings)
    if (r.stream == stream) ring = &r;
  if (!ring) {
    int rc = add_stream_scratch(p, stream);
    if (rc) return rc;
    ring = &p->chain_rings.back();
  }
  if (a.scal_defer) a.scal_rows = ring->scal;
  if (a.chain_groups > 0 && a.need_spectrum && a.need_mfcc) a.chain_rows = ring->rows;
  // The tail pool at N = 2048 (the kernels without a frame prefetch; not the reference-order ones): the
  // last pool_pct percent of the groups taken by ticket (kernels.hip; 15 %: -2.7 % per launch against the static
  // shares alone, outputs identical, profiles/r05_tail_pool.txt).
  if (p->n == 2048 && !(a.chain_groups > 0 && a.need_spectrum && a.need_mfcc) && p->pool_pct > 0) {
    // (nb here counts groups of 16 frames, the kernel's groups; the pool's tickets are batches of 4 frames)
    const uint64_t ng_all = nb, pg = ng_all * (uint64_t)p->pool_pct / 100;
    if (pg > 0 && pg < ng_all && ring->pool_ctr) {
      a.pool_ctr = ring->pool_ctr;
      a.pool_groups = (uint32_t)pg;
    }
  }
  // (a launch on the plan's own compute stream records no event: destroy synchronises that
  // stream, and the small host path saves the record's ~1 us per call)
  // (a NULL caller stream is never the plan's: s_comp may not exist yet, and then both are NULL)
  hipEvent_t ring_done = (p->s_comp != nullptr && stream == static_cast<void*>(p->s_comp)) ? nullptr : ring->done;
  // (a launch captured into a graph records no event either: the graph's replays are the caller's to
  // wait for before mgx_plan_destroy, as any work it launches on the plan's memory)
  if (ring_done) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) ring_done = nullptr;
  }
  if (done) {
    a.done_flag = const_cast<uint32_t*>(done);
    a.done_count = p->d_done_count;
    a.done_seq = p->done_seq;
    a.done_waves = (uint32_t)grid * 4;
  }
  e = mgx::launch_extract(p->n, (int)p->d.precision, (int)p->d.mode, a, grid, (hipStream_t)stream, inline_frame);
  if (e != hipSuccess) return hip_fail(e, "extract kernel launch");
  if (ring_done) {
    e = hipEventRecord(ring_done, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "hipEventRecord(mel chain rows)");
  }
  return MGX_OK;
}

}  // namespace

namespace {

// Host batches: `nframes` frames through two plan-owned device slots, kHostChunk frames at a
// time. `fill(f0, cnt, slot, stream)` enqueues the copy of frames [f0, f0 + cnt) into slot
// `slot` (p->s_frames[slot]) on the copy stream. Chunk i+1's host-to-device copy runs while
// chunk i is extracted on the compute stream; chunk i's outputs then return to the host
// arrays of `o` (laid out over all nframes) on the copy stream.
int ensure_host_staging(mgx_plan* p, uint64_t chunk, size_t out_bytes) {
  hipError_t e = hipSetDevice(p->d.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  if (!p->s_copy) {
    // (the small host path may have created s_comp already: it is created once, never replaced)
    e = hipStreamCreateWithFlags(&p->s_copy, hipStreamNonBlocking);
    if (e == hipSuccess && !p->s_comp) e = hipStreamCreateWithFlags(&p->s_comp, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
      e = hipEventCreateWithFlags(&p->ev_loaded[i], hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ev_done[i], hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ev_back[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) return hip_fail(e, "host staging streams");
  }
  if (p->s_chunk >= chunk && p->s_out_bytes >= out_bytes) return MGX_OK;
  for (int i = 0; i < 2; ++i) {
    if (p->s_frames[i]) (void)hipFree(p->s_frames[i]);
    if (p->s_out[i]) (void)hipFree(p->s_out[i]);
    p->s_frames[i] = nullptr;
    p->s_out[i] = nullptr;
  }
  p->s_chunk = 0;
  p->s_out_bytes = 0;
  for (int i = 0; i < 2; ++i) {
    e = hipMalloc(reinterpret_cast<void**>(&p->s_frames[i]), chunk * p->n * sizeof(float));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(staging frames)");
    e = hipMalloc(reinterpret_cast<void**>(&p->s_out[i]), out_bytes);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(staging outputs)");
  }
  p->s_chunk = chunk;
  p->s_out_bytes = out_bytes;
  return MGX_OK;
}

// Device bytes per frame of the requested outputs (host staging layouts).
size_t out_bytes_per_frame(const mgx_plan* p, const mgx_outputs* o) {
  const size_t ss = p->d.scalar_f64 ? 8 : 4;
  size_t per = 0;
  for (int i = 0; i < MGX_NUM_SCALARS; ++i) per += o->scalars[i] ? ss : 0;
  per += (o->loudness_specific ? (size_t)mgx::kBark * 4 : 0) + (o->mfcc ? (size_t)p->d.num_mfcc_coeffs * 4 : 0) +
         (o->amplitude_spectrum ? (size_t)p->L * 4 : 0) + (o->power_spectrum ? (size_t)p->L * 4 : 0) +
         (o->complex_real ? 2 * (size_t)p->n * 4 : 0);
  return per;
}

// Ends the plan's resident launch if one may be on the device: the stop word into the mailbox's first word
// (kernels.hip res_take), then its stream (one that already ended on its idle timeout costs only the
// synchronisation).
void resident_ended(mgx_plan* p) {
  p->res_live = false;
  g_resident_live[p->d.device >= 0 && p->d.device < kMaxDevices ? p->d.device : 0].fetch_sub(1, std::memory_order_relaxed);
}

void resident_stop(mgx_plan* p) {
  if (!p->res_live) return;
  __atomic_store_n(&p->h_mail[0], (uint64_t)mgx::kResStop << 32, __ATOMIC_RELEASE);
  (void)hipStreamSynchronize(p->s_res);
  resident_ended(p);
}

// bit k: output k of mgx_outputs requested (the scalars, then loudness, mfcc, amplitude, power, complex)
uint32_t output_key(const mgx_outputs* o) {
  uint32_t k = 0;
  for (int i = 0; i < MGX_NUM_SCALARS; ++i) k |= o->scalars[i] ? 1u << i : 0u;
  const void* v[] = {o->loudness_specific, o->mfcc, o->amplitude_spectrum, o->power_spectrum, o->complex_real, o->complex_imag};
  for (int i = 0; i < 6; ++i) k |= v[i] ? 1u << (MGX_NUM_SCALARS + i) : 0u;
  return k;
}

// One frame (in p->h_in) through the plan's resident launch (MGX_FLAG_RESIDENT), its outputs landing in the
// small path's pinned layout h (device addresses d) under request number seq:
//  * a live launch that writes another output layout, or waits for another request number (a call of
//    another kind ended it, or the numbers wrapped), is ended first: its kernel arguments fix both;
//  * the frame goes into the mailbox, each word one 8-byte store tagged with seq (kernels.hip res_wait);
//  * a launch that ended on its idle timeout is collected, and one is started when none is live -- after
//    the post, so its first read finds the frame;
//  * the host spins on the completion word, which the launch releases after each request's outputs (a launch
//    that does not end leaves its plain stores in the GPU's L2 until a release writes them back: the output
//    words themselves cannot be waited on as the one-launch path does). A launch that ends while the host
//    waits (it read the mailbox before the frame landed, then timed out) is started again, twice at most;
//    past 1 s the call fails with the launch ended.
int resident_request(mgx_plan* p, const mgx_outputs* o, const mgx_outputs& d, uint32_t seq) {
  const int n = p->n;
  hipError_t e = hipSuccess;
  const uint32_t key = output_key(o);
  if (p->res_live && (p->res_key != key || p->res_next != seq)) resident_stop(p);
  if (!p->h_mail) {
    uint64_t* hm = nullptr;
    const size_t bytes = (size_t)(n + 8) * sizeof(uint64_t);  // the words, then a 64-byte line for the exit word
    e = hipHostMalloc(reinterpret_cast<void**>(&hm), bytes, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(resident mailbox)");
    memset(hm, 0, bytes);
    e = hipHostGetDevicePointer(reinterpret_cast<void**>(&p->d_mail), hm, 0);
    if (e != hipSuccess) {
      (void)hipHostFree(hm);
      return hip_fail(e, "hipHostGetDevicePointer(resident mailbox)");
    }
    p->h_mail = hm;
  }
  if (!p->s_res) {
    // A stream with a CU mask (every CU) gets a hardware queue of its own: the HIP runtime spreads ordinary
    // streams over a few shared queues, and a queue shared with the resident launch would hold every later
    // kernel of the other stream behind it until its idle timeout (tests/test_gpu_resident.py).
    std::vector<uint32_t> mask((size_t)(p->cus + 31) / 32, 0xFFFFFFFFu);
    e = hipExtStreamCreateWithCUMask(&p->s_res, (uint32_t)mask.size(), mask.data());
    if (e != hipSuccess) return hip_fail(e, "hipExtStreamCreateWithCUMask(resident)");
  }
  // (two words per 16-byte store, the samples interleaved with seq: each aligned 8-byte half is written whole,
  // which is all the device's word-by-word check needs. Half the stores of word-by-word writes; the call's
  // time did not move measurably, the device's reads overlap the post.)
  const float* src = p->h_in;
  const __m128i sq = _mm_set1_epi32((int)seq);
  for (int i = 0; i < n; i += 4) {
    const __m128i xv = _mm_castps_si128(_mm_loadu_ps(src + i));
    _mm_store_si128(reinterpret_cast<__m128i*>(p->h_mail + i), _mm_unpacklo_epi32(xv, sq));
    _mm_store_si128(reinterpret_cast<__m128i*>(p->h_mail + i + 2), _mm_unpackhi_epi32(xv, sq));
  }
  std::atomic_thread_fence(std::memory_order_release);
  uint32_t* const exitw = reinterpret_cast<uint32_t*>(p->h_mail + n);
  auto collect = [&]() -> int {  // the launch has ended (its exit word): its stream, for a fault it may report
    e = hipStreamSynchronize(p->s_res);
    resident_ended(p);
    return e == hipSuccess ? MGX_OK : hip_fail(e, "resident launch");
  };
  auto start = [&]() -> int {
    __atomic_store_n(exitw, 0u, __ATOMIC_RELEASE);
    const ResidentLaunch rl{seq};
    const int rc = extract_device_impl(p, p->t.window, 1, &d, p->s_res, p->d_done_map, nullptr, &rl);
    if (rc) return rc;
    p->res_live = true;
    g_resident_live[p->d.device >= 0 && p->d.device < kMaxDevices ? p->d.device : 0].fetch_add(1, std::memory_order_relaxed);
    p->res_key = key;
    return MGX_OK;
  };
  int rc = MGX_OK;
  if (p->res_live && __atomic_load_n(exitw, __ATOMIC_ACQUIRE) != 0) rc = collect();
  if (!rc && !p->res_live) rc = start();
  if (rc) return rc;
  p->res_next = seq + 1;
  auto landed = [&]() { return __atomic_load_n(p->h_done, __ATOMIC_ACQUIRE) == seq; };
  const auto t0 = std::chrono::steady_clock::now();
  int restarts = 0;
  for (unsigned spins = 0;; ++spins) {
    if (landed()) break;
    __builtin_ia32_pause();
    if ((spins & 63) != 63) continue;
    const auto now = std::chrono::steady_clock::now();
    if (__atomic_load_n(exitw, __ATOMIC_ACQUIRE) != 0) {
      if ((rc = collect())) return rc;
      if (landed()) break;
      if (++restarts > 2) return fail(MGX_E_DEVICE, "resident launch: request %u not answered", seq);
      if ((rc = start())) return rc;
      continue;
    }
    if (now - t0 > std::chrono::seconds(1)) {
      resident_stop(p);
      return fail(MGX_E_DEVICE, "resident launch: request %u not answered within 1 s", seq);
    }
  }
  return MGX_OK;
}

// A small host batch (at most p->small_max frames): the frames into the plan's pinned input
// buffer, one launch that reads them over PCIe and writes the features into the pinned output
// buffer, one synchronisation, the features out to the caller's arrays. `fill(dst)` writes the
// batch's float32 frames to host memory at dst. The buffers are coherent (fine-grained) host
// memory mapped into the device, so no cache of either side holds a stale copy between calls.
template <typename Fill>
int extract_host_small(mgx_plan* p, uint64_t nframes, const mgx_outputs* o, Fill fill) {
  const int n = p->n, L = p->L;
  const size_t ss = p->d.scalar_f64 ? 8 : 4;
  const size_t nb = mgx::kBark, nc = p->d.num_mfcc_coeffs;
  const size_t in_bytes = nframes * (size_t)n * sizeof(float);
  const size_t out_bytes = out_bytes_per_frame(p, o) * nframes + 20 * 256;
  hipError_t e = hipSetDevice(p->d.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  if (!p->s_comp) {
    e = hipStreamCreateWithFlags(&p->s_comp, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
  }
  // (a one-frame call may return before its launch has ended (the output words below): nothing may free
  // or reuse the pinned buffers under it)
  if (p->h_in_bytes < in_bytes || p->h_out_bytes < out_bytes) {
    resident_stop(p);  // (it writes into h_out)
    e = hipStreamSynchronize(p->s_comp);
    if (e != hipSuccess) return hip_fail(e, "small host batch (previous launch)");
  }
  if (p->h_in_bytes < in_bytes) {
    if (p->h_in) (void)hipHostFree(p->h_in);
    p->h_in = nullptr;
    p->h_in_bytes = 0;
    const size_t want = std::max<size_t>(in_bytes, 16 * (size_t)n * sizeof(float));
    e = hipHostMalloc(reinterpret_cast<void**>(&p->h_in), want, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(small batch frames)");
    e = hipHostGetDevicePointer(&p->d_in_map, p->h_in, 0);
    if (e != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer(small batch frames)");
    p->h_in_bytes = want;
  }
  if (p->h_out_bytes < out_bytes) {
    if (p->h_out) (void)hipHostFree(p->h_out);
    p->h_out = nullptr;
    p->h_out_bytes = 0;
    e = hipHostMalloc(reinterpret_cast<void**>(&p->h_out), out_bytes, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(small batch outputs)");
    e = hipHostGetDevicePointer(&p->d_out_map, p->h_out, 0);
    if (e != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer(small batch outputs)");
    p->h_out_bytes = out_bytes;
  }
  int rc = fill(p->h_in);
  if (rc) return rc;
  void* const din = p->d_in_map;
  void* const dout = p->d_out_map;
  mgx_outputs d{};
  const mgx_outputs h = [&] {  // the same layout, host addresses
    mgx_outputs r{};
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t at = off; off += (bytes + 255) / 256 * 256; return at; };
    size_t at[19];
    for (int k = 0; k < MGX_NUM_SCALARS; ++k) at[k] = o->scalars[k] ? take(nframes * ss) : 0;
    at[13] = o->loudness_specific ? take(nframes * nb * 4) : 0;
    at[14] = o->mfcc ? take(nframes * nc * 4) : 0;
    at[15] = o->amplitude_spectrum ? take(nframes * L * 4) : 0;
    at[16] = o->power_spectrum ? take(nframes * L * 4) : 0;
    at[17] = o->complex_real ? take(nframes * (size_t)n * 4) : 0;
    at[18] = o->complex_imag ? take(nframes * (size_t)n * 4) : 0;
    unsigned char* dv = static_cast<unsigned char*>(dout);
    for (int k = 0; k < MGX_NUM_SCALARS; ++k) {
      d.scalars[k] = o->scalars[k] ? dv + at[k] : nullptr;
      r.scalars[k] = o->scalars[k] ? p->h_out + at[k] : nullptr;
    }
    auto both = [&](bool want, size_t a, float*& dd, float*& hh) {
      dd = want ? reinterpret_cast<float*>(dv + a) : nullptr;
      hh = want ? reinterpret_cast<float*>(p->h_out + a) : nullptr;
    };
    both(o->loudness_specific, at[13], d.loudness_specific, r.loudness_specific);
    both(o->mfcc, at[14], d.mfcc, r.mfcc);
    both(o->amplitude_spectrum, at[15], d.amplitude_spectrum, r.amplitude_spectrum);
    both(o->power_spectrum, at[16], d.power_spectrum, r.power_spectrum);
    both(o->complex_real, at[17], d.complex_real, r.complex_real);
    both(o->complex_imag, at[18], d.complex_imag, r.complex_imag);
    return r;
  }();
  if (!p->h_done) {
    uint32_t* hd = nullptr;
    e = hipHostMalloc(reinterpret_cast<void**>(&hd), 64, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(completion word)");
    *hd = 0;
    e = hipMalloc(reinterpret_cast<void**>(&p->d_done_count), sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(p->d_done_count, 0, sizeof(uint32_t));
    if (e != hipSuccess) {
      (void)hipHostFree(hd);
      return hip_fail(e, "completion counter");
    }
    e = hipHostGetDevicePointer(reinterpret_cast<void**>(&p->d_done_map), hd, 0);
    if (e != hipSuccess) {
      (void)hipHostFree(hd);
      return hip_fail(e, "hipHostGetDevicePointer(completion word)");
    }
    p->h_done = hd;
  }
  uint32_t* const ddone = p->d_done_map;
  // never 0 (the word's initial value) nor the resident launch's stop word
  p->done_seq = (p->done_seq + 1 == 0 || p->done_seq + 1 == mgx::kResStop) ? 1 : p->done_seq + 1;
  // One frame without spectrum outputs (at most 13 + 24 + 32 words): the host waits on the output words
  // themselves -- each preset to an all-ones NaN and polled until the kernel's store has landed -- and the
  // launch releases no completion word, which spares the system-scope release (a wait for the outputs'
  // write acknowledgements) and the word's own trip back. Stores of 4 and 8 aligned bytes arrive whole. An
  // output that is itself that NaN (a NaN input can carry any payload) only ends the spin at its limit.
  const bool word_wait = nframes == 1 && !o->amplitude_spectrum && !o->power_spectrum && !o->complex_real && !o->complex_imag;
  constexpr uint64_t kSent = ~(uint64_t)0;
  if (word_wait && !(p->resident && nframes == 1)) {
    for (int k = 0; k < MGX_NUM_SCALARS; ++k)
      if (o->scalars[k]) memset(h.scalars[k], 0xFF, ss);
    if (o->loudness_specific) memset(h.loudness_specific, 0xFF, nb * 4);
    if (o->mfcc) memset(h.mfcc, 0xFF, nc * 4);
    std::atomic_thread_fence(std::memory_order_release);
  }
  const bool res = p->resident && nframes == 1;
  if (res) {
    rc = resident_request(p, o, d, p->done_seq);
    if (rc) return rc;
  } else {
    // (one frame: also handed over in the kernel arguments, read there by the kernels that take it)
    rc = extract_device_impl(p, static_cast<const float*>(din), nframes, &d, p->s_comp, word_wait ? nullptr : ddone,
                             nframes == 1 ? p->h_in : nullptr);
    if (rc) {
      (void)hipStreamSynchronize(p->s_comp);
      return rc;
    }
  }
  if (!res && word_wait) {
    const auto t0 = std::chrono::steady_clock::now();
    bool late = false;
    unsigned spins = 0;
    auto wait_word = [&](const void* w, size_t bytes) {
      for (;; ++spins) {
        const uint64_t v = bytes == 8 ? __atomic_load_n(static_cast<const uint64_t*>(w), __ATOMIC_ACQUIRE)
                                      : (uint64_t)__atomic_load_n(static_cast<const uint32_t*>(w), __ATOMIC_ACQUIRE);
        if (v != (bytes == 8 ? kSent : (uint64_t)0xFFFFFFFFu)) return;
        __builtin_ia32_pause();
        if (late || ((spins & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSmallSpinUs))) {
          late = true;
          return;
        }
      }
    };
    for (int k = 0; k < MGX_NUM_SCALARS; ++k)
      if (o->scalars[k]) wait_word(h.scalars[k], ss);
    for (size_t i = 0; o->loudness_specific && i < nb; ++i) wait_word(h.loudness_specific + i, 4);
    for (size_t i = 0; o->mfcc && i < nc; ++i) wait_word(h.mfcc + i, 4);
    if (late) {  // a busy device, a failed launch, or an output equal to the preset: the stream decides
      e = hipStreamSynchronize(p->s_comp);
      if (e != hipSuccess) return hip_fail(e, "small host batch");
    }
  }
  // The last wave of the launch releases done_seq to the host word after every output store is
  // visible (kernels.hip done_signal): polling it returns ~9 us sooner than waiting for the
  // stream (tools/ubench/small_latency.hip). Past 20 ms (a busy device) the wait blocks on the
  // stream instead, which also reports a failed launch. The spin pauses the core between reads
  // (a contended device leaves N-API worker threads waiting here) and gives up after kSmallSpinUs.
  if (!res && !word_wait) {
    const auto t0 = std::chrono::steady_clock::now();
    bool seen = false;
    for (unsigned spins = 0;; ++spins) {
      if (__atomic_load_n(p->h_done, __ATOMIC_ACQUIRE) == p->done_seq) {
        seen = true;
        break;
      }
      __builtin_ia32_pause();
      if ((spins & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSmallSpinUs)) break;
    }
    if (!seen) {
      e = hipStreamSynchronize(p->s_comp);
      if (e != hipSuccess) return hip_fail(e, "small host batch");
      if (__atomic_load_n(p->h_done, __ATOMIC_ACQUIRE) != p->done_seq)
        return fail(MGX_E_DEVICE, "small host batch: the launch completed without its completion word");
    }
  }
  for (int k = 0; k < MGX_NUM_SCALARS; ++k)
    if (o->scalars[k]) memcpy(o->scalars[k], h.scalars[k], nframes * ss);
  if (o->loudness_specific) memcpy(o->loudness_specific, h.loudness_specific, nframes * nb * 4);
  if (o->mfcc) memcpy(o->mfcc, h.mfcc, nframes * nc * 4);
  if (o->amplitude_spectrum) memcpy(o->amplitude_spectrum, h.amplitude_spectrum, nframes * L * 4);
  if (o->power_spectrum) memcpy(o->power_spectrum, h.power_spectrum, nframes * L * 4);
  if (o->complex_real) memcpy(o->complex_real, h.complex_real, nframes * (size_t)n * 4);
  if (o->complex_imag) memcpy(o->complex_imag, h.complex_imag, nframes * (size_t)n * 4);
  return MGX_OK;
}

template <typename Fill>
int extract_host_chunked(mgx_plan* p, uint64_t nframes, const mgx_outputs* o, Fill fill) {
  const int n = p->n, L = p->L;
  const size_t ss = p->d.scalar_f64 ? 8 : 4;
  const size_t nb = mgx::kBark, nc = p->d.num_mfcc_coeffs;
  // device bytes per frame for the requested outputs
  size_t per = 0;
  for (int i = 0; i < MGX_NUM_SCALARS; ++i) per += o->scalars[i] ? ss : 0;
  per += (o->loudness_specific ? nb * 4 : 0) + (o->mfcc ? nc * 4 : 0) + (o->amplitude_spectrum ? L * 4 : 0) +
         (o->power_spectrum ? L * 4 : 0) + (o->complex_real ? 2 * (size_t)n * 4 : 0);
  const uint64_t chunk = std::min<uint64_t>(nframes, kHostChunk);
  int rc = ensure_host_staging(p, chunk, per * chunk + 4096);
  if (rc) return rc;
  const uint64_t nch = (nframes + chunk - 1) / chunk;
  hipError_t e = hipSuccess;
  auto fail_sync = [&](int code) {  // leave no work in flight on the plan's buffers
    (void)hipStreamSynchronize(p->s_comp);
    (void)hipStreamSynchronize(p->s_copy);
    return code;
  };
  rc = fill(0, std::min<uint64_t>(chunk, nframes), 0, p->s_copy);
  if (rc) return fail_sync(rc);
  e = hipEventRecord(p->ev_loaded[0], p->s_copy);
  for (uint64_t i = 0; i < nch && e == hipSuccess; ++i) {
    const int sl = (int)(i & 1);
    const uint64_t f0 = i * chunk, cnt = std::min<uint64_t>(chunk, nframes - f0);
    mgx_outputs d{};
    size_t off = 0;
    auto take = [&](size_t bytes) { unsigned char* q = p->s_out[sl] + off; off += (bytes + 255) / 256 * 256; return q; };
    for (int k = 0; k < MGX_NUM_SCALARS; ++k) d.scalars[k] = o->scalars[k] ? take(cnt * ss) : nullptr;
    d.loudness_specific = o->loudness_specific ? reinterpret_cast<float*>(take(cnt * nb * 4)) : nullptr;
    d.mfcc = o->mfcc ? reinterpret_cast<float*>(take(cnt * nc * 4)) : nullptr;
    d.amplitude_spectrum = o->amplitude_spectrum ? reinterpret_cast<float*>(take(cnt * L * 4)) : nullptr;
    d.power_spectrum = o->power_spectrum ? reinterpret_cast<float*>(take(cnt * L * 4)) : nullptr;
    d.complex_real = o->complex_real ? reinterpret_cast<float*>(take(cnt * n * 4)) : nullptr;
    d.complex_imag = o->complex_imag ? reinterpret_cast<float*>(take(cnt * n * 4)) : nullptr;
    // extraction of chunk i: after its frames arrived and chunk i-2's outputs left the slot
    e = hipStreamWaitEvent(p->s_comp, p->ev_loaded[sl], 0);
    if (e == hipSuccess && i >= 2) e = hipStreamWaitEvent(p->s_comp, p->ev_back[sl], 0);
    if (e != hipSuccess) break;
    rc = mgx_extract_device(p, p->s_frames[sl], cnt, &d, p->s_comp);
    if (rc) return fail_sync(rc);
    e = hipEventRecord(p->ev_done[sl], p->s_comp);
    // chunk i+1's frames into the other slot once chunk i-1's extraction has read them
    if (e == hipSuccess && i + 1 < nch) {
      const uint64_t g0 = (i + 1) * chunk, gc = std::min<uint64_t>(chunk, nframes - g0);
      if (i >= 1) e = hipStreamWaitEvent(p->s_copy, p->ev_done[sl ^ 1], 0);
      if (e != hipSuccess) break;
      rc = fill(g0, gc, sl ^ 1, p->s_copy);
      if (rc) return fail_sync(rc);
      e = hipEventRecord(p->ev_loaded[sl ^ 1], p->s_copy);
    }
    // chunk i's outputs back to the caller's arrays
    if (e == hipSuccess) e = hipStreamWaitEvent(p->s_copy, p->ev_done[sl], 0);
    auto back = [&](void* host, const void* dev, size_t bytes) {
      return host ? hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, p->s_copy) : hipSuccess;
    };
    for (int k = 0; k < MGX_NUM_SCALARS && e == hipSuccess; ++k)
      if (o->scalars[k]) e = back(static_cast<unsigned char*>(o->scalars[k]) + f0 * ss, d.scalars[k], cnt * ss);
    if (e == hipSuccess && o->loudness_specific) e = back(o->loudness_specific + f0 * nb, d.loudness_specific, cnt * nb * 4);
    if (e == hipSuccess && o->mfcc) e = back(o->mfcc + f0 * nc, d.mfcc, cnt * nc * 4);
    if (e == hipSuccess && o->amplitude_spectrum) e = back(o->amplitude_spectrum + f0 * L, d.amplitude_spectrum, cnt * L * 4);
    if (e == hipSuccess && o->power_spectrum) e = back(o->power_spectrum + f0 * L, d.power_spectrum, cnt * L * 4);
    if (e == hipSuccess && o->complex_real) e = back(o->complex_real + f0 * n, d.complex_real, cnt * n * 4);
    if (e == hipSuccess && o->complex_imag) e = back(o->complex_imag + f0 * n, d.complex_imag, cnt * n * 4);
    if (e == hipSuccess) e = hipEventRecord(p->ev_back[sl], p->s_copy);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(p->s_copy);
  if (e != hipSuccess) return fail_sync(hip_fail(e, "host batch copies"));
  return MGX_OK;
}

uint32_t sample_bytes(uint32_t format) {
  switch (format) {
    case MGX_PCM_F32: return 4;
    case MGX_PCM_S16: return 2;
    case MGX_PCM_U8: return 1;
    case MGX_PCM_S24: return 3;
    case MGX_PCM_S32: return 4;
    default: return 0;
  }
}

uint16_t rd16(const unsigned char* b) { return (uint16_t)(b[0] | (b[1] << 8)); }
uint32_t rd32(const unsigned char* b) { return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24); }

}  // namespace

extern "C" {

int mgx_extract_host(mgx_plan* p, const float* frames, uint64_t nframes, const mgx_outputs* o) {
  if (!p || !o) return fail(MGX_E_INVALID_ARGUMENT, "NULL plan or outputs");
  if (nframes == 0) return MGX_OK;
  if (!frames) return fail(MGX_E_INVALID_ARGUMENT, "frames is NULL");
  if ((o->complex_real == nullptr) != (o->complex_imag == nullptr))
    return fail(MGX_E_INVALID_ARGUMENT, "complex_real and complex_imag must be given together");
  const int n = p->n;
  if (nframes <= p->small_max)
    return extract_host_small(p, nframes, o, [&](float* dst) {
      memcpy(dst, frames, nframes * (size_t)n * sizeof(float));
      return MGX_OK;
    });
  return extract_host_chunked(p, nframes, o, [&](uint64_t f0, uint64_t cnt, int slot, hipStream_t st) {
    hipError_t e = hipMemcpyAsync(p->s_frames[slot], frames + f0 * n, cnt * n * sizeof(float), hipMemcpyHostToDevice, st);
    return e == hipSuccess ? MGX_OK : hip_fail(e, "hipMemcpyAsync(frames)");
  });
}

int mgx_wav_parse(const void* bytes, uint64_t len, mgx_wav_info* info) {
  if (!bytes || !info) return fail(MGX_E_INVALID_ARGUMENT, "NULL argument");
  if (info->struct_size != sizeof(mgx_wav_info))
    return fail(MGX_E_INVALID_ARGUMENT, "mgx_wav_info.struct_size is %u, expected %zu", info->struct_size, sizeof(mgx_wav_info));
  const unsigned char* b = static_cast<const unsigned char*>(bytes);
  if (len < 12 || memcmp(b, "RIFF", 4) != 0 || memcmp(b + 8, "WAVE", 4) != 0)
    return fail(MGX_E_INVALID_ARGUMENT, "not a RIFF/WAVE file");
  bool have_fmt = false;
  uint16_t tag = 0, channels = 0, bits = 0, align = 0;
  uint32_t rate = 0;
  uint64_t off = 12;
  while (off + 8 <= len) {
    const unsigned char* c = b + off;
    const uint64_t size = rd32(c + 4);
    if (memcmp(c, "fmt ", 4) == 0) {
      if (size < 16 || off + 8 + 16 > len) return fail(MGX_E_INVALID_ARGUMENT, "truncated fmt chunk");
      tag = rd16(c + 8);
      channels = rd16(c + 10);
      rate = rd32(c + 12);
      align = rd16(c + 20);
      bits = rd16(c + 22);
      if (tag == 0xFFFE) {  // WAVE_FORMAT_EXTENSIBLE: the subformat GUID starts with the real tag
        if (size < 40 || off + 8 + 26 > len) return fail(MGX_E_INVALID_ARGUMENT, "truncated WAVE_FORMAT_EXTENSIBLE fmt chunk");
        tag = rd16(c + 8 + 24);
      }
      have_fmt = true;
    } else if (memcmp(c, "data", 4) == 0) {
      if (!have_fmt) return fail(MGX_E_INVALID_ARGUMENT, "data chunk before fmt chunk");
      uint32_t fmt = 0xFFFFFFFFu;
      if (tag == 1 && bits == 8) fmt = MGX_PCM_U8;
      else if (tag == 1 && bits == 16) fmt = MGX_PCM_S16;
      else if (tag == 1 && bits == 24) fmt = MGX_PCM_S24;
      else if (tag == 1 && bits == 32) fmt = MGX_PCM_S32;
      else if (tag == 3 && bits == 32) fmt = MGX_PCM_F32;
      if (fmt == 0xFFFFFFFFu) return fail(MGX_E_UNSUPPORTED, "unsupported WAV encoding (format tag %u, %u bits)", tag, bits);
      if (channels == 0) return fail(MGX_E_INVALID_ARGUMENT, "WAV with 0 channels");
      if (align != channels * sample_bytes(fmt))
        return fail(MGX_E_INVALID_ARGUMENT, "block_align %u does not match %u channels x %u bytes", align, channels, sample_bytes(fmt));
      const uint64_t avail = len - (off + 8);
      const uint64_t data = std::min<uint64_t>(size, avail);
      info->pcm_format = fmt;
      info->channels = channels;
      info->sample_rate = rate;
      info->bits_per_sample = bits;
      info->block_align = align;
      info->data_offset = off + 8;
      info->data_bytes = data / align * align;
      info->sample_frames = data / align;
      return MGX_OK;
    }
    off += 8 + size + (size & 1);
  }
  return fail(MGX_E_INVALID_ARGUMENT, have_fmt ? "no data chunk" : "no fmt chunk");
}

int mgx_pcm_decode_device(const void* pcm, uint64_t sample_frames, uint32_t format, uint32_t channels,
                          uint32_t channel, float* out, void* stream) {
  if (sample_frames == 0) return MGX_OK;
  if (!pcm || !out) return fail(MGX_E_INVALID_ARGUMENT, "NULL pointer");
  if (!sample_bytes(format)) return fail(MGX_E_INVALID_ARGUMENT, "unknown PCM format %u", format);
  if (channels == 0 || channel >= channels) return fail(MGX_E_INVALID_ARGUMENT, "channel %u of %u", channel, channels);
  hipError_t e = mgx::launch_pcm_decode(pcm, sample_frames, format, channels, channel, out, (hipStream_t)stream);
  return e == hipSuccess ? MGX_OK : hip_fail(e, "PCM decode launch");
}

int mgx_extract_host_pcm(mgx_plan* p, const void* pcm, uint64_t pcm_bytes, uint64_t sample_frames, uint32_t format,
                         uint32_t channels, uint32_t channel, const mgx_outputs* o) {
  if (!p || !o) return fail(MGX_E_INVALID_ARGUMENT, "NULL plan or outputs");
  const uint32_t bps = sample_bytes(format);
  if (!bps) return fail(MGX_E_INVALID_ARGUMENT, "unknown PCM format %u", format);
  if (channels == 0 || channel >= channels) return fail(MGX_E_INVALID_ARGUMENT, "channel %u of %u", channel, channels);
  if ((o->complex_real == nullptr) != (o->complex_imag == nullptr))
    return fail(MGX_E_INVALID_ARGUMENT, "complex_real and complex_imag must be given together");
  const int n = p->n;
  const uint64_t nframes = sample_frames / (uint64_t)n;
  if (nframes == 0) return MGX_OK;
  if (!pcm) return fail(MGX_E_INVALID_ARGUMENT, "pcm is NULL");
  const uint64_t align = (uint64_t)bps * channels;
  if (sample_frames > pcm_bytes / align)
    return fail(MGX_E_INVALID_ARGUMENT, "%llu sample frames of %llu bytes exceed the %llu-byte PCM buffer",
                (unsigned long long)sample_frames, (unsigned long long)align, (unsigned long long)pcm_bytes);
  const uint64_t chunk_bytes = std::min<uint64_t>(nframes, kHostChunk) * n * align;
  if (p->s_pcm_bytes < chunk_bytes) {
    if (p->s_copy) (void)hipStreamSynchronize(p->s_copy);
    for (int i = 0; i < 2; ++i) {
      if (p->s_pcm[i]) (void)hipFree(p->s_pcm[i]);
      p->s_pcm[i] = nullptr;
    }
    p->s_pcm_bytes = 0;
    hipError_t e = hipSetDevice(p->d.device);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipMalloc(reinterpret_cast<void**>(&p->s_pcm[i]), chunk_bytes);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(staging PCM)");
    p->s_pcm_bytes = chunk_bytes;
  }
  const unsigned char* src = static_cast<const unsigned char*>(pcm);
  return extract_host_chunked(p, nframes, o, [&](uint64_t f0, uint64_t cnt, int slot, hipStream_t st) {
    const uint64_t bytes = cnt * n * align;
    hipError_t e = hipMemcpyAsync(p->s_pcm[slot], src + f0 * n * align, bytes, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(pcm)");
    e = mgx::launch_pcm_decode(p->s_pcm[slot], cnt * n, format, channels, channel, p->s_frames[slot], st);
    return e == hipSuccess ? MGX_OK : hip_fail(e, "PCM decode launch");
  });
}

int mgx_synth_frames_device(float* frames, uint64_t nframes, uint32_t n, uint64_t seed, uint64_t first_frame, void* stream) {
  if (!frames && nframes) return fail(MGX_E_INVALID_ARGUMENT, "frames is NULL");
  if (nframes == 0) return MGX_OK;
  hipError_t e = mgx::launch_synth(frames, nframes * (uint64_t)n, seed, first_frame * (uint64_t)n, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "synth kernel launch");
  return MGX_OK;
}

}  // extern "C"
