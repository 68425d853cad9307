// Fused per-frame feature extraction for gfx950 (MI355X).
//
// One persistent launch processes a batch of frames. Each of the 4 waves of a 256-thread
// workgroup loops over its own batches of FPW frames:
//
//  Phase 1 (one wave per frame, the next frame prefetched mid-frame):
//    load + rms/energy/zcr      src/extractors/rms.js, energy.js, zcr.js
//    window                     src/meyda.js:158-168
//    FFT                        lib/jsfft/fft.js:123-208, restated as a Hermitian
//                               half-spectrum radix-2 network: the
//                               frame is real, so each stage output block is kept as
//                               N/2 complex "slots"; every stage is rounded to
//                               float32 exactly where jsfft stores to Float32Array,
//                               with float64 butterflies.
//    amplitude                  src/meyda.js:104-114 -> the wave's LDS slot buffer
//    per-frame reductions       moments (src/utils.js:1-11), log sum
//                               (spectralFlatness.js), prefix sums (spectralRolloff.js,
//                               loudness band sums loudness.js:47-66), DPP wave sums
//    mel filterbank             mfcc.js:40-62 as a segmented scan over the bins (7 %
//                               dense: no dense contraction for the matrix cores, §4.3)
//  Phase 2 (the wave, over its FPW-frame batch):
//    specific loudness          loudness.js:55-63 (x^0.23, float32 store)
//    log mel + DCT              mfcc.js:64-93: the 13 x 26 DCT, the path's one dense
//                               contraction, on the FP64 matrix cores (v_mfma_f64_4x4x4_4b:
//                               16 coefficients x the batch's 4 frames per instruction);
//                               MGX_FLAG_DCT_SEQUENTIAL keeps the reference's sequential
//                               VALU order instead
//    scalar features            spectral*.js, perceptual*.js
//
// Compiled with -ffp-contract=off: every fused multiply-add below is explicit.
#include <cstring>
#include <type_traits>

#include "mgx_internal.h"

namespace mgx {
namespace {

typedef const __attribute__((address_space(1))) double2* GTw;
typedef const __attribute__((address_space(1))) float2* GTwf;
typedef const __attribute__((address_space(1))) double* GD;
typedef const __attribute__((address_space(1))) float* GF;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr double kS = 0.7071067811865476;  // Math.SQRT1_2 (lib/jsfft/fft.js:10)
constexpr float kSf = 0.70710677f;
constexpr double kLn2 = 0.6931471805599453;

// Tuning knobs (-DMGX_...) select among equivalent forms measured in DESIGN.md; every
// setting computes the same results. Timing ablations that drop work are not in this file:
// tools/ablate.py builds them from a patched copy.

constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v >> 1); }
constexpr int rev_bits(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r = (r << 1) | ((x >> i) & 1);
  return r;
}

// Padded slot address of an FFT exchange: loc + sum k (loc >> s), additive over the
// disjoint lane and register bits of a location, so phys(lane part) + phys(register part)
// (the register part an immediate offset). Chosen per N by a search over the LDS bank
// rule of ds_write2_b64 / ds_read2_b64 (4 groups of 16 lanes, banks (a/4) mod 32): the
// exchanges then take the conflict-free minimum of LDS cycles at N = 512, 1024 and 2048.
template <int N>
__host__ __device__ constexpr int phys(int loc) {
  return N == 256 ? loc + 2 * (loc >> 4) + (loc >> 6)
       : N == 512 ? loc + 4 * (loc >> 4) + (loc >> 6)
       : N == 1024 ? loc + 2 * (loc >> 4) + (loc >> 7)
       : loc + (loc >> 6);
}

template <int N>
struct Geo {
  static constexpr int L = N / 2;           // slots per frame == amplitude bins
  static constexpr int R = L / 64;          // slots per lane
  static constexpr int SB = ilog2c(L);      // slot-location bits
  static constexpr int RB = ilog2c(R);      // register bits
  static constexpr int NPASS = (SB + RB - 1) / RB;
  static constexpr int CH = N / 64;         // 64-sample input chunks per frame
  static constexpr int FPW = 4;             // frames per wave batch (phase 2 works on a wave batch)
  static constexpr int FB = 4 * FPW;        // frames per workgroup iteration
  // Register budget (VGPRs + AGPRs): 4 waves/SIMD (<= 128) up to N = 1024, where LDS
  // allows 4 workgroups per CU; 3 waves (<= 168) at N = 2048 (without the frame prefetch:
  // measured 3 % faster than 2 waves with it). Without the bound the allocator drifts past
  // the threshold (129 VGPRs, or 251 + 32 AGPRs) and occupancy drops.
  // N = 256 fits 6 waves (<= 80 VGPRs; measured 2.5 % faster than 5); at N = 512 a bound of
  // 5 waves measured slower than 4 until the LDS twiddles took the passes' global loads out
  // (81 VGPRs then, 3.9 % faster than 4 waves at 98).
  static constexpr int WPE = N <= 256 ? 6 : N <= 512 ? 5 : N <= 1024 ? 4 : 3;
  // Slot buffer entries (8 bytes): the padded exchange image, the natural-order half
  // spectrum X[0..L] (complex output), the padded prefix row (pd) and the mel scratch.
  static constexpr int cmax(int a, int b) { return a > b ? a : b; }
  // (at N = 512 also room for the moment transpose, MOM_SLOT: 41 entries more than the FFT
  // needs, against the 11.5 KB table it replaces; the workgroup keeps 5 per CU with the
  // LDS twiddles)
  static constexpr int SLOT_PHYS =
      cmax(cmax(cmax(phys<N>(L - 1) + 1, L + 1), cmax(L + 2 * (L >> 5) + 1, R * 64 + 2)), N == 512 ? 5 * 72 : 0);
  // Moment sums through an LDS transpose (5 rows of 64 doubles per wave, row stride 72 so
  // the rows read together fall in different banks) rather than 5 DPP wave sums: measured
  // faster at every N (at 2048 once it ran in the slot buffer: a table of its own cost 3 waves
  // their LDS).
  // (at 2048 through the slot buffer, MOM_SLOT: 1.5 % faster than DPP sums)
  static constexpr bool MOM_LDS = true;
  static constexpr int MOM_STRIDE = 72;
  // MOM_SLOT: the moment transpose runs in the wave's slot buffer right after the partials are
  // written (one more LDS round trip, no table of its own: 11.5 KB less LDS per workgroup)
  static constexpr bool MOM_SLOT = MOM_LDS && SLOT_PHYS >= 5 * MOM_STRIDE;
  // TW_LDS (N = 1024): the per-lane twiddles of passes >= 1 (the mixed-table entries and the
  // generic twiddles the tame passes read) are staged in LDS once per workgroup, in the space
  // the moment table left: LDS reads (lgkmcnt) instead of vector loads (vmcnt) in the passes
  static constexpr bool TW_LDS = (N == 1024 && MOM_SLOT) || N == 2048 || (N == 512 && MOM_SLOT);
  // Register prefetch of the next frame. A vector-memory wait is in issue order (vmcnt),
  // so a table load a frame waits on (window, twiddles) also waits for a prefetch issued
  // before it: prefetching at the start of the frame made every frame wait for the next
  // one's HBM read at its window step (at N = 1024 loading each frame only when its wave
  // starts it was 2.7 % faster).
  // PF = 1 loads the next frame at the start of this one; PF = 2 issues it in the middle of
  // this frame, after the last table loads this frame waits on (twiddles: the passes are
  // done; the mel records: issued just before), so no wait of this frame is held up by
  // it; PF = 0 loads each frame when its wave starts it (N = 2048: a mid-frame prefetch
  // measured -0.3 %, noise, and costs the tail pool, which needs PF = 0).
  static constexpr int PF = N <= 256 ? 1 : N <= 1024 ? 2 : 0;  // measured best per N
  // WIN_REG: the window held in registers for the whole launch (CH VGPRs) instead of loaded
  // per frame (N = 1024, where the LDS twiddles freed the registers: 1.1-1.5 % faster, 119
  // VGPRs; the frame prefetch at the frame's start instead, PF = 1, 0.9-1.1 %, and both
  // together 1.1 %)
  static constexpr bool WIN_REG = N == 1024;
  // BLIM_REG: each band lane's two prefix-row offsets (bark limits, loudness.js:25-45) held in
  // one packed register for the launch instead of read from LDS per frame (N <= 512: -0.5 %;
  // at 1024 the register spills two others, +1.3 %; at 2048 a value kept live across the
  // frame loop spills)
  static constexpr bool BLIM_REG = N <= 512;
  static constexpr bool PREFETCH = PF != 0;
  // GROUP_SYNC: a workgroup barrier after every GROUP_SYNC-th full group of 16 frames, so the
  // group's output lines are written together (extract_kernel; 0 = none). Measured per N
  // (profiles/r03_group_sync.txt): 1024 +0.0 % (time-only -3.8 %), 256 -0.1 %; the all-feature
  // launch at 512 +1.6 % and at 2048 (3 waves per SIMD) +2.3 %, so those keep none.
  static constexpr int GROUP_SYNC = (N == 1024 || N == 256) ? 2 : 0;
  static constexpr bool LPREMAT = N == 2048;  // measured: N = 2048 1 % faster, N = 256 7 % slower
  static constexpr int MIX = 1;  // bfly_mixed_tame (form 0 was faster at N = 1024 at 128 live VGPRs)
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


// LDS image of the tame passes' per-lane twiddles (Geo<N>::TW_LDS), in double2 entries. In
// pass P >= 1 the location bits below the pass's first stage bit q0 that are lane bits are the
// lowest nl = min(q0, 6) (the lanes take the lowest free bits), and every bit in [nl, q) below
// stage q is a register bit (the stage bits [q0, q), at N = 2048 also the leftover register
// bits [6, 8) of the last pass). So the mixed pairs of stage q read mixed-table entries
// mask + la, la < 2^nl (two double2 each: (b, c0), (t4, kL)), and the generic ones
// mask + (la | rp), rp != 0: the contiguous [mask + 2^nl, mask + 2^q). Per (P, I): the mixed
// block, then the generic one. At N = 2048 only pass 1 is staged (pass_lds: 4.9 KB; with the
// last pass's mixed entries too, 9 KB, the workgroup no longer fit 3 per CU and the launch ran
// 20 % slower); the last pass reads its twiddles from global memory as before.
template <int N>
struct TwLds {
  using PG = PassGeo<N>;
  static constexpr int nl(int P) { return PG::q0(P) < 6 ? PG::q0(P) : 6; }
  static constexpr bool pass_lds(int P) { return !(N == 2048 && P == 2); }
  static constexpr int mixed_n(int P) { return pass_lds(P) ? 2 << nl(P) : 0; }
  static constexpr int gen_n(int P, int I) { return pass_lds(P) ? (1 << (PG::q0(P) + I)) - (1 << nl(P)) : 0; }
  static constexpr int off(int P, int I, bool gen) {
    int o = 0;
    for (int p = 1; p < Geo<N>::NPASS; ++p)
      for (int i = 0; i < PG::m(p); ++i) {
        if (p == P && i == I) return gen ? o + mixed_n(p) : o;
        o += mixed_n(p) + gen_n(p, i);
      }
    return o;
  }
  // after the per-stage blocks: the lane-uniform (f_x, S f_y) of each tame stage's block-start
  // pair (the mixed table's entry N/2 - 1 + q), one double2 per stage q = q0(P) + I
  static constexpr int fw_off(int P, int I) {
    int o = off(Geo<N>::NPASS, 0, false);
    for (int p = 1; p < Geo<N>::NPASS; ++p)
      for (int i = 0; i < PG::m(p); ++i) {
        if (p == P && i == I) return o;
        if (pass_lds(p)) ++o;
      }
    return o;
  }
  static constexpr int total() { return fw_off(Geo<N>::NPASS, 0); }
};

// The fast precision's LDS image (MGX_PRECISION_FAST, in the same LDS region): the float32
// twiddles of the staged passes' stages are one contiguous range of the plan's twf table
// (stage q at offset 2^q - 1, entries la | rp of both the mixed and the generic pairs).
template <int N>
struct TwLdsF {
  using PG = PassGeo<N>;
  static constexpr int first = (1 << PG::q0(1)) - 1;
  static constexpr int qend() {
    int q = PG::q0(1);
    for (int p = 1; p < Geo<N>::NPASS; ++p)
      if (TwLds<N>::pass_lds(p)) q = PG::q0(p) + PG::m(p);
    return q;
  }
  static constexpr int count = (1 << qend()) - 1 - first;
  static_assert(count * 8 <= TwLds<N>::total() * 16, "the float32 image fits the float64 one's LDS");
};

// Bank-padded layouts of the amplitude row (floats) and of its prefix sums (doubles) in
// the slot buffer: lane l reads the row (ds_read2_b64) and writes the prefix
// (ds_write2_b64) as R consecutive entries; both instructions serve 16 consecutive lanes
// per LDS cycle with banks (a/4) mod 32 (MI355X_MICROARCH.md §LDS). The prefix row's 1
// double of padding per 16 gives those 16 lanes 16 distinct bank pairs at every R (the
// former 2 per 32 left 2-way conflicts: 32 extra LDS cycles per frame at N = 1024,
// SQ_LDS_BANK_CONFLICT). The amplitude row keeps 4 floats per 64 (2-way on its reads): 2
// per 32 removes those too but changed the surrounding code generation and measured
// 2.5 % slower; the LDS is not what bounds the kernel.
__device__ __forceinline__ int pa(int k) { return k + 4 * (k >> 6); }
__device__ __forceinline__ int pa_inv(int k) { return k - 4 * (k / 68); }  // pa(b) = 68 (b >> 6) + (b & 63)
__device__ __forceinline__ int pd(int d) { return d + (d >> 4); }


// Wave priority (s_setprio) in the frame's low-ILP sections: a wave in an LDS round trip or a
// serial chain (DPP reductions, the amplitude's conversions, phase 2's scalar steps) issues
// ahead of the other waves, whose FFT passes have independent butterflies to fill the gaps,
// so its latency overlaps their arithmetic instead of adding to it. kPrioSet selects the
// regions: 1 the FFT exchanges, 2 the amplitude row's LDS round trip, 4 phase 2, 8 the
// per-frame reductions (moment transpose, prefix and rolloff, band sums, mel scan), 16 the
// frame start (energy/zcr, window, stage 0), 32 the amplitude, 64 the moment partials.
// Measured (interleaved A/B, all features; profiles/design_history_r01_r04.md): 1 alone 0.5-1 % faster than none;
// 111 (all but the frame start, level 2) another 5.0 % at N = 1024, 4.3 % at 2048, 7.4 % at 512;
// then levels: the exchanges and phase 2 at 3, the frame start at 1 (above the FFT's register
// passes at 0), 127: another 1.4 % at 1024, 2.5 % at 2048, 2.1 % at 512.
constexpr int kPrioSet = 127;  // every region: 1 | 2 | 4 | 8 | 16 | 32 | 64
constexpr int prio_level(int region) {
  return region == 4 ? 3 : region == 1 ? 3 : region == 16 ? 1 : 2;  // phase 2 and exchanges 3, frame start 1
}
template <int REGION>
__device__ __forceinline__ void prio_hi() {
  if constexpr ((kPrioSet & REGION) != 0) __builtin_amdgcn_s_setprio(prio_level(REGION));
}
template <int REGION>
__device__ __forceinline__ void prio_lo() {
  if constexpr ((kPrioSet & REGION) != 0) __builtin_amdgcn_s_setprio(0);
}

// pa(spectrum bin) of each register after the last pass, live across the whole frame loop:
// two 16-bit entries per VGPR (packed measured 1 % faster than one int per register at
// N = 512, 0.2 % at 1024).
template <int N>
struct KlTab {
  static constexpr int R = N / 128;
  uint32_t w[R / 2];
  __device__ __forceinline__ void set(int r, int v) {
    if (r & 1) w[r >> 1] |= (uint32_t)v << 16;
    else w[r >> 1] = (uint32_t)v;
  }
  __device__ __forceinline__ int operator()(int r) const { return (int)((w[r >> 1] >> (16 * (r & 1))) & 0xFFFFu); }
};

// A frame's samples: read once and never again. A batch larger than the 256 MiB MALL cannot stay
// resident across launches, and its frames are read with non-temporal loads (KernelArgs::nt_frames,
// plan.cpp), which keep the L2 for the lines that are read back -- the scalar windows, the CHAIN
// kernels' power-row ring (always nt: -0.6..-1.2 % per reference-order launch, profiles/r03_mfcc_tracks.txt).
// The HBM-bound time-only features ran 12 % faster with them on a 1 GiB batch (5.9 TB/s) and the
// all-feature launch 1.2 % (profiles/r05_prologue_ab.txt); a smaller batch keeps plain loads, because
// then it stays in the MALL between launches of the same frames (C2's 128 MiB: 12 % slower with nt).
// A spectrum output element (amplitude, power, complex: 2-8 KB per frame, written once and never
// read back): a non-temporal store, which streams past the caches instead of filling them (every
// output at N = 1024: -8.1..-8.8 % per launch; C2's 1 GiB batch -0.7 %, outputs identical; the same
// for the scalar, loudness and MFCC outputs, tens of bytes per frame, measured no gain).
template <class P>
__device__ __forceinline__ void st_out(P p, float v) {
  __builtin_nontemporal_store(v, p);
}

// (the lane's CH samples of the frame at p; nt: the launch's run-time choice, NT: always. The empty asm
// statements keep the two branches apart: without them the compiler hoists or sinks the loads of both
// into one plain load, the non-temporal hint dropped as metadata the two did not share.)
template <bool NT, int CH>
__device__ __forceinline__ void ld_frame(float (&xv)[CH], GF p, unsigned lane, bool nt) {
  if (NT || nt) {
    if constexpr (!NT) asm volatile("; nt frame");
#pragma unroll
    for (int c = 0; c < CH; ++c) xv[c] = __builtin_nontemporal_load(p + (c * 64 + lane));
    if constexpr (!NT) asm volatile("; nt frame issued");
  } else {
#pragma unroll
    for (int c = 0; c < CH; ++c) xv[c] = p[c * 64 + lane];
  }
}

// Static instruction accounting (tools/isa_phases.py): -DMGX_MARKS puts an assembly comment
// at each phase boundary; the default build has none.
#ifdef MGX_MARKS
#define MGX_MARK(tag) asm volatile(";mgxmark " #tag)
#else
#define MGX_MARK(tag) ((void)0)
#endif

// Phase stamps of the diagnostic build (-DMGX_WAVE_TIMES=1 only; tools/small_stamps.py): the 100 MHz
// real-time clock at MGX_STAMP(i), written by the first lane of a one-workgroup launch (a small host
// batch; in a large launch the stamps would slow its first wave at every frame).
#if MGX_WAVE_TIMES
__device__ unsigned long long g_stamps[16];
#define MGX_STAMP(i)                                                                              \
  do {                                                                                            \
    if (gridDim.x == 1 && threadIdx.x == 0) ((volatile unsigned long long*)g_stamps)[i] = wall_clock64(); \
  } while (0)
#else
#define MGX_STAMP(i) ((void)0)
#endif
// (and the shader clock beside it, g_stamps[i] = clock64(): the core clock the one-frame launch ran at)
#if MGX_WAVE_TIMES
#define MGX_CLOCK_STAMP(i)                                                                        \
  do {                                                                                            \
    if (gridDim.x == 1 && threadIdx.x == 0) ((volatile unsigned long long*)g_stamps)[i] = clock64(); \
  } while (0)
#else
#define MGX_CLOCK_STAMP(i) ((void)0)
#endif

// Wave-level LDS ordering (no global-memory fence: in-flight prefetch loads stay in flight).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// Workgroup barrier ordering LDS only. __syncthreads() also fences global memory, which
// makes every wave drain its outstanding loads (the next frame's prefetch) at each barrier.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ double2 ld_tw_u(GTw p, int i);
__device__ __forceinline__ double2 ld_tw(GTw p, int i) {
  const GD q = (GD)p;
  return make_double2(q[2 * i], q[2 * i + 1]);
}
// A twiddle whose index is the same on every lane (pass 0, and every block-start pair):
// read through the constant address space, so it is an s_load into SGPRs (scalar cache)
// instead of a vector load through the texture path, and costs no VGPRs.
typedef const __attribute__((address_space(4))) double* CD;
typedef const __attribute__((address_space(4))) float* CF;
__device__ __forceinline__ double2 ld_tw_u(GTw p, int i) {
  const CD q = (CD)(uintptr_t)p;
  return make_double2(q[2 * i], q[2 * i + 1]);
}
__device__ __forceinline__ float2 ld_twf_u(GTwf p, int i) {
  const CF q = (CF)(uintptr_t)p;
  return make_float2(q[2 * i], q[2 * i + 1]);
}
__device__ __forceinline__ float2 ld_twf(GTwf p, int i) {
  const GF q = (GF)p;
  return make_float2(q[2 * i], q[2 * i + 1]);
}

// ---------------------------------------------------------------- butterflies
// Twiddle table of stage q (input blocks of 2^(q+1) samples) at offset 2^q - 1:
// entry a holds c = SQRT1_2 * f_k(a) for the slot pair (a, a + 2^q) (entry 0: S f_0 =
// (S, 0)); after the N/2 - 1 stage entries, entry N/2 - 1 + q holds S f_{w/2}
// for the block-start pair, whose slots pack (X[0], X[w/2]).
//
// Generic pair:      lo <- s L + c R,   hi <- conj(s L - c R)
// Block-start pair:  exactly jsfft's operations for j = 0 and j = w/2.
template <bool FAITH, bool UNI = false>
__device__ __forceinline__ void bfly_generic(float2& lo, float2& hi, GTw tw, GTwf twf, int idx) {
  if constexpr (FAITH) {
    const double2 c = UNI ? ld_tw_u(tw, idx) : ld_tw(tw, idx);
    const double Lr = lo.x, Li = lo.y, Rr = hi.x, Ri = hi.y;
    const double Ar = __builtin_fma(c.x, Rr, -(c.y * Ri));
    const double Ai = __builtin_fma(c.x, Ri, c.y * Rr);
    lo.x = (float)__builtin_fma(kS, Lr, Ar);
    lo.y = (float)__builtin_fma(kS, Li, Ai);
    hi.x = (float)__builtin_fma(kS, Lr, -Ar);
    hi.y = (float)__builtin_fma(-kS, Li, Ai);
  } else {
    const float2 c = UNI ? ld_twf_u(twf, idx) : ld_twf(twf, idx);
    const float Ar = __builtin_fmaf(c.x, hi.x, -(c.y * hi.y));
    const float Ai = __builtin_fmaf(c.x, hi.y, c.y * hi.x);
    const float Lr = lo.x, Li = lo.y;
    lo.x = __builtin_fmaf(kSf, Lr, Ar);
    lo.y = __builtin_fmaf(kSf, Li, Ai);
    hi.x = __builtin_fmaf(kSf, Lr, -Ar);
    hi.y = __builtin_fmaf(-kSf, Li, Ai);
  }
}

// The fast precision's generic and mixed pairs with the per-lane twiddle from LDS (TwLdsF).
__device__ __forceinline__ void bfly_generic_f(float2& lo, float2& hi, float2 c) {
  const float Ar = __builtin_fmaf(c.x, hi.x, -(c.y * hi.y));
  const float Ai = __builtin_fmaf(c.x, hi.y, c.y * hi.x);
  const float Lr = lo.x, Li = lo.y;
  lo.x = __builtin_fmaf(kSf, Lr, Ar);
  lo.y = __builtin_fmaf(kSf, Li, Ai);
  hi.x = __builtin_fmaf(kSf, Lr, -Ar);
  hi.y = __builtin_fmaf(-kSf, Li, Ai);
}
__device__ __forceinline__ void bfly_mixed_f(float2& lo, float2& hi, float2 c, float2 f, bool sp) {
  const float Lr = lo.x, Li = lo.y, Rr = hi.x, Ri = hi.y;
  const float Ar = __builtin_fmaf(c.x, Rr, -(c.y * Ri));
  const float Ai = __builtin_fmaf(c.x, Ri, c.y * Rr);
  const float g0 = __builtin_fmaf(kSf, Lr, Ar), g1 = __builtin_fmaf(kSf, Li, Ai);
  const float g2 = __builtin_fmaf(kSf, Lr, -Ar), g3 = __builtin_fmaf(-kSf, Li, Ai);
  const float s0 = kSf * (Lr + Rr), s1 = kSf * (Lr - Rr);
  const float s2 = __builtin_fmaf(kSf, Li, f.x * Ri), s3 = f.y * Ri;
  lo.x = sp ? s0 : g0;
  lo.y = sp ? s1 : g1;
  hi.x = sp ? s2 : g2;
  hi.y = sp ? s3 : g3;
}

// The faithful generic pair with its twiddle already in registers (TwLds).
__device__ __forceinline__ void bfly_generic_c(float2& lo, float2& hi, double2 c) {
  const double Lr = lo.x, Li = lo.y, Rr = hi.x, Ri = hi.y;
  const double Ar = __builtin_fma(c.x, Rr, -(c.y * Ri));
  const double Ai = __builtin_fma(c.x, Ri, c.y * Rr);
  lo.x = (float)__builtin_fma(kS, Lr, Ar);
  lo.y = (float)__builtin_fma(kS, Li, Ai);
  hi.x = (float)__builtin_fma(kS, Lr, -Ar);
  hi.y = (float)__builtin_fma(-kS, Li, Ai);
}

template <bool FAITH>
__device__ __forceinline__ void bfly_special(float2& lo, float2& hi, GTw tw, GTwf twf, int idx) {
  // f = SQRT1_2 f_{w/2}: S (Lh + f_x Rh) as S Lh + (S f_x) Rh and S (f_y Rh) as (S f_y) Rh
  // (one f64 rounding moved in each; the exact j = 0 sums S (L0 +- R0) stay as written)
  if constexpr (FAITH) {
    const double2 f = ld_tw_u(tw, idx);
    const double L0 = lo.x, Lh = lo.y, R0 = hi.x, Rh = hi.y;
    lo.x = (float)(kS * (L0 + R0));
    lo.y = (float)(kS * (L0 - R0));
    hi.x = (float)__builtin_fma(kS, Lh, f.x * Rh);
    hi.y = (float)(f.y * Rh);
  } else {
    const float2 f = ld_twf_u(twf, idx);
    const float L0 = lo.x, Lh = lo.y, R0 = hi.x, Rh = hi.y;
    lo.x = kSf * (L0 + R0);
    lo.y = kSf * (L0 - R0);
    hi.x = __builtin_fmaf(kSf, Lh, f.x * Rh);
    hi.y = f.y * Rh;
  }
}

// A pair that is block-start on some lanes (sp) and generic on the others: both forms
// are evaluated and selected, so the wave never diverges. The block-start form keeps
// jsfft's exact operations (S (L + R), not S L + S R): exact cancellations to 0 (DC /
// Nyquist of symmetric blocks) must stay 0 for spectralFlatness.
template <bool FAITH>
__device__ __forceinline__ void bfly_mixed(float2& lo, float2& hi, GTw tw, GTwf twf, int idx, int fidx, bool sp) {
  if constexpr (FAITH) {
    const double2 c = ld_tw(tw, idx);
    const double2 f = ld_tw_u(tw, fidx);
    const double Lr = lo.x, Li = lo.y, Rr = hi.x, Ri = hi.y;
    const double Ar = __builtin_fma(c.x, Rr, -(c.y * Ri));
    const double Ai = __builtin_fma(c.x, Ri, c.y * Rr);
    const double g0 = __builtin_fma(kS, Lr, Ar), g1 = __builtin_fma(kS, Li, Ai);
    const double g2 = __builtin_fma(kS, Lr, -Ar), g3 = __builtin_fma(-kS, Li, Ai);
    const double s0 = kS * (Lr + Rr), s1 = kS * (Lr - Rr);
    const double s2 = __builtin_fma(kS, Li, f.x * Ri), s3 = f.y * Ri;  // f = S f_{w/2}
    lo.x = (float)(sp ? s0 : g0);
    lo.y = (float)(sp ? s1 : g1);
    hi.x = (float)(sp ? s2 : g2);
    hi.y = (float)(sp ? s3 : g3);
  } else {
    const float2 c = ld_twf(twf, idx);
    const float2 f = ld_twf_u(twf, fidx);
    const float Lr = lo.x, Li = lo.y, Rr = hi.x, Ri = hi.y;
    const float Ar = __builtin_fmaf(c.x, Rr, -(c.y * Ri));
    const float Ai = __builtin_fmaf(c.x, Ri, c.y * Rr);
    const float g0 = __builtin_fmaf(kSf, Lr, Ar), g1 = __builtin_fmaf(kSf, Li, Ai);
    const float g2 = __builtin_fmaf(kSf, Lr, -Ar), g3 = __builtin_fmaf(-kSf, Li, Ai);
    const float s0 = kSf * (Lr + Rr), s1 = kSf * (Lr - Rr);
    const float s2 = __builtin_fmaf(kSf, Li, f.x * Ri), s3 = f.y * Ri;
    lo.x = sp ? s0 : g0;
    lo.y = sp ? s1 : g1;
    hi.x = sp ? s2 : g2;
    hi.y = sp ? s3 : g3;
  }
}

// The mixed pair of a frame whose samples are all finite and below 2^50 in magnitude
// (no infinity can arise in the FFT). One form serves both lane kinds, with per-lane
// coefficients (b, c0, t4, kL) from the plan's mixed table (entry a = la | rp of the stage,
// two double2 per entry):
//   generic lanes (b = f_x, c0 = S f_y, t4 = S f_x, kL = -S):
//     lo = (S fma(f_x, Rr, Lr) - c0 Ri, S fma(f_x, Ri, Li) + c0 Rr),
//     hi = (S fma(-f_x, Rr, Lr) + c0 Ri, t4 Ri + (kL Li + c0 Rr));
//   block-start lanes (b = 1, c0 = 0, t4 = S f_y(w/2), kL = 0): t1 = L0 + R0 and
//     t3 = L0 - R0 exactly as jsfft, lo = (S t1, S t3), hi = (S (Lh + f_x Rh), S f_y Rh)
//     with f = f_{w/2} (fwx: lane-uniform f_x): the two middle outputs swap places.
// 10 f64 operations and 4 selects (2 of them per stage, shared by the stage's pairs);
// the c0 and kL products are 0 x finite on block-start lanes, which is why L, R must be finite.
__device__ __forceinline__ void bfly_mixed_tame(float2& lo, float2& hi, double2 m, double2 k, double fwx, bool sp) {
  const double b2 = sp ? fwx : m.x;
  const double Lr = lo.x, Li = lo.y, Rr = hi.x, Ri = hi.y;
  const double ui = m.y * Ri, ur = m.y * Rr;
  const float o1 = (float)__builtin_fma(kS, __builtin_fma(m.x, Rr, Lr), -ui);
  const float o3 = (float)__builtin_fma(kS, __builtin_fma(-m.x, Rr, Lr), ui);
  const float o2 = (float)__builtin_fma(kS, __builtin_fma(b2, Ri, Li), ur);
  const float o4 = (float)__builtin_fma(k.x, Ri, __builtin_fma(k.y, Li, ur));
  lo.x = o1;
  lo.y = sp ? o3 : o2;
  hi.x = sp ? o2 : o3;
  hi.y = o4;
}
// The same pair with the last output selected per lane (S f_y(w/2) Ri on block-start
// lanes): 11 f64 operations and 6 selects, no (t4, kL) — cheaper for a stage's only pair.
[[maybe_unused]] __device__ __forceinline__ void bfly_mixed_tame1(float2& lo, float2& hi, double2 m, double2 fw, bool sp) {
  const double b2 = sp ? fw.x : m.x;
  const double Lr = lo.x, Li = lo.y, Rr = hi.x, Ri = hi.y;
  const double ui = m.y * Ri, ur = m.y * Rr;
  const float o1 = (float)__builtin_fma(kS, __builtin_fma(m.x, Rr, Lr), -ui);
  const float o3 = (float)__builtin_fma(kS, __builtin_fma(-m.x, Rr, Lr), ui);
  const float o2 = (float)__builtin_fma(kS, __builtin_fma(b2, Ri, Li), ur);
  const double o4 = sp ? fw.y * Ri : __builtin_fma(-kS, __builtin_fma(-b2, Ri, Li), ur);
  lo.x = o1;
  lo.y = sp ? o3 : o2;
  hi.x = sp ? o2 : o3;
  hi.y = (float)o4;
}

// How the tame mixed pairs of a stage get (t4, kL) (Geo<N>::MIX): 0 = per pair
// (bfly_mixed_tame1), 1 = from the plan table, 2 = computed once per stage (t4 = S b,
// kL = -S; block start: S f_y(w/2), 0). Measured (all features): the table form is 1 % faster
// at N = 512, 3 % at N = 2048 and 1.9 % at N = 1024 (there only once the moment and
// amplitude changes had freed registers; before, 1.8 % slower).

// One radix-2 stage on location bit q = q0(P) + I, entirely in registers.
template <int N, int P, int I, bool FAITH, bool TAME, bool TWL>
__device__ __forceinline__ void run_stage(float2 (&v)[Geo<N>::R], int lp, GTw tw, GTwf twf, GTw twm,
                                          const double2* twl) {
  constexpr bool LT = FAITH && TAME && TWL && P > 0 && TwLds<N>::pass_lds(P);  // twiddles from the LDS image
  constexpr bool LTF = !FAITH && TWL && P > 0 && TwLds<N>::pass_lds(P);        // the fast precision's (TwLdsF)
  const float2* twlf = reinterpret_cast<const float2*>(twl);
  using G = Geo<N>;
  using PG = PassGeo<N>;
  constexpr int q = PG::q0(P) + I;
  constexpr int mask = (1 << q) - 1;
  constexpr int fidx = G::L - 1 + q;  // f_{w/2} of this stage
  const int la = lp & mask;  // 0 in pass 0
#pragma unroll
  for (int r = 0; r < G::R; ++r) {
    if (r & (1 << I)) continue;
    const int rp = PG::rpart(P, r) & mask;
    const int hi = r | (1 << I);
    if constexpr (P == 0) {
      if (rp == 0) bfly_special<FAITH>(v[r], v[hi], tw, twf, fidx);
      else bfly_generic<FAITH, true>(v[r], v[hi], tw, twf, mask + rp);
    } else if (rp == 0) {
      if constexpr (FAITH && TAME) {
        // every mixed pair of the stage has rp == 0: one coefficient entry per lane and stage
        constexpr int npairs = G::R >> (I + 1);
        const bool sp = la == 0;
        const double2 fw = LT ? twl[TwLds<N>::fw_off(P, I)] : ld_tw_u(twm, 2 * fidx);
        const double2 m = LT ? twl[TwLds<N>::off(P, I, false) + 2 * la] : ld_tw(twm, 2 * (mask + la));
        if constexpr (G::MIX == 0 || (G::MIX == 2 && npairs == 1)) {
          bfly_mixed_tame1(v[r], v[hi], m, fw, sp);
        } else if constexpr (G::MIX == 1) {
          bfly_mixed_tame(v[r], v[hi], m, LT ? twl[TwLds<N>::off(P, I, false) + 2 * la + 1] : ld_tw(twm, 2 * (mask + la) + 1),
                          fw.x, sp);
        } else {
          const double2 k = make_double2(sp ? fw.y : kS * m.x, sp ? 0.0 : -kS);
          bfly_mixed_tame(v[r], v[hi], m, k, fw.x, sp);
        }
      }
      else if constexpr (LTF) bfly_mixed_f(v[r], v[hi], twlf[mask - TwLdsF<N>::first + la], ld_twf_u(twf, fidx), la == 0);
      else bfly_mixed<FAITH>(v[r], v[hi], tw, twf, mask + la, fidx, la == 0);
    } else if constexpr (LT) {
      bfly_generic_c(v[r], v[hi], twl[TwLds<N>::off(P, I, true) + ((la | rp) - (1 << TwLds<N>::nl(P)))]);
    } else if constexpr (LTF) {
      bfly_generic_f(v[r], v[hi], twlf[mask - TwLdsF<N>::first + (la | rp)]);
    } else {
      bfly_generic<FAITH>(v[r], v[hi], tw, twf, mask + (la | rp));
    }
  }
}

template <int N, int P, int I, bool FAITH, bool TAME, bool TWL>
__device__ __forceinline__ void run_stages(float2 (&v)[Geo<N>::R], int lp, GTw tw, GTwf twf, GTw twm,
                                           const double2* twl) {
  if constexpr (I < PassGeo<N>::m(P)) {
    run_stage<N, P, I, FAITH, TAME, TWL>(v, lp, tw, twf, twm, twl);
    run_stages<N, P, I + 1, FAITH, TAME, TWL>(v, lp, tw, twf, twm, twl);
  }
}

// Move the slots from pass P-1's lane/register layout to pass P's through LDS.
template <int N, int P>
__device__ __forceinline__ void exchange(float2 (&v)[Geo<N>::R], int lp_prev, int lp_cur, float2* buf) {
  using G = Geo<N>;
  using PG = PassGeo<N>;
  const int bprev = phys<N>(lp_prev), bcur = phys<N>(lp_cur);
  MGX_MARK(xchg_begin);
  prio_hi<1>();
  wave_sync();
#pragma unroll
  for (int r = 0; r < G::R; ++r) buf[bprev + phys<N>(PG::rpart(P - 1, r))] = v[r];
  wave_sync();
#pragma unroll
  for (int r = 0; r < G::R; ++r) v[r] = buf[bcur + phys<N>(PG::rpart(P, r))];
  prio_lo<1>();
  MGX_MARK(xchg_end);
}

template <int N, int P, bool FAITH, bool TAME, bool TWL>
__device__ __forceinline__ void run_passes(float2 (&v)[Geo<N>::R], const int (&lp)[Geo<N>::NPASS],
                                           float2* buf, GTw tw, GTwf twf, GTw twm, const double2* twl) {
  if constexpr (P < Geo<N>::NPASS) {
    if constexpr (P > 0) exchange<N, P>(v, lp[P - 1], lp[P], buf);
    run_stages<N, P, 0, FAITH, TAME, TWL>(v, lp[P], tw, twf, twm, twl);
    run_passes<N, P + 1, FAITH, TAME, TWL>(v, lp, buf, tw, twf, twm, twl);
  }
}

// ------------------------------------------------------- DPP wave reductions
// Cross-lane moves on the VALU (no LDS round trips): quad_perm / row mirrors /
// row shifts / row broadcasts of gfx9 DPP, applied to both halves of a double.
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROW_MASK, BANK_MASK, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, ROW_MASK, BANK_MASK, true);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Sum over the 64 lanes; the result is wave-uniform.
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror: every lane holds its row's sum
  v += dpp_d<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3 hold rows 0+1, 2+3
  v += dpp_d<0x143, 0xC>(v);  // row_bcast:31 -> row 3 holds the total
  return readlane_d(v, 63);
}

// Inclusive prefix sum over the lanes.
__device__ __forceinline__ double wave_inclusive_scan(double v) {
  v += dpp_d<0x111>(v);            // row_shr:1
  v += dpp_d<0x112>(v);            // row_shr:2
  v += dpp_d<0x114>(v);            // row_shr:4
  v += dpp_d<0x118>(v);            // row_shr:8
  v += dpp_d<0x142, 0xA>(v);       // row_bcast:15 -> rows 1, 3
  v += dpp_d<0x143, 0xC>(v);       // row_bcast:31 -> rows 2, 3
  return v;
}


// Amplitude of one slot: src/meyda.js:104-114, sqrt(re^2 + im^2) in double, stored to float32.
template <bool FAITH>
__device__ __forceinline__ float slot_amp(float re, float im) {
  if constexpr (FAITH) {
    // s = re^2 + im^2 lies in [2^-298, 2^256) or is 0/inf/NaN, so the library sqrt's
    // range scaling is not needed: rsq seed + the two-residual refinement (full double
    // accuracy), then 0/inf/NaN pass through.
    const double xr = re, xi = im;
    const double s = __builtin_fma(xr, xr, xi * xi);
    const double y = __builtin_amdgcn_rsq(s);
    double g = s * y, h = 0.5 * y;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, s);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, s);
    g = __builtin_fma(d, h, g);
    return (float)((s > 0.0 && s < __builtin_huge_val()) ? g : s);
  } else {
    return sqrtf(__builtin_fmaf(re, re, im * im));
  }
}

// The same amplitude through the f32 hardware reciprocal square root plus one f64 Heron
// correction (about half the issue cycles: v_rsq_f64 alone costs 16 cycles per wave, the
// f64 Newton chain 9 more f64 operations). s = re^2 + im^2 exactly as above; q = rsq(s) in
// f32, y = s q (~2^-22 relative), r = s - y^2 exactly in f64, then g = y + r q / 2 as one
// float32 FMA of (float)r (~2^-43 relative before its single rounding): equal to the
// correctly rounded sqrt unless sqrt(s) lies within 2^-43 of a float32 rounding boundary
// (~2^-19 of the bins; those move by one ulp). ok is false when s leaves [2^-80, 2^120]
// (0, tiny -- where r would be a float32 denormal --, huge, inf, NaN): the caller then
// redoes the wave's frame with slot_amp.
__device__ __forceinline__ float slot_amp_rsq(float re, float im, bool& ok) {
  const double xr = re, xi = im;
  const double s = __builtin_fma(xr, xr, xi * xi);
  const float sf = (float)s;
  const float q = __builtin_amdgcn_rsqf(sf);
  const float yf = sf * q;
  const double y = yf;
  const float r = (float)__builtin_fma(-y, y, s);
  const float a = __builtin_fmaf(r, 0.5f * q, yf);
  // s in [2^-80, 2^120] <=> a in [2^-40, 2^60] (outside, the rsq seed is a denormal, 0,
  // inf or NaN and so is a, or a is out of range): float32 compares instead of f64 ones
  ok = a >= 0x1p-40f && a <= 0x1p60f;
  return a;
}

struct FrameRec {
  double S[5];      // sum_k k^p a_k, p = 0..4 (S[0] = sum a_k)
  double ln2sum;    // sum_k log2 a_k (must follow S[4]: written as (&S[1])[4])
  double energy;    // sum x^2
  double band[kBark];
  float lm[kMaxMel];  // mel band energies, then their logs (zero-padded to a multiple of 8)
  int zcr;
  int roll_m;
  // 520 bytes: phase 2 reads across frames hit distinct LDS banks (512 would not). Phase 2's
  // loudness step leaves the frame's loudness max (float bits) and sharpness sum here, and
  // the total in band[0] (the band sums are read by then), for the scalar step.
  uint32_t loud_max;
  float sharp_sum;
};

// A frame's inputs to the thirteen scalar formulas (scalar_value), as phase 2 leaves them in its
// record: the first eight words and the last two of a FrameRec, copied word for word into the
// wave's scalar window (scalar_pass).
struct ScalIn {
  double S[5];
  double ln2sum;
  double energy;
  double band[1];  // the loudness total (FrameRec::band[0] after phase 2's loudness step)
  int zcr;
  int roll_m;
  uint32_t loud_max;
  float sharp_sum;
};
static_assert(sizeof(ScalIn) == 80, "10 words");
static_assert(offsetof(FrameRec, band) == 56 && offsetof(FrameRec, zcr) == 504 && offsetof(FrameRec, sharp_sum) == 516,
              "the scalar inputs: FrameRec words 0..7 and 63..64");
// Scalars once per window of kScalBatches batches, one lane per frame (scalar_pass), instead of
// one lane per (feature, frame) in every batch's phase 2 -- for launches that compute a spectrum
// (KernelArgs::scal_defer; plan.cpp says when)
constexpr bool kScalDefer = true;

// Record fb (< 4) of the wave's batch and small per-lane offsets by 24-bit multiplies: the lane
// indices come through opaque() (no range the compiler can see), and a 32-bit v_mul_lo_u32 /
// 64-bit v_mad_u64_u32 is a multi-pass instruction where v_mul_u32_u24 is one VALU op.
__device__ __forceinline__ FrameRec& rec_at(FrameRec* recs, int fb) {
  return *reinterpret_cast<FrameRec*>(reinterpret_cast<unsigned char*>(recs) + __umul24((unsigned)fb, (unsigned)sizeof(FrameRec)));
}

// Math.pow(x, 0.23) rounded to float32 (loudness.js:62), without the f64 exp/log routines: x = m 2^e with m in
// [0.5, 1); log2 m from the f32 hardware log of (float)m (the rounding of m moves log2 m by < 2^-24 / ln 2);
// 0.23 e = q + r / 100 exactly in integers (23 e = 100 q + r, 0 <= r < 100), so y = 0.23 log2 x = q + f with
// f = r / 100 + 0.23 log2 m in float32 (|error| < 1e-7), and 2^y = 2^q 2^f from the f32 hardware exp2.
// Relative error ~1.2e-7 (a float32 ulp or two).
__device__ __forceinline__ float pow023(double x) {
  // 0, inf, NaN (a band sum is never negative): pow's values, without the library routine
  // (its f64 log/exp code would run for a whole wave whenever one band of a frame is silent)
  if (!(x > 0.0 && x < __builtin_huge_val())) return x == 0.0 ? 0.0f : x > 0.0 ? __builtin_huge_valf() : (float)x;
  const int e = __builtin_amdgcn_frexp_exp(x);                  // x = m 2^e, m in [0.5, 1); e in [-1073, 1024]
  const float l2m = __builtin_amdgcn_logf((float)__builtin_amdgcn_frexp_mant(x));  // [-1, 0]
  const uint32_t u = (uint32_t)(23 * e + 25000);                 // 23 e + 250 * 100 > 0
  const uint32_t qq = u / 100u, r = u - 100u * qq;
  float f = __builtin_fmaf(0.23f, l2m, (float)r * 0.01f);        // (-0.23, 1)
  int q = (int)qq - 250;
  if (f < 0.0f) {
    f += 1.0f;
    q -= 1;
  }
  return ldexpf(__builtin_amdgcn_exp2f(f), q);
}

// Math.log(x) of a float32, rounded to float32 (mfcc.js:64): ln x = (e + log2 m) ln 2 with
// x = m 2^e, m in [1, 2) exact and log2 m from the f32 hardware log; |error| ~4e-8 absolute.
__device__ __forceinline__ float ln_f32(float x) {
  // 0 -> -inf, inf -> inf, NaN -> NaN (a mel energy is never negative), as Math.log
  if (!(x > 0.0f && x < __builtin_huge_valf())) return x == 0.0f ? -__builtin_huge_valf() : x;
  int e;
  const float m = 2.0f * frexpf(x, &e);
  return (float)(((double)(e - 1) + (double)__builtin_amdgcn_logf(m)) * kLn2);
}

// Math.log of a float32 in double, rounded to float32 (mfcc.js:64 as the reference-order MFCC runs it), without
// the library's double-double log for almost every input: x = 2^e m, m in [1, 2) with c the centre of m's 1/64
// of the range (plan table: 1/c rounded, -ln(1/c)), r = m (1/c) - 1 (|r| <= 2^-7, one rounding), ln(1 + r) to
// r^6 (truncation < 2^-51.8), y = e ln2 - ln(1/c) + ln(1 + r): |y - ln x| < 2^-50.5 + 2^-52 |y|, and so is the
// reference's own log (within an ulp). When y +- (2^-50 + 2^-51 |y|) round to one float32, that float is the
// reference's; otherwise -- and for 0, denormal, infinite or NaN inputs -- the library log decides (rare: the
// interval straddles a float32 rounding boundary with probability ~2^-27 at |y| ~ 1).
__device__ __forceinline__ float ref_ln(float v, GTw lt) {
  const uint32_t b = __builtin_bit_cast(uint32_t, v);
  const uint32_t ef = b >> 23;  // the exponent field; >= 256 for a negative input
  float out = 0.0f;
  bool slow = ef - 1u >= 254u;  // not a positive normal float
  if (!slow) {
    const double m = (double)__builtin_bit_cast(float, (b & 0x7FFFFFu) | 0x3F800000u);
    const double2 t = ld_tw(lt, (int)((b >> 17) & 63u));
    const double ed = (double)((int)ef - 127);
    const double r = __builtin_fma(m, t.x, -1.0);
    double q = __builtin_fma(r, -1.0 / 6.0, 0.2);
    q = __builtin_fma(r, q, -0.25);
    q = __builtin_fma(r, q, 1.0 / 3.0);
    q = __builtin_fma(r, q, -0.5);
    const double p = __builtin_fma(r * r, q, r);
    double y = p + t.y;
    y = __builtin_fma(ed, 1.90821492927058770002e-10, y);  // ln2_lo
    y = __builtin_fma(ed, 6.93147180369123816490e-01, y);  // ln2_hi (32 significant bits: e ln2_hi exact)
    const double d = __builtin_fma(__builtin_fabs(y), 0x1p-51, 0x1p-50);
    const float lo = (float)(y - d), hi = (float)(y + d);
    out = lo;
    slow = lo != hi;
  }
  if (__ballot(slow)) {
    if (slow) out = (float)log((double)v);
  }
  return out;
}

// Arguments live in the kernarg segment (constant address space 4: scalar loads).
typedef const KernelArgs __attribute__((address_space(4))) KArgs;

// Kernel arguments read through an opaque pointer into the kernarg segment: the compiler
// re-loads fields (scalar loads, K$ hits) after each acquisition point instead of keeping
// ~40 pointers resident in registers across the whole batch loop.
__device__ __forceinline__ KArgs* args_ptr() {
  KArgs* p = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

// KernelArgsInline::frame of a one-frame launch that carries its frame in the kernel arguments (INL)
__device__ __forceinline__ const float* inline_frame_ptr() {
  return (const float*)((const __attribute__((address_space(4))) unsigned char*)args_ptr() + kInlineFrameOff);
}

// Pointers read through args_ptr() are generic; re-type them as global (address space 1)
// so loads and stores are global_* (vmcnt only), never flat_* (which also ties up lgkmcnt).
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gbl(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}

// A wave-uniform pointer passed through readfirstlane: loop strength reduction cannot then fold
// a lane offset added later into a per-lane 64-bit induction variable. Such a variable (the
// frame address, the complex output's) was carried across the batch loop in a VGPR pair and
// spilled once per batch, and those scratch stores reached HBM: 128 B per frame, WRITE_SIZE
// 1.8x the outputs. The loads and stores then take an SGPR base and a 32-bit lane offset.
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return (T*)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <typename T>
__device__ __forceinline__ void put_scalar(KArgs* a, int i, uint64_t f, double v) {
  if (a->out.scalars[i]) gbl(static_cast<T*>(a->out.scalars[i]))[f] = (T)v;
}

template <int N>
struct Lds {
  using G = Geo<N>;
  // One slot buffer per wave: FFT exchanges, then the frame's amplitude row, its prefix
  // sums and the mel segment sums (mel_energies) in turn.
  static constexpr size_t slot_off = 0;
  static constexpr size_t slot_bytes = (size_t)4 * G::SLOT_PHYS * 8;
  static_assert(G::SLOT_PHYS >= G::R * 64 + 2, "the dense mel entries (mel_energies) must fit the slot buffer");
  // Per wave, the 5 x 64 table of moment partials (transposed reduction) when it is not in
  // the slot buffer (MOM_SLOT: only N = 256 keeps a table of its own).
  static constexpr size_t mom_off = slot_off + slot_bytes;
  static constexpr size_t mom_bytes = (G::MOM_LDS && !G::MOM_SLOT) ? (size_t)4 * 5 * G::MOM_STRIDE * 8 : 0;
  static_assert(!G::MOM_SLOT || (size_t)G::SLOT_PHYS >= (size_t)5 * G::MOM_STRIDE, "moment table must fit the slot buffer");
  // Frame records: FPW per wave.
  static constexpr size_t rec_off = mom_off + mom_bytes;
  // Kernel constants read per lane, staged once per workgroup: the 13 scalar output
  // pointers and the 25 bark band limits. Read from LDS (lgkmcnt) rather than global
  // memory: a vector-memory wait is in issue order (vmcnt), so a global read here would
  // also wait for every output store and frame load issued before it.
  static constexpr size_t kc_off = rec_off + (size_t)G::FB * sizeof(FrameRec);
  static constexpr size_t kc_bytes = 16 * 8 + 32 * 4;
  // The tame passes' per-lane twiddles (Geo<N>::TW_LDS, TwLds), staged once per workgroup.
  static constexpr size_t twl_off = kc_off + kc_bytes;
  static constexpr size_t twl_bytes = Geo<N>::TW_LDS ? (size_t)TwLds<N>::total() * 16 : 0;
  static_assert(twl_off % 16 == 0, "double2 alignment");
  // The DCT table (mfcc.js:67-83), staged once per workgroup, sized per plan.
  static constexpr size_t dct_off = twl_off + twl_bytes;
  static size_t bytes(int ncoef, int nfilt) { return dct_off + (size_t)ncoef * ((nfilt + 7) & ~7) * 4; }
};

// DPP move of one dword (bound_ctrl: lanes without a source read 0).
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, true));
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xF, true);
}

// Mel band energies of one frame, mfcc.js:40-62: E_j = sum_k w_jk p_k, p_k = a_k^2 (float32).
// The triangular filters split the bins into segments m = [b_m, b_{m+1}): every bin
// belongs to one segment, and band j = (rising half on segment j) + (falling half on
// segment j+1). So E_j = U_j + D_{j+1} with U_m = sum_{k in m} up(k) p_k and
// D_m = sum_{k in m} dn(k) p_k: two segmented sums over the bins, computed as in-lane
// runs plus one segmented scan across the lanes. Where the segments start
// does not depend on the frame, so every branch of that logic is a plan table
// (plan.cpp mel_lane_tables): per bin a keep factor (0 restarts the sums) and the scratch
// slot the running sums are stored to, per lane the keeps of the six scan steps and the two
// slots of the head and tail totals. No selects, one packed multiply and one packed FMA per
// bin, one DPP-fused FMA per scan step and sum. No cross-segment sums are formed, so there
// is no cancellation; the sums are float32 like the reference's Float32Array accumulation,
// in a different order.
// The lane's record of the frame-independent mel tables (plan.cpp mel_lane_tables), issued
// before the moment sums so that the load latency hides behind the reductions.
template <int N>
struct MelTab {
  static constexpr int R = Geo<N>::R, W = mel_rec_words(R), B = (R + 3) / 4;
  uint32_t w[W];
  __device__ __forceinline__ void load(KArgs* ap, int lane) {
    const auto src = gbl(ap->t.mel_rec) + W * lane;
#pragma unroll
    for (int i = 0; i < W; ++i) w[i] = src[i];
  }
  static constexpr int WW = mel_weight_words(R);
  // (rise, fall) of bin jj: the stored pair, or the rising weight and 1 - rising in float32
  __device__ __forceinline__ f32x2 weights(int jj) const {
    if constexpr (WW == 2 * R) return f32x2{__builtin_bit_cast(float, w[2 * jj]), __builtin_bit_cast(float, w[2 * jj + 1])};
    const float up = __builtin_bit_cast(float, w[jj]);
    return f32x2{up, 1.0f - up};
  }
  __device__ __forceinline__ float keep(int jj) const { return (float)((w[WW + jj / 4] >> (8 * (jj % 4))) & 0xFFu); }
  __device__ __forceinline__ float scan_keep(int s) const { return (float)((w[WW + B + s / 4] >> (8 * (s % 4))) & 0xFFu); }
  __device__ __forceinline__ uint32_t asm_u() const { return w[WW + B + 2]; }  // byte offsets of U_band
  __device__ __forceinline__ uint32_t asm_d() const { return w[WW + B + 3]; }  // ... and of D_{band+1}
};

// Mel band energies of one frame, mfcc.js:40-62: E_j = sum_k w_jk p_k, p_k = a_k^2 (float32).
// The triangular filters split the bins into segments m = [b_m, b_{m+1}): every bin
// belongs to one segment, and band j = (rising half on segment j) + (falling half on
// segment j+1). So E_j = U_j + D_{j+1} with U_m = sum_{k in m} up(k) p_k and
// D_m = sum_{k in m} dn(k) p_k: two segmented sums over the bins, computed as in-lane
// runs plus one segmented scan across the lanes. Where the segments start
// does not depend on the frame, so every branch of that logic is a plan table (MelTab,
// plan.cpp mel_lane_tables): per bin the weight pair and a keep factor (0 restarts the sums),
// per lane the keeps of the six scan steps and, per band, where its two segment totals end up.
// Each lane stores its running sums before bins 1..R-1 at fixed entries of the slot buffer
// (immediate offsets: no per-bin address), then the scan's carry into it; band j sums
// carry-or-zero + entry for U_j and D_{j+1}. No selects: per bin a packed multiply and a packed
// FMA, per scan step two DPP moves and a packed FMA. No cross-segment sums are formed, so there
// is no cancellation; the sums are float32 like the reference's Float32Array accumulation, in a
// different order (and the falling weight is 1 - rising in float32, within an ulp of the f64 ratio).
template <int N>
__device__ __forceinline__ void mel_energies(KArgs* ap, const float (&av)[Geo<N>::R], int lane, float2* buf,
                                             FrameRec& rec, const MelTab<N>& mt) {
  constexpr int R = Geo<N>::R;
  const int nf = ap->nfilt;
  wave_sync();  // band-sum reads of the prefix buffer are done
  float2* mine = buf + lane;
  f32x2 acc = {0.0f, 0.0f};
#pragma unroll
  for (int jj = 0; jj < R; ++jj) {
    const float p = av[jj] * av[jj];  // powerSpectrum.js
    if (jj > 0) mine[(jj - 1) * 64] = make_float2(acc.x, acc.y);
    const float kp = mt.keep(jj);
    const f32x2 w = mt.weights(jj), pp = {p, p}, kk = {kp, kp};
    acc = __builtin_elementwise_fma(w, pp, acc * kk);
  }
  f32x2 sc = acc;
  auto step = [&](float u, float d, int s) {
    const f32x2 src = {u, d}, ks = {mt.scan_keep(s), mt.scan_keep(s)};
    sc = __builtin_elementwise_fma(src, ks, sc);
  };
  step(dpp_f<0x111>(sc.x), dpp_f<0x111>(sc.y), 0);  // row_shr:1
  step(dpp_f<0x112>(sc.x), dpp_f<0x112>(sc.y), 1);  // row_shr:2
  step(dpp_f<0x114>(sc.x), dpp_f<0x114>(sc.y), 2);  // row_shr:4
  step(dpp_f<0x118>(sc.x), dpp_f<0x118>(sc.y), 3);  // row_shr:8
  // (the row broadcasts write every row: the rows a step must not add to have keep 0 in the plan,
  // so no zero has to be written ahead of a row-masked move)
  step(dpp_f<0x142>(sc.x), dpp_f<0x142>(sc.y), 4);  // row_bcast:15 (rows 1, 3)
  step(dpp_f<0x143>(sc.x), dpp_f<0x143>(sc.y), 5);  // row_bcast:31 (rows 2, 3)
  const float xu = dpp_f<0x138>(sc.x), xd = dpp_f<0x138>(sc.y);  // exclusive: carry into this lane
  mine[(R - 1) * 64] = make_float2(xu, xd);
  if (lane == 63) buf[R * 64] = make_float2(sc.x, sc.y);
  if (lane == 0) buf[R * 64 + 1] = make_float2(0.0f, 0.0f);
  wave_sync();
  if (lane < nf) {  // nf <= kMaxMel = 64
    const unsigned char* b = reinterpret_cast<const unsigned char*>(buf);
    const uint32_t u = mt.asm_u(), d = mt.asm_d();
    const float U = reinterpret_cast<const float2*>(b + (u & 0xFFFFu))->x + reinterpret_cast<const float2*>(b + (u >> 16))->x;
    const float D = reinterpret_cast<const float2*>(b + (d & 0xFFFFu))->y + reinterpret_cast<const float2*>(b + (d >> 16))->y;
    rec.lm[lane] = U + D;
  }
}

// float32 bits of 2^64: an amplitude a >= 2^64 has a * a = +inf in float32 (a < 2^64 stays
// below FLT_MAX after rounding), i.e. an infinite power spectrum bin (powerSpectrum.js).
constexpr uint32_t kPowOverflowBits = 0x5F800000u;

// Bark-band sums and mel energies of a frame with a non-finite amplitude or power (or an
// amplitude total of 2^64 or more), summed exactly as the reference does (see frame_phase1).
// The amplitude row is rewritten to the slot buffer.
template <int N>
__device__ __forceinline__ void nonfinite_frame_sums(KArgs* ap, const float (&av)[Geo<N>::R], int lane,
                                                               float2* buf, FrameRec& rec, int lmo = 0) {
  constexpr int L = N / 2, R = Geo<N>::R;
  float* amp = reinterpret_cast<float*>(buf);
  wave_sync();  // prefix reads (band sums) are done
#pragma unroll
  for (int jj = 0; jj < R; ++jj) amp[R * lane + jj] = av[jj];
  wave_sync();
  if (lane < kBark) {  // loudness.js:47-66: sumArray over [lim_b, lim_{b+1}) in double
    const auto lim = gbl(ap->t.bblim);
    double sum = 0.0;
    for (int k = lim[lane]; k < lim[lane + 1]; ++k) sum += (double)amp[k];
    rec.band[lane] = sum;
  }
  if (ap->need_mfcc) {  // mfcc.js:53-62: every bin, double weight x float power, float32 sum
    const int nf = ap->nfilt;
    const auto b = gbl(ap->t.mel_bins);
    for (int j = lane; j < nf; j += 64) {
      const int b0 = b[j], b1 = b[j + 1], b2 = b[j + 2];
      float e = 0.0f;
      for (int k = 0; k < L; ++k) {
        double w = 0.0;
        if (k >= b0 && k < b1) w = (double)(k - b0) / (b1 - b0);
        if (k >= b1 && k < b2) w = (double)(b2 - k) / (b2 - b1);
        const float p = amp[k] * amp[k];
        e = (float)((double)e + w * (double)p);
      }
      rec.lm[lmo + j] = e;
    }
  }
}

// MGX_FLAG_MFCC_REFERENCE (the CHAIN kernels): the mel band energies in the reference's
// own order (mfcc.js:53-62), over the power rows phase 1 left in the wave's ring in device memory
// (KernelArgs::chain_rows). Each band of each frame is one serial chain: from its first bin in
// ascending order, the weight (an IEEE double quotient, plan table) times the float32 power rounded
// to double, added to the Float32Array element in double and stored back to float32 -- exactly the
// reference's operations, so the sums are the reference's bits. The host schedule (plan.cpp
// chain_schedule) packs the chains into 64 / F tracks of F lanes (one lane per frame), each track
// running its bands' chains back to back in groups of 8 steps; per group and lane a control word
// gives the row offset, whether a chain starts (its first step adds to 0) and where the chain that
// ends there is stored (a FrameRec::lm entry, or the lane's scratch word in the slot buffer, which
// is free in phase 2).
//   F = 8 (KernelArgs::chain_pair, nfilt <= 31): the chains of two consecutive batches of the wave
//     run together, in the second batch's phase 2 (ring slots 0..3 the first batch, 4..7 the
//     second): the first batch's energies go to the upper half of its records' lm (lm[32 + band]);
//     lm[31] / lm[63] hold the frame's non-finite flag. have_cur = false (the wave's last batch was
//     the first of a pair): the second batch's chains run on stale rows into lm[band] of records
//     nobody reads.
//   F = 4 (more bands): the batch's chains in its own phase 2, slots 0..3, the non-finite flag a bit
//     of the record's zcr count.
// A non-finite frame's energies (nonfinite_frame_sums) wait at the start of its ring slot and are
// put back after the chains. Per step: the conversion, product, sum and the two roundings on the
// VALU; per group two 16-byte row loads, the 8 weights (shared by the track's F lanes), the next
// control word and one LDS store.
template <int N, bool PAIR>
__device__ __forceinline__ void mel_chains(KArgs* q, int lane, GF ring, FrameRec* recs, float2* buf, bool have_cur) {
  constexpr bool pair = PAIR;
  constexpr int L = N / 2;
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) f32x4* GF4;
  static_assert(sizeof(FrameRec) == kRecBytes && offsetof(FrameRec, lm) == kRecLmOff, "chain_schedule's record offsets");
  const auto ctl = gbl(q->t.chain_ctl);
  constexpr int F = PAIR ? 8 : 4;
  const int ng = q->chain_groups;
  const auto wp = gbl(q->t.chain_w) + (lane / F) * (ng * 8);
  unsigned char* const rb = reinterpret_cast<unsigned char*>(recs);
  float* const scratch = reinterpret_cast<float*>(buf) + lane;
  auto store = [&](uint32_t c, double acc) {
    float* dst = (c & (1u << 26)) ? reinterpret_cast<float*>(rb + ((c >> 13) & 0xFFFu)) : scratch;
    *dst = (float)acc;
  };
  double acc = 0.0;  // the Float32Array element, held exactly in double
  uint32_t c = ctl[lane], cn = ctl[64 + lane];  // (the table has ng + 1 >= 2 rows)
  // A group's power-row values are loaded one group ahead: their loads issue before the previous group's 8
  // steps, so the ring's memory latency (it is written to device memory in phase 1 and rarely still in the L2)
  // overlaps those steps instead of stalling every group. (The weights, a few KB read by every wave, come from
  // the L2; holding them one group ahead as well took the kernel past 128 VGPRs.)
  // (N = 256, at 6 waves per SIMD: the second set spilled; it keeps the loads in the group)
  constexpr bool kAhead = N >= 512;
  f32x4 p0, p1;
  if constexpr (kAhead) {
    const GF4 pr = (GF4)(ring + (c & 0x1FFFu));  // a multiple of 4 floats (chain_schedule)
    p0 = pr[0];
    p1 = pr[1];
  }
  for (int g = 0; g < ng; ++g) {
    if constexpr (!kAhead) {
      const GF4 pr = (GF4)(ring + (c & 0x1FFFu));
      p0 = pr[0];
      p1 = pr[1];
    }
    // (the last group fetches its own row again: a harmless reload in place of a branch)
    const GF4 prn = (GF4)(ring + ((kAhead && g + 1 < ng ? cn : c) & 0x1FFFu));
    const f32x4 n0 = kAhead ? prn[0] : p0, n1 = kAhead ? prn[1] : p1;
    double w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) w[u] = wp[g * 8 + u];
    const uint32_t cnn = ctl[(g + 2 < ng ? g + 2 : ng) * 64 + lane];
    const float p[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
    store(c, acc);  // the chain that ends here (or the scratch word)
    // a chain starting here adds its first product to 0 (a select: acc may be an overflowed +inf)
    const double a0 = (c & (1u << 25)) ? 0.0 : acc;
    acc = (double)(float)(a0 + w[0] * (double)p[0]);
#pragma unroll
    for (int u = 1; u < 8; ++u) acc = (double)(float)(acc + w[u] * (double)p[u]);  // two roundings, the float32 store
    p0 = n0;
    p1 = n1;
    c = cn;
    cn = cnn;
  }
  store(c, acc);
  // the non-finite frames' own sums back from their ring slots (wave-uniform, rare)
  wave_sync();
  for (int fr = 0; fr < F; ++fr) {
    FrameRec& r = recs[fr & 3];
    const int lmo = pair && fr < 4 ? 32 : 0;
    const bool nf = pair ? r.lm[lmo + 31] != 0.0f : (r.zcr & kChainSkip) != 0;
    if (nf && (!pair || fr < 4 || have_cur) && lane < q->nfilt) r.lm[lmo + lane] = ring[fr * L + lane];
  }
}

// One frame of phase 1 (wave-level). x holds the raw samples (lane-strided chunks). WREG: the window in
// wreg (registers loaded once per launch: Geo::WIN_REG, and the resident launches, whose one-frame requests
// would otherwise each wait for the window's table loads).
template <int N, bool FAITH, bool LITERAL, bool SUB, bool LIGHT, bool NOTIME, bool CHAIN, bool WREG = Geo<N>::WIN_REG>
__device__ __forceinline__ void frame_phase1(KArgs* ap, float (&x)[Geo<N>::CH], int fb, uint64_t f, bool valid,
                                             int lane, const int (&lp)[Geo<N>::NPASS], const KlTab<N>& kl,
                                             bool dc_lane, float2* buf, double* mom, FrameRec* recs,
                                             const int* klim, float (&xn)[Geo<N>::PREFETCH ? Geo<N>::CH : 1],
                                             GF next, const double2* twl, const float (&wreg)[Geo<N>::CH],
                                             uint32_t blim, float* rows, int it, bool ntf) {
  using G = Geo<N>;
  using PG = PassGeo<N>;
  constexpr int L = G::L, R = G::R, CH = G::CH;
  constexpr bool TWL = Geo<N>::TW_LDS;
  float* amp = reinterpret_cast<float*>(buf);  // the frame's amplitude row, once the FFT is done
  double* pbuf = reinterpret_cast<double*>(buf);

  // mid-frame prefetch of the next frame (G::PF == 2), after the mel records are issued
  // (frames without spectral features: right away)
  auto prefetch_next = [&]() {
    if constexpr (G::PF == 2) ld_frame<CHAIN>(xn, next, (unsigned)lane, ntf);
  };
  // The window: held in registers for the launch at N = 1024 (Geo::WIN_REG); otherwise its
  // table loads are issued before the energy / zcr reductions, so their latency hides behind
  // them rather than at the window step after the reductions' branches (1 % faster at
  // N = 512; a lane-major table read as 16-byte loads was 2-5 % slower at 512 and 2048).
  float wv[CH];
  if (WREG) {
#pragma unroll
    for (int c = 0; c < CH; ++c) wv[c] = wreg[c];
  } else if (ap->need_spectrum) {
    const GF w = gbl(ap->t.window);
#pragma unroll
    for (int c = 0; c < CH; ++c) wv[c] = w[c * 64 + lane];
  }
  MGX_MARK(energy_zcr);
  prio_hi<16>();
  // rms.js / energy.js: sum of squares; zcr.js: sign changes of adjacent samples,
  // `x >= 0` vs `x < 0` (so -0 is non-negative and NaN never counts).
  // Sum of squares as packed float32 FMAs over pairs of chunks; zcr from one ballot per
  // chunk (x < 0): without NaN samples, x >= 0 is its complement. A NaN sample makes that
  // lane's sum of squares NaN, and such frames count with both comparisons.
  f32x2 e2 = {0.0f, 0.0f};
#pragma unroll
  for (int c = 0; c < CH; c += 2) {
    const f32x2 xv = {x[c], x[c + 1]};
    e2 = __builtin_elementwise_fma(xv, xv, e2);
  }
  const float e32 = e2.x + e2.y;
  int z = 0;
  uint64_t pge = 0, plt = 0;
  // (a feature subset, SUB, skips the ballots without zcr and the wave sum without rms /
  // energy; the lane partials e32 stay: the FFT's range test reads them)
  // (NOTIME: the all-feature kernel's schedule without rms / energy / zcr, compiled out)
  const bool want_zcr = SUB ? (bool)ap->need_zcr : !NOTIME, want_energy = SUB ? (bool)ap->need_energy : !NOTIME;
  if (!want_zcr) {
  } else if (__ballot(e32 != e32)) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const uint64_t g = __ballot(x[c] >= 0.0f), l = __ballot(x[c] < 0.0f);
      z += __popcll(((g & (l >> 1)) | (l & (g >> 1))) & 0x7FFFFFFFFFFFFFFFull);
      if (c > 0) z += (int)((((pge >> 63) & l) | ((plt >> 63) & g)) & 1ull);
      pge = g;
      plt = l;
    }
  } else {
    // without NaN samples x >= 0 is the complement of x < 0, so a sign change between samples
    // i and i + 1 is bit i of s ^ (s >> 1) over the frame's sign sequence s (sample 64 c + l is
    // bit l of chunk c's ballot): the chunk's 63 inner pairs and, in bit 63, the pair it forms
    // with the next chunk's first sample (the last chunk's bit 63 compares with itself: 0)
    uint64_t l[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) l[c] = __ballot(x[c] < 0.0f);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const uint64_t nxt = c + 1 < CH ? l[c + 1] << 63 : l[c] & 0x8000000000000000ull;
      z += __popcll(l[c] ^ ((l[c] >> 1) | nxt));
    }
  }
  // float32 partial sums are within 1e-6 relative of the double sum; a wave whose
  // partials leave [2^-100, 2^100] (silence, denormal or huge input) redoes it in double.
  double e = 0.0;
  if (!want_energy) {
  } else if (__ballot(!(e32 >= 0x1p-100f && e32 <= 0x1p100f))) {
    double e64 = 0.0;
#pragma unroll
    for (int c = 0; c < CH; ++c) e64 = __builtin_fma((double)x[c], (double)x[c], e64);
    e = wave_sum(e64);
  } else {
    // the 64 lane partials summed in float32 too (6 DPP-fused adds instead of 6 f64 DPP
    // steps): ~4e-7 relative at most on top of the partials' own ~1e-6, against the 1e-5 bar
    // (only lane 63 is read: the row broadcasts need no row mask -- rows that should not add get
    // values nobody reads -- so no zero has to be written ahead of them)
    float t = e32;
    t += dpp_f<0xB1>(t);
    t += dpp_f<0x4E>(t);
    t += dpp_f<0x141>(t);
    t += dpp_f<0x140>(t);
    t += dpp_f<0x142>(t);
    t += dpp_f<0x143>(t);
    e = (double)__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t), 63));
  }
  if (lane == 0) {
    recs[fb].energy = e;
    recs[fb].zcr = z;
  }
  if (!ap->need_spectrum) {  // time-only features: the next frame now (its registers are free)
    prefetch_next();
    prio_lo<16>();
    return;
  }
  // Every sample finite and |x| <= 2^50 (each lane's sum of squares <= 2^100, not NaN):
  // no stage of the FFT can reach an infinity (bfly_mixed_tame).
  const bool tame = !__ballot(!(e32 <= 0x1p100f));
  MGX_MARK(window);

  // src/meyda.js:158-168: windowed[i] = sig[i] * w[i], stored to Float32Array
  // (the exact double product rounded once == a float32 multiply).
  {
#pragma unroll
    for (int c = 0; c < CH; c += 2) {  // packed float32 multiplies
      const f32x2 xv = {x[c], x[c + 1]}, wp = {wv[c], wv[c + 1]};
      const f32x2 y = xv * wp;
      x[c] = y.x;
      x[c + 1] = y.y;
    }
  }
  if constexpr (LITERAL) {
    // The snapshot never transforms per buffer: |w x| is the "spectrum".
#pragma unroll
    for (int c = 0; c < R; ++c) amp[pa(c * 64 + lane)] = fabsf(x[c]);
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
    prio_lo<16>();
    MGX_MARK(stage0_done);
    MGX_STAMP(3);
    GTw tw = gbl(ap->t.tw);
    GTwf twf = gbl(ap->t.twf);
    GTw twm = gbl(ap->t.twm);
    // G::LPREMAT: the lane parts are recomputed from the lane id in each frame (a few bit
    // operations) instead of being kept live across the frame loop, where the allocator
    // spilled them and reloaded from scratch in the middle of the FFT (a vector-memory wait).
    int lpf[G::NPASS];
#pragma unroll
    for (int p = 0; p < G::NPASS; ++p) lpf[p] = G::LPREMAT ? PG::lanepart(p, opaque(lane)) : lp[p];
    if constexpr (FAITH) {
      // pass 0 has no mixed pairs; the later passes take the tame form when they can
      run_stages<N, 0, 0, FAITH, false, TWL>(v, lpf[0], tw, twf, twm, twl);
      MGX_MARK(pass0_done);
      if (tame) run_passes<N, 1, FAITH, true, TWL>(v, lpf, buf, tw, twf, twm, twl);
      else run_passes<N, 1, FAITH, false, TWL>(v, lpf, buf, tw, twf, twm, twl);
    } else {
      run_passes<N, 0, FAITH, false, TWL>(v, lpf, buf, tw, twf, twm, twl);
    }
    MGX_MARK(fft_done);
    MGX_STAMP(4);
    prio_hi<32>();
    const bool want_cplx = ap->out.complex_real != nullptr;
    // src/meyda.js:104-114: |X_k| for k < N/2, rounded to float32.
    float ar[R];
    if constexpr (FAITH) {
      // The range test of every slot as one unsigned min and max of the float bits: each a is
      // >= +0 or NaN, so unsigned order is float order with NaN above +inf (caught by the max).
      uint32_t amin = 0xFFFFFFFFu, amax = 0u;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        bool okr;
        ar[r] = slot_amp_rsq(v[r].x, v[r].y, okr);
        uint32_t b = __builtin_bit_cast(uint32_t, ar[r]);
        // (the packed DC/Nyquist slot is replaced below: its range does not matter)
        if (PG::rpart(G::NPASS - 1, r) == 0) b = dc_lane ? 0x3F800000u : b;
        amin = min(amin, b);
        amax = max(amax, b);
      }
      const bool ok = amin >= __builtin_bit_cast(uint32_t, 0x1p-40f) && amax <= __builtin_bit_cast(uint32_t, 0x1p60f);
      if (__ballot(!ok)) {  // a zero, tiny, huge or non-finite |X|^2 somewhere in the frame
#pragma unroll
        for (int r = 0; r < R; ++r) ar[r] = slot_amp<FAITH>(v[r].x, v[r].y);
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) ar[r] = slot_amp<FAITH>(v[r].x, v[r].y);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool dc = (PG::rpart(G::NPASS - 1, r) == 0) && dc_lane;
      if (dc) ar[r] = fabsf(v[r].x);  // slot 0 packs (X[0], X[N/2]), both real
    }
    prio_lo<32>();
    MGX_MARK(amp_done);
    MGX_STAMP(5);
    wave_sync();  // the last exchange's reads are done: the slot buffer is free
    if (want_cplx) {
      // natural-order half spectrum X[0..N/2] in the slot buffer
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool dc = (PG::rpart(G::NPASS - 1, r) == 0) && dc_lane;
        if (dc) {
          buf[0] = make_float2(v[r].x, 0.0f);
          buf[L] = make_float2(v[r].y, 0.0f);
        } else {
          // kl holds pa(bin). (opaque: the complex output's 2R addresses, derived here, were otherwise
          // hoisted out of the frame loop and held in R VGPRs for the whole launch -- spilled at N = 2048
          // -- by every launch, with or without a complex output)
          buf[pa_inv(opaque(kl(r)))] = v[r];
        }
      }
      wave_sync();
      if (valid) {
        // complexSpectrum.js: the full N-point spectrum, X[N-k] = conj(X[k])
        auto cr = uniform_ptr(gbl(ap->out.complex_real) + f * (uint64_t)N);
        auto ci = uniform_ptr(gbl(ap->out.complex_imag) + f * (uint64_t)N);
        for (unsigned i = lane; i < (unsigned)N; i += 64) {
          const float2 zz = i <= L ? buf[i] : buf[N - i];
          st_out(&cr[i], zz.x);
          st_out(&ci[i], i <= L ? zz.y : -zz.y);
        }
      }
      wave_sync();
    }
    prio_hi<2>();
#pragma unroll
    for (int r = 0; r < R; ++r) amp[kl(r)] = ar[r];  // kl(r) = pa(bin)
  }
  wave_sync();

  if (valid && ap->out.amplitude_spectrum) {
    auto o = uniform_ptr(gbl(ap->out.amplitude_spectrum) + f * (uint64_t)L);
#pragma unroll
    for (int c = 0; c < R; ++c) st_out(&o[c * 64 + (unsigned)lane], amp[pa(c * 64 + lane)]);
  }
  if (valid && ap->out.power_spectrum) {
    auto o = uniform_ptr(gbl(ap->out.power_spectrum) + f * (uint64_t)L);
#pragma unroll
    for (int c = 0; c < R; ++c) {
      const float av = amp[pa(c * 64 + lane)];
      st_out(&o[c * 64 + (unsigned)lane], av * av);  // powerSpectrum.js
    }
  }
  if constexpr (CHAIN) {
    // the frame's power row (powerSpectrum.js) for the mel chains in phase 2 (mel_chains): ring slot fb, or
    // with paired batches 4 (it & 1) + fb. Stored here from the amplitude row in LDS, lane l of store c
    // writing bin 64 c + l: 256 contiguous bytes per store, where the lane's own bins [R l, R l + R) were
    // R 4-byte stores 4 R bytes apart; profiles/r05_chain_rows.txt).
    // A non-finite frame's slot then takes its mel sums instead (below).
    if (ap->need_mfcc) {
      auto row = gbl(rows) + ((ap->chain_pair ? 4 * (it & 1) : 0) + fb) * L;
#pragma unroll
      for (int c = 0; c < R; ++c) {
        const float a = amp[pa(c * 64 + lane)];
        row[c * 64 + (unsigned)lane] = a * a;
      }
    }
  }

  // Per-frame reductions, lane t owns bins [R t, R t + R).
  float av[R];
#pragma unroll
  for (int jj = 0; jj < R; ++jj) av[jj] = amp[pa(R * lane + jj)];
  prio_lo<2>();
  prio_hi<64>();
  MGX_MARK(amp_row_done);
  // The moment and log sums only as far as a feature reads them (need_mom: 0 none, 1 S1 for
  // centroid / slope, 2 S1..S4 and sum log2 a); the amplitude total T0 always (S0, rolloff,
  // the non-finite test). SUB: a feature subset, the flags are read at run time; otherwise
  // every feature is requested and the branches compile away (the all-feature kernel keeps
  // its schedule: run-time branches there cost 0.7 %).
  const int mom_level = LIGHT ? 0 : SUB ? ap->need_mom : 2;
  // light: a subset reading neither the moments nor the prefix row (mfcc alone, spectra):
  // no amplitude total, no scan; the non-finite test from the amplitudes' float bits
  const bool light = LIGHT || (SUB && mom_level == 0 && !ap->need_prefix);
  const bool need_mom = mom_level > 0, need_hi = mom_level > 1;
  double T0 = 0, T1 = 0, T2 = 0, T3 = 0, T4 = 0;
  float l2f = 0.0f;
  // (the sums start from bins 0 and 1 instead of from 0.0: every amplitude is >= +0 or NaN,
  // so 0 + a and fma(1, a, 0) are a itself -- the same sums without the no-op adds)
  if (need_hi) {
    T0 = (double)av[0];
    {
      const double a1 = av[1];
      T0 += a1;
      T1 = T2 = T3 = T4 = a1;
    }
#pragma unroll
    for (int jj = 2; jj < R; ++jj) {
      const double ad = av[jj];
      T0 += ad;
      T1 = __builtin_fma((double)jj, ad, T1);
      T2 = __builtin_fma((double)(jj * jj), ad, T2);
      T3 = __builtin_fma((double)(jj * jj * jj), ad, T3);
      T4 = __builtin_fma((double)(jj * jj * jj * jj), ad, T4);
    }
    // sum log2 a by pairs, log2(a_j a_{j+1}) with the bare v_log_f32 (== log2f for normal
    // inputs; one hardware log per two bins, and the product's rounding is ~2^-24 relative,
    // finer than the log's own ulp). v_log_f32 flushes a denormal input to 0 (-inf): a wave
    // whose sum is not finite (a zero, tiny, infinite or NaN amplitude, or a pair product
    // leaving the normal range; rare) recomputes bin by bin with log2f's scaling.
#pragma unroll
    for (int jj = 0; jj < R; jj += 2) l2f += __builtin_amdgcn_logf(av[jj] * av[jj + 1]);
    if (__ballot(!(__builtin_fabsf(l2f) < __builtin_huge_valf()))) {
      l2f = 0.0f;
#pragma unroll
      for (int jj = 0; jj < R; ++jj) l2f += log2f(av[jj]);
    }
  } else if (need_mom) {
    T0 = (double)av[0];
    T1 = av[1];
    T0 += T1;
#pragma unroll
    for (int jj = 2; jj < R; ++jj) {
      const double ad = av[jj];
      T0 += ad;
      T1 = __builtin_fma((double)jj, ad, T1);
    }
  } else if (!light) {
    T0 = (double)av[0];
#pragma unroll
    for (int jj = 1; jj < R; ++jj) T0 += (double)av[jj];
  }
  // (every amplitude is >= +0 or NaN: unsigned order of the bits is float order, NaN and
  // +inf on top; one max per slot, as the amplitude's range test)
  bool light_nonfinite = false;
  if (light) {
    uint32_t am = 0u;
#pragma unroll
    for (int jj = 0; jj < R; ++jj) am = max(am, __builtin_bit_cast(uint32_t, av[jj]));
    light_nonfinite = __ballot(am >= kPowOverflowBits) != 0;
  }
  MGX_MARK(moments_done);
  prio_hi<8>();
  wave_sync();  // every lane has read the amplitude row: the buffer takes the prefix sums next
  FrameRec& rec = recs[fb];
  // Moments S1..S4 (bin-offset polynomial shift of the local partials) and sum log2 a:
  // five sums over the lanes, through one LDS transpose: lane l writes column l of a 5 x 64
  // table, lanes 0..39 each add 8 entries (stride 8) of one row and 3 DPP steps finish the row
  // in 8-lane groups. With MOM_SLOT (every N but 256) the table is the wave's slot buffer and is
  // reduced right away, before the prefix row takes the buffer; otherwise it has its own LDS
  // and is read back at the end of the frame (after the mel sums).
  constexpr bool kMomLds = G::MOM_LDS;
  constexpr int MS = G::MOM_STRIDE;
  // P_p = sum_j (b + j)^p a_j = sum_m C(p, m) b^(p-m) T_m by a Taylor shift (c_i += b c_{i-1},
  // four sweeps: 10 FMAs; every term is non-negative, so nothing cancels)
  const double bb = (double)(R * lane);
  double P1 = T1, P2 = T2, P3 = T3, P4 = T4;
  if (need_hi) {
    P4 = __builtin_fma(bb, P3, P4); P3 = __builtin_fma(bb, P2, P3); P2 = __builtin_fma(bb, P1, P2); P1 = __builtin_fma(bb, T0, P1);
    P4 = __builtin_fma(bb, P3, P4); P3 = __builtin_fma(bb, P2, P3); P2 = __builtin_fma(bb, P1, P2);
    P4 = __builtin_fma(bb, P3, P4); P3 = __builtin_fma(bb, P2, P3);
    P4 = __builtin_fma(bb, P3, P4);
  } else {
    P1 = __builtin_fma(bb, T0, P1);
  }
  double* const momt = G::MOM_SLOT ? pbuf : mom;
  if (kMomLds && need_mom) {
    // (one lane address per frame, the rows as immediate offsets: five addresses kept across the frame
    // loop were spilled at N = 2048 and reloaded per frame)
    double* const mcol = momt + opaque(lane);
    mcol[0 * MS] = P1;
    if (need_hi) {
      mcol[1 * MS] = P2;
      mcol[2 * MS] = P3;
      mcol[3 * MS] = P4;
      mcol[4 * MS] = (double)l2f;
    }
  }
  // prefix P(k) = sum_{i<k} a_i: lane-exclusive offset + local prefix
  double excl = 0.0, total = 0.0;
  if (!light) {
    const double incl = wave_inclusive_scan(T0);
    excl = dpp_d<0x138>(incl);  // wave_shr:1 (lane 0 reads 0)
    total = readlane_d(incl, 63);
  }
  // the moment transpose's reduction (lanes 0..39: 8 entries of one row, then 3 DPP steps)
  auto mom_reduce = [&]() {
    const int row = lane < 40 ? lane >> 3 : 0;
    const double* src = momt + row * MS + (lane & 7);  // entries g, g+8, ..., g+56 of the row
    double t = ((src[0] + src[8]) + (src[16] + src[24])) + ((src[32] + src[40]) + (src[48] + src[56]));
    t += dpp_d<0xB1>(t);   // quad_perm [1,0,3,2]
    t += dpp_d<0x4E>(t);   // quad_perm [2,3,0,1]
    t += dpp_d<0x141>(t);  // row_half_mirror: each 8-lane group holds its row's total
    if (lane < 40 && (lane & 7) == 0) (&rec.S[1])[row] = t;  // S[1..4], then ln2sum
  };
  if (G::MOM_SLOT && need_mom) {
    wave_sync();
    mom_reduce();
    wave_sync();  // the table's reads are done: the buffer takes the prefix row
  }
  // spectralRolloff.js:6-15: the largest m with P(m) <= 0.99 total (P(0) = 0).
  const double thr = 0.99 * total;
  int cnt = 0;
  const bool need_prefix = LIGHT ? false : SUB ? (bool)ap->need_prefix : true;
  if (need_prefix) {
    double pk = excl;  // P(R lane + jj), accumulated again rather than kept (registers)
#pragma unroll
    for (int jj = 0; jj < R; ++jj) {
      pbuf[pd(R * lane + jj)] = pk;
      cnt += __popcll(__ballot(pk <= thr));
      pk += (double)av[jj];
    }
  }
  const int roll_m = (total > thr) ? cnt - 1 : L;
  MGX_MARK(prefix_done);
  MGX_STAMP(6);
  // The lane's mel records, then (G::PF == 2) the next frame: issued after the last table
  // load this frame waits on before them, so no wait of this frame is held up by the
  // prefetch; the band and mel sums, the moment finish and phase 2 run while it is in
  // flight. (Issued any earlier, the extra live registers spill around the moment sums,
  // and a spill reload is a vector-memory wait behind the prefetch.)
  MelTab<N> mt;
  if (!CHAIN && ap->need_mfcc) mt.load(ap, lane);
  prefetch_next();
  if (!kMomLds && need_mom) {
    const double S1 = wave_sum(P1);
    double S2 = 0, S3 = 0, S4 = 0, l2 = 0;
    if (need_hi) {
      S2 = wave_sum(P2); S3 = wave_sum(P3); S4 = wave_sum(P4);
      l2 = wave_sum((double)l2f);
    }
    wave_sync();
    if (lane == 0) {
      rec.S[1] = S1; rec.S[2] = S2; rec.S[3] = S3; rec.S[4] = S4;
      rec.ln2sum = l2;
    }
  }
  MGX_MARK(prefetch_issued);
  if (need_prefix && lane < kBark) {
    if constexpr (G::BLIM_REG) {
      rec.band[lane] = pbuf[blim >> 16] - pbuf[blim & 0xFFFFu];
    } else {
      const int lb = opaque(lane);  // (an address kept live across the frame loop spills at N = 2048)
      // limits staged in LDS as byte offsets of their prefix-row entries (pd(lim) * 8)
      const unsigned char* pb = reinterpret_cast<const unsigned char*>(pbuf);
      rec.band[lb] = *reinterpret_cast<const double*>(pb + klim[lb + 1]) - *reinterpret_cast<const double*>(pb + klim[lb]);
    }
  }
  if (lane == 0) {
    rec.S[0] = total;
    rec.roll_m = roll_m;
  }
  // A non-finite amplitude (Inf/NaN samples, or overflow in the FFT) breaks the prefix
  // differences (Inf - Inf) and the segment decomposition of the mel sums (the reference's
  // zero weights turn Inf into NaN in every band). Such frames — wave-uniform, rare — take
  // the reference's own summation: bark bands bin by bin in double (loudness.js:47-66),
  // mel bands over all bins in reference order (mfcc.js:53-62).
  // (total = sum of the amplitudes in double: non-finite iff some amplitude is.) A finite
  // amplitude of 2^64 or more has an infinite float32 power (powerSpectrum.js), which the
  // reference's zero weights turn into NaN in every mel band (0 x Inf): such frames take the
  // same path (a total of 2^64 or more is the cheap, conservative test: the path is the
  // reference's own summation, right for any frame).
  MGX_MARK(bands_done);
  MGX_STAMP(7);
  const bool nonfinite = light ? light_nonfinite : !(total < 0x1p64);
  if (nonfinite) {
    // (CHAIN with paired batches: the pair's first batch keeps its mel sums in the upper half of lm)
    nonfinite_frame_sums<N>(ap, av, lane, buf, rec, CHAIN && ap->chain_pair && !(it & 1) ? 32 : 0);
  } else if (!CHAIN && ap->need_mfcc) {
    mel_energies<N>(ap, av, lane, buf, rec, mt);
  }
  if constexpr (CHAIN) {
    // A non-finite frame keeps the mel sums nonfinite_frame_sums formed (its flag: lm[31] of its half, or a
    // bit of its zcr count): they go to the start of its ring slot, over its power row, and mel_chains puts
    // them back after its chains (whose stores do not look at the flag).
    if (ap->need_mfcc) {
      const bool pair = ap->chain_pair;
      auto row = gbl(rows) + ((pair ? 4 * (it & 1) : 0) + fb) * L;
      if (nonfinite) {  // (over the power row stored above)
        wave_sync();
        if (lane < ap->nfilt) row[lane] = rec.lm[(pair && !(it & 1) ? 32 : 0) + lane];
      }
      if (pair) {
        if (lane == 0) rec.lm[(it & 1 ? 0 : 32) + 31] = nonfinite ? 1.0f : 0.0f;
      } else if (nonfinite && lane == 0) {
        rec.zcr = rec.zcr | kChainSkip;
      }
    }
  }
  MGX_MARK(mel_done);
  if (kMomLds && !G::MOM_SLOT && need_mom) {
    wave_sync();
    mom_reduce();
  }
  prio_lo<8>();
  MGX_MARK(frame_end);
  MGX_STAMP(8);
  wave_sync();  // pbuf reads done before the next frame's exchanges reuse the buffer
}

// mfcc.js:85-93: coefficient c of one frame, sum_n dct[c][n] * lm[n] in double, in the
// reference's sequential order. The product of two floats is exact in double, so an FMA
// equals the reference's multiply-then-add. lm and the LDS table are zero-padded to a
// multiple of 8 bands (0 * 0 adds nothing), so groups of 8 loads issue together.
// v / d for the DCT's 1 / ncoef scale (mfcc.js:91) without the IEEE division sequence:
// q0 = v r with r the correctly rounded 1/d, e = v - q0 d (exact by FMA), q0 + e r. By
// Markstein's theorem that is the correctly rounded quotient -- the division's own result --
// for every finite nonzero v (tests/test_capi_host.py checks it against v / d); a zero,
// infinite or NaN v keeps q0, which has the quotient's sign and class there.
__device__ __forceinline__ double div_by(double v, double d, double r) {
  const double q0 = v * r;
  const double q = __builtin_fma(__builtin_fma(-q0, d, v), r, q0);
  return (q0 != 0.0 && __builtin_fabs(q0) < __builtin_huge_val()) ? q : q0;
}

__device__ __forceinline__ double dct_sum(const float* dct, const float* lm, int c, int nc, int nfilt) {
  double v = 0.0;
  for (int n0 = 0; n0 < nfilt; n0 += 8) {
    float dv[8], lv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      dv[u] = dct[c + (n0 + u) * nc];
      lv[u] = lm[n0 + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) v = __builtin_fma((double)dv[u], (double)lv[u], v);
  }
  return v;
}

// 2^y in double for the geometric mean of spectralFlatness.js: 2^floor(y) * 2^frac(y) with
// the f32 hardware exp2 on [0, 1) (relative error ~1.5e-7, against the 1e-5 bar).
__device__ __forceinline__ double exp2_mean(double y) {
  // -inf (a zero amplitude) -> 0, +inf -> inf, NaN -> NaN; v_ldexp_f64 saturates to 0 / inf
  // for any exponent the int conversion holds
  if (!(__builtin_fabs(y) < 1e9)) return y != y ? y : y > 0.0 ? __builtin_huge_val() : 0.0;
  const double n = floor(y);
  return ldexp((double)__builtin_amdgcn_exp2f((float)(y - n)), (int)n);
}

// sqrt(x) from the hardware reciprocal square root and one Newton step (relative error
// ~1e-15) instead of the IEEE square-root sequence; 0, +inf and negative/NaN inputs give
// sqrt's own values (0, inf, NaN).
__device__ __forceinline__ double sqrt_d(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double g = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-h, g, 0.5);
  const double s = __builtin_fma(g, r, g);
  return (x > 0.0 && x < __builtin_huge_val()) ? s : (x == 0.0 || x == __builtin_huge_val()) ? x : __builtin_nan("");
}

// 1/x from the hardware reciprocal and one Newton step (relative error ~1e-16, against the
// 1e-5 bar) instead of the IEEE division sequence; 0, +-inf and NaN keep the raw reciprocal's
// IEEE values (inf, 0, NaN), where the Newton step would turn them into NaN.
__device__ __forceinline__ double rcp_d(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  const double e = __builtin_fma(-x, r, 1.0);
  return __builtin_fabs(e) < 1.0 ? __builtin_fma(r, e, r) : r;
}

// One of the thirteen scalars of a frame from its record (phase 1's sums, phase 2's loudness
// entries), formulas as written in the reference extractors. Every lane evaluates the shared
// terms (moments, spread) and takes its feature's numerator and denominator (the loudness
// quotients joined from a tail of their own: one reciprocal chain per batch instead of three).
template <int N, bool SUB, class Rec>
__device__ __forceinline__ double scalar_value(KArgs* q, const Rec& rc, int sc) {
  constexpr int L = N / 2;
  const double S0 = rc.S[0];
  // utils.js:1-11 mu(p) = sum k^p a_k / sum a_k: one reciprocal and four products (S0 is
  // 0, >= 2^-149 or non-finite, so 1/S0 neither overflows nor hides a NaN of the quotient)
  const double inv = rcp_d(S0);
  const double m1 = rc.S[1] * inv, m2 = rc.S[2] * inv, m3 = rc.S[3] * inv, m4 = rc.S[4] * inv;
  // A feature subset (SUB) forms the square root and the geometric mean only when the request
  // reads S2..S4 / sum log2 a (a wave-uniform branch: C2's centroid alone skips them)
  double sd = 0.0, geo = 0.0;
  if constexpr (SUB) {
    if (q->need_mom > 1) {
      sd = sqrt_d(m2 - m1 * m1);
      geo = exp2_mean(rc.ln2sum * (1.0 / L)) * L;
    }
  } else {
    sd = sqrt_d(m2 - m1 * m1);  // spectralSpread.js
  }
  double num, den = 1.0, k = 1.0;
  // (at thirteen cases the compiler lowers the switch to a branch tree the wave runs case by
  // case; one lane per frame in straight-line code instead measured 0.4-0.6 % slower)
  switch (sc) {
    case MGX_RMS: num = rc.energy * (1.0 / N); break;  // rms.js: sqrt(sum / N), N a power of 2
    case MGX_ENERGY: num = rc.energy; break;           // energy.js
    case MGX_ZCR: num = (double)(rc.zcr & (kChainSkip - 1)); break;  // zcr.js (the CHAIN kernels' flag bit masked)
    case MGX_SPECTRAL_CENTROID: num = m1; break;       // spectralCentroid.js
    case MGX_SPECTRAL_FLATNESS:                        // spectralFlatness.js: geometric / arithmetic mean
      num = SUB ? geo : exp2_mean(rc.ln2sum * (1.0 / L)) * L;
      den = S0;
      break;
    case MGX_SPECTRAL_SLOPE:                           // spectralSlope.js:9-21
      num = L * ((q->sample_rate / N) * rc.S[1]) - q->freq_sum * S0;
      den = S0 * (q->pow_freq_sum - q->freq_sum * q->freq_sum);
      break;
    case MGX_SPECTRAL_ROLLOFF: num = (double)rc.roll_m * q->nyq_bin; break;  // spectralRolloff.js:6-15
    case MGX_SPECTRAL_SPREAD: num = sd; break;
    case MGX_SPECTRAL_SKEWNESS:                        // spectralSkewness.js
      num = 2.0 * m1 * m1 * m1 - 3.0 * m1 * m2 + m3;
      den = sd * sd * sd;
      break;
    case MGX_SPECTRAL_KURTOSIS:                        // spectralKurtosis.js (6 mu1 mu2 as written)
      num = -3.0 * m1 * m1 * m1 * m1 + 6.0 * m1 * m2 - 4.0 * m1 * m3 + m4;
      den = sd * sd * sd * sd;
      break;
    // the loudness total (double, loudness.js:67-69) in band[0], from phase 2's loudness step
    case MGX_LOUDNESS_TOTAL: num = rc.band[0]; break;
    case MGX_PERCEPTUAL_SPREAD:                        // perceptualSpread.js:7-12, squared below
      num = rc.band[0] - (double)__builtin_bit_cast(float, rc.loud_max);
      den = rc.band[0];
      break;
    default:                                           // perceptualSharpness.js:7-14 (0.11 / total)
      num = (double)rc.sharp_sum + q->sharp_tail_sum;
      den = rc.band[0];
      k = 0.11;
      break;
  }
  const double v = num * (k * rcp_d(den));
  return sc == MGX_RMS ? sqrt_d(v) : sc == MGX_PERCEPTUAL_SPREAD ? v * v : v;
}

// The scalar features of one window of a wave's batches (kScalDefer), one lane per frame: lane l
// takes frame l & 3 of the window's batch l >> 2 (nbat batches; frame f0 + (l >> 2) fstep + (l & 3)),
// its ScalIn from the wave's window in device memory (win: word c of lane l at c * 64 + l, phase 2
// put it there), and stores every requested feature -- the formulas of scalar_value, evaluated
// with each feature a constant, so the thirteen share their common terms and nothing diverges.
template <int N, bool SUB, class WinPtr>
__device__ __forceinline__ void scalar_pass(KArgs* q, WinPtr win, void* const* kptr, uint64_t f0, uint64_t fstep, int nbat,
                                            int lane) {
  // the window's words were stored by this wave (phase 2 of each batch): visible to its loads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const auto w = win + (unsigned)lane;
  uint64_t wd[10];
#pragma unroll
  for (int c = 0; c < 10; ++c) wd[c] = w[c * 64];
  ScalIn r;
  __builtin_memcpy(&r, wd, sizeof(r));
  const uint64_t f = f0 + (uint64_t)(lane >> 2) * fstep + (uint64_t)(lane & 3);
  const bool ok = (lane >> 2) < nbat && f < q->num_frames;
  double v[MGX_NUM_SCALARS];
#pragma unroll
  for (int sc = 0; sc < MGX_NUM_SCALARS; ++sc) v[sc] = scalar_value<N, SUB>(q, r, sc);
  const bool f64 = q->scalar_f64;
#pragma unroll
  for (int sc = 0; sc < MGX_NUM_SCALARS; ++sc) {
    // the output pointers from the workgroup's constant table, as wave-uniform values
    const uint64_t pv = reinterpret_cast<const uint64_t*>(kptr)[sc];
    const uint64_t pu = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pv) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pv >> 32)) << 32;
    if (pu == 0) continue;
    if (ok) {
      if (f64) gbl(reinterpret_cast<double*>(pu))[f] = v[sc];
      else gbl(reinterpret_cast<float*>(pu))[f] = (float)v[sc];
    }
  }
}

// mfcc.js:64: Math.log of the batch's band energies (lm[lmo + band] of its FPW records), stored
// to Float32Array; bands past nfilt (up to the DCT table's padded width) become 0. Two bands per
// lane (a pair of adjacent floats: one LDS read and write each): the batch's 4 frames x 32 bands in
// one pass.
template <bool CHAIN, bool SUB>
__device__ __forceinline__ void mfcc_log(KArgs* q, int l2, FrameRec* recs, int lmo) {
  constexpr int FPW = 4;
  const int nfilt = q->nfilt, nfp = (nfilt + 7) & ~7;
  const bool ref_log = CHAIN;  // MGX_FLAG_MFCC_REFERENCE: the double Math.log, then float32
  auto ln1 = [&](float v, int band) {
    return band < nfilt ? (ref_log ? ref_ln(v, gbl(q->t.log_tab)) : ln_f32(v)) : 0.0f;  // padding for dct_sum
  };
  for (int i = l2; i < FPW * (nfp / 2); i += 64) {
    const int fb = i & (FPW - 1), band = 2 * (int)((unsigned)i / FPW);  // (i >= 0: unsigned division)
    f32x2* pp = reinterpret_cast<f32x2*>(&rec_at(recs, fb).lm[lmo + band]);
    const f32x2 v = *pp;
    *pp = f32x2{ln1(v.x, band), ln1(v.y, band + 1)};
  }
}

// mfcc.js:67-93: the DCT of the batch's log energies (lm[lmo + ...] of its FPW records), stored to
// the mfcc rows of frames fbase .. fbase + FPW - 1.
template <bool CHAIN, bool SUB>
__device__ __forceinline__ void mfcc_dct(KArgs* q, int l2, FrameRec* recs, const float* dct_lds, int lmo, uint64_t fbase) {
  constexpr int FPW = 4;
  const int nc = q->ncoef, nfilt = q->nfilt;
  if (q->dct_sequential) {
    // MGX_FLAG_DCT_SEQUENTIAL: VALU FMAs in the reference's sequential order, one lane per (coefficient,
    // frame). The matrix-core form below computes the same sums: v_mfma_f64_4x4x4 adds its four products to
    // the accumulator one FMA after another in k order (tools/ubench/mfma_f64_order.hip: 128,000 of 128,000
    // chained outputs bit-equal to the sequential chain), so a chain of steps over ascending band quartets IS
    // mfcc.js's sequential double sum -- the reference-order MFCC (CHAIN) takes it too.
    for (int i = l2; i < FPW * nc; i += 64) {
      const int c = (int)((unsigned)i / FPW), fb = i & (FPW - 1);
      const uint64_t f = fbase + fb;
      const double v = dct_sum(dct_lds, recs[fb].lm + lmo, c, nc, nfilt);
      if (f < q->num_frames && q->out.mfcc) gbl(q->out.mfcc)[f * nc + c] = (float)div_by(v, nc, q->rcp_ncoef);
    }
    return;
  }
  // mfcc.js:85-93 on the FP64 matrix cores, v_mfma_f64_4x4x4_4b_f64: 4 blocks of a 4 x 4 x 4
  // product per instruction. Block g holds coefficients 4g..4g+3 of a 16-coefficient tile against
  // the batch's 4 frames; a step covers 4 bands. Lane layout (measured,
  // tools/ubench/mfma_f64_4x4_layout.hip): A[i][k] of block g at lane 16k + 4g + i, B[k][j] at
  // 16k + 4g + j, D[i][j] at 16i + 4g + j. So lane l loads DCT[c = l & 15][band n0 + (l >> 4)] and
  // lm[frame l & 3][band n0 + (l >> 4)], and ends with coefficient 4 ((l >> 2) & 3) + (l >> 4) of
  // frame l & 3. The products of two floats are exact in double, and the matrix core adds them in band
  // order (one FMA per k, see above): the reference's sequential sum, bit for bit.
  static_assert(FPW == 4, "one 4 x 4 block column per frame of the batch");
  const int kk = (l2 >> 4) & 3, fa = l2 & 3, nsteps = (nfilt + 3) >> 2;
  const float* lmrow = rec_at(recs, fa).lm + lmo;
  // the batch's mfcc rows from a wave-uniform base (scalar 64-bit arithmetic), lanes at 24-bit offsets
  const auto mrow = q->out.mfcc ? uniform_ptr(gbl(q->out.mfcc) + fbase * (uint64_t)nc) : nullptr;
  for (int mt = 0; mt < nc; mt += 16) {
    // (a tile row past the last coefficient reads the last row again instead of a guarded zero:
    // a row of A only feeds its own coefficient's outputs, never stored)
    const int ca = min(mt + (l2 & 15), nc - 1);
    const float* dcol = dct_lds + ca + __umul24((unsigned)kk, (unsigned)nc);  // row n = 4 st + kk
    double acc = 0.0;
    for (int st = 0; st < nsteps; ++st) {
      const int n = 4 * st + kk;  // < nfilt rounded up to 8: the tables are zero-padded
      const float av = dcol[__umul24((unsigned)(4 * st), (unsigned)nc)];
      acc = __builtin_amdgcn_mfma_f64_4x4x4f64((double)av, (double)lmrow[n], acc, 0, 0, 0);
    }
    const int c = mt + 4 * ((l2 >> 2) & 3) + kk;
    const uint64_t f = fbase + fa;
    if (c < nc && f < q->num_frames && mrow) mrow[__umul24((unsigned)fa, (unsigned)nc) + c] = (float)div_by(acc, nc, q->rcp_ncoef);
  }
}

// Copy of the TwLds image from the plan tables, once per workgroup (before its LDS barrier).
template <int N, int P, int I>
__device__ __forceinline__ void stage_twiddles(double2* twl, GTw tw, GTw twm) {
  if constexpr (P < Geo<N>::NPASS) {
    if constexpr (I < PassGeo<N>::m(P)) {
      using T = TwLds<N>;
      constexpr int mask = (1 << (PassGeo<N>::q0(P) + I)) - 1;
      for (int i = threadIdx.x; i < T::mixed_n(P); i += kThreads)
        twl[T::off(P, I, false) + i] = ld_tw(twm, 2 * mask + i);  // entries mask + la, la < 2^nl
      for (int i = threadIdx.x; i < T::gen_n(P, I); i += kThreads)
        twl[T::off(P, I, true) + i] = ld_tw(tw, mask + (1 << T::nl(P)) + i);
      if (T::pass_lds(P) && threadIdx.x == 0) twl[T::fw_off(P, I)] = ld_tw(twm, 2 * (Geo<N>::L - 1 + PassGeo<N>::q0(P) + I));
      stage_twiddles<N, P, I + 1>(twl, tw, twm);
    } else {
      stage_twiddles<N, P + 1, 0>(twl, tw, twm);
    }
  }
}

// The workgroup's LDS tables (Lds<N>: the bark limits' prefix-row offsets, the tame passes' twiddles,
// the DCT table) written at `base` = the image of LDS byte Lds<N>::kc_off + 128: lds_image_kernel writes
// them once per plan to device memory, and every launch's prologue copies that image into LDS.
template <int N, bool FAITH, bool LITERAL>
__device__ void stage_tables(KArgs* ap, unsigned char* base) {
  using LY = Lds<N>;
  constexpr size_t at = LY::kc_off + 128;
  int* klim = reinterpret_cast<int*>(base);
  // the bark limits as byte offsets of their entries in the padded prefix row (band sums)
  if (threadIdx.x >= 64 && threadIdx.x < 64 + kBark + 1) klim[threadIdx.x - 64] = 8 * pd(gbl(ap->t.bblim)[threadIdx.x - 64]);
  if constexpr (Geo<N>::TW_LDS && FAITH && !LITERAL) {  // the tame passes' twiddles (TwLds)
    stage_twiddles<N, 1, 0>(reinterpret_cast<double2*>(base + (LY::twl_off - at)), gbl(ap->t.tw), gbl(ap->t.twm));
  } else if constexpr (Geo<N>::TW_LDS && !FAITH && !LITERAL) {  // the fast precision's (TwLdsF)
    float2* d = reinterpret_cast<float2*>(base + (LY::twl_off - at));
    const GTwf src = gbl(ap->t.twf);
    for (int i = threadIdx.x; i < TwLdsF<N>::count; i += kThreads) d[i] = ld_twf(src, TwLdsF<N>::first + i);
  }
  const int nt = ap->ncoef * ap->nfilt, ntp = ap->ncoef * ((ap->nfilt + 7) & ~7);
  const auto dct = gbl(ap->t.dct);
  float* dd = reinterpret_cast<float*>(base + (LY::dct_off - at));
  for (int i = threadIdx.x; i < ntp; i += kThreads) dd[i] = i < nt ? dct[i] : 0.0f;
}

template <int N, bool FAITH, bool LITERAL>
__global__ __launch_bounds__(kThreads) void lds_image_kernel(KernelArgs a, unsigned char* image) {
  stage_tables<N, FAITH, LITERAL>(args_ptr(), image);
}

// The completion word of a small host batch (KernelArgs::done_flag): this wave's output stores
// complete and visible to the host (a system-scope release), then one count per wave from lane 0
// (a vector atomic); the wave that makes the count whole resets it for the next launch and
// releases done_seq to the host word. The host, polling that word, reads the outputs without
// waiting for the kernel's completion to reach the runtime (profiles/r04_small_latency.txt).
__device__ __forceinline__ void done_signal(KArgs* q, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (gridDim.x == 1) {
    // one workgroup (a real-time launch of at most 16 frames): its four waves meet at a barrier instead of
    // counting themselves in device memory, and the first releases the word (no atomic round trip)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (threadIdx.x == 0) __hip_atomic_store(q->done_flag, q->done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (lane == 0) {
    const uint32_t before = __hip_atomic_fetch_add(q->done_count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (before + 1 == q->done_waves) {
      __hip_atomic_store(q->done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(q->done_flag, q->done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// MGX_FLAG_RESIDENT: wave 0 of the resident launch reads the whole mailbox (KernelArgs::res_mail) with two
// reads in flight -- the next issued before the oldest is checked; vector loads return in issue order -- so a
// posted frame is taken about one PCIe round trip after it lands (tools/ubench/resident_latency.hip: the
// host's post to its answer 3.1 us at N = 512, against 4.6 with one read at a time and 8.4 for a launch per
// call that reads the same frame). Lane l reads words 64c + l: the frame's samples land as x[c], the
// kernel's own layout.
template <int CH>
__device__ __forceinline__ void res_issue(uint64_t (&w)[CH], const uint64_t* mail, unsigned lane) {
#pragma unroll
  for (int c = 0; c < CH; ++c)
    w[c] = __hip_atomic_load(gbl(mail) + (c * 64 + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// 1: every word carries request seq (its samples into x); -1: word 0 carries the stop word; 0: not yet
template <int CH>
__device__ __forceinline__ int res_take(const uint64_t (&w)[CH], uint32_t seq, float (&x)[CH]) {
  uint32_t bad = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) bad |= (uint32_t)(w[c] >> 32) ^ seq;
  if ((uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(w[0] >> 32)) == kResStop) return -1;
  if (__ballot(bad != 0)) return 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = __uint_as_float((uint32_t)w[c]);
  return 1;
}
// The wait for request seq: true with its frame in x; false on the stop word, or when res_idle ticks of the
// 100 MHz clock pass without it (every launch ends on its own: a host that stops posting leaves no wave
// behind for longer than the idle timeout). light (MGX_RESIDENT_POLL=light): the waiting reads only the first
// word (8 bytes per read, two in flight, instead of the whole frame), then the frame is read until it is
// whole -- one PCIe round trip more per request, for almost no PCIe traffic while waiting.
template <int CH>
__device__ __forceinline__ bool res_wait(const uint64_t* mail, uint32_t seq, uint32_t idle, bool light, float (&x)[CH],
                                         unsigned lane) {
  const unsigned long long t0 = wall_clock64();
  if (light) {
    const auto head = gbl(mail);
    uint64_t h = __hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
      const uint64_t hn = __hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint32_t tag = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(h >> 32));
      if (tag == kResStop) return false;
      if (tag == seq) break;
      h = hn;
      if (wall_clock64() - t0 > idle) return false;
    }
    for (;;) {  // (the host writes the frame in ~0.5 us: a read or two sees it whole)
      uint64_t a[CH];
      res_issue<CH>(a, mail, lane);
      const int r = res_take<CH>(a, seq, x);
      if (r != 0) return r > 0;
      if (wall_clock64() - t0 > idle) return false;
    }
  }
  uint64_t a[CH], b[CH];
  res_issue<CH>(a, mail, lane);
  for (;;) {
    res_issue<CH>(b, mail, lane);
    int r = res_take<CH>(a, seq, x);
    if (r != 0) return r > 0;
    res_issue<CH>(a, mail, lane);
    r = res_take<CH>(b, seq, x);
    if (r != 0) return r > 0;
    if (wall_clock64() - t0 > idle) return false;
  }
}

#if MGX_WAVE_TIMES
// (diagnostic build only, tools/wave_times.py) per wave: start, after the prologue, end (the
// 100 MHz real-time clock) and the CU id / workgroup; and the first wave's phase stamps of its first
// frame (g_stamps[i] at MGX_STAMP(i), tools/small_stamps.py: where a one-frame launch's time goes)
__device__ unsigned long long g_wave_times[65536 * 4];
#endif

template <int N, bool FAITH, bool LITERAL, bool SUB, bool LIGHT, bool NOTIME, bool CHAIN, bool INL = false, bool RES = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(RES ? 1 : Geo<N>::WPE))) void extract_kernel(
    std::conditional_t<INL, KernelArgsInline<N>, KernelArgs> a) {
  using G = Geo<N>;
  using PG = PassGeo<N>;
  using LY = Lds<N>;
  constexpr int R = G::R, CH = G::CH, FPW = G::FPW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* slot_all = reinterpret_cast<float2*>(smem + LY::slot_off);
  float* dct_lds = reinterpret_cast<float*>(smem + LY::dct_off);
  double* mom = G::MOM_SLOT ? nullptr : reinterpret_cast<double*>(smem + LY::mom_off) + (threadIdx.x >> 6) * (5 * G::MOM_STRIDE);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float2* buf = slot_all + wave * G::SLOT_PHYS;
  FrameRec* recs = reinterpret_cast<FrameRec*>(smem + LY::rec_off) + wave * FPW;  // this wave's records
  // CHAIN: the wave's ring of power rows in device memory (2 FPW rows: paired batches, mel_chains)
  float* rows = CHAIN ? uniform_ptr(args_ptr()->chain_rows + ((uint64_t)blockIdx.x * 4 + wave) * (uint64_t)(2 * FPW * G::L))
                      : nullptr;
  KArgs* ap = args_ptr();
#if MGX_WAVE_TIMES
  const unsigned long long wt0 = wall_clock64();
  MGX_STAMP(0);
  MGX_CLOCK_STAMP(13);
#endif
  // The 13 scalar output pointers (per launch) as the first load: its address needs nothing but the kernarg
  // pointer, and issued first its wait (vmcnt, in issue order) holds for no later load
  void* kp = nullptr;
  if (threadIdx.x < MGX_NUM_SCALARS) kp = ap->out.scalars[threadIdx.x];
  // INL (a one-frame launch with its frame in the kernel arguments): the frame's loads next, from the
  // kernarg segment the wave addresses from its start, so they overlap every wait below
  float xn[G::PREFETCH ? CH : 1];
  if constexpr (INL && G::PREFETCH) {
    const GF xin = (GF)uniform_ptr(gbl(inline_frame_ptr()));
#pragma unroll
    for (int c = 0; c < CH; ++c) xn[c] = xin[c * 64 + (unsigned)lane];
  }
  // The kernel arguments the prologue reads, loaded in one burst and waited for together (the empty asm
  // keeps their loads here, ahead of every branch): a one-frame launch (the real-time path) then pays one
  // round trip to the kernarg segment before its table and frame loads issue, not one per dependent step.
  const uint64_t nf = ap->num_frames;
  const uint32_t nr32 = (uint32_t)ap->wg_ranks, nimg = ap->t.lds_image_chunks, grid = gridDim.x;
  const void* const img_p = ap->t.lds_image;
  // (INL: the launch's one frame in the kernarg segment, KernelArgsInline::frame)
  const float* const frames_p = INL ? inline_frame_ptr() : ap->frames;
  const float* const win_p = ap->t.window;
  const int* const klist_p = ap->t.klist;
  // ... with one word of every other 64-byte line of the arguments in the same burst, so the scalar cache
  // holds them all: the fields read later (the feature flags, the output and table pointers, the constants)
  // then hit instead of each costing a round trip of a one-frame launch's serial chain
  static_assert(sizeof(KernelArgs) <= 8 * 64, "the argument lines touched below");
  const auto kw = reinterpret_cast<const __attribute__((address_space(4))) uint32_t*>(ap);
  const uint32_t t2 = kw[32], t3 = kw[48], t4 = kw[64], t5 = kw[80], t6 = kw[96], t7 = kw[(sizeof(KernelArgs) - 4) / 4];
  asm volatile("" ::"s"(nf), "s"(nr32), "s"(nimg), "s"(grid), "s"(img_p), "s"(frames_p), "s"(win_p), "s"(klist_p), "s"(t2),
               "s"(t3), "s"(t4), "s"(t5), "s"(t6), "s"(t7));

  int lp[G::NPASS];
#pragma unroll
  for (int p = 0; p < G::NPASS; ++p) lp[p] = PG::lanepart(p, lane);
  // (the bin list's loads issued here, read after the table staging below)
  int kraw[R];
  {
    const auto klist = gbl(klist_p);
#pragma unroll
    for (int r = 0; r < R; ++r) kraw[r] = klist[lp[G::NPASS - 1] | PG::rpart(G::NPASS - 1, r)];
  }
  const bool dc_lane = lp[G::NPASS - 1] == 0;

  // Every wave works through its own batches of FPW consecutive frames: phase 1 per
  // frame, then phase 2 over the batch, with wave-level synchronisation only.
  const uint64_t nb = (nf + FPW - 1) / FPW;
  // Each workgroup owns one contiguous range of batches, its 4 waves interleaved
  // (wave w takes batches 4k + w), so the 16 frames the waves finish together are
  // consecutive: a workgroup fills whole 64/128-byte lines of every scalar output in its
  // own XCD's L2 instead of sharing each line with a workgroup on another XCD.
  const uint64_t wstride = 4;
  // The shares are not equal at N = 1024: the four workgroups of a CU are dispatched in
  // blockIdx order (rank r = blockIdx / (grid / 4) on every CU), and at equal priority the
  // SIMD's arbiter favours the oldest wave, so with equal shares rank 0 finished at 64 % of
  // the launch and the SIMDs ran 3, 2, then 1 wave for the rest (tools/wave_times.py).
  // Rank r takes a share of its own instead (22 / 18 / 14 / 10 of 64 at N = 1024).
  // (the tail pool: the static shares cover the first ng - pool_groups groups, kPool kernels only)
  constexpr bool kPool = G::PF == 0 && !CHAIN && !INL && !RES;
  const uint64_t ng_all = (nb + 3) / 4;
  const uint64_t pool_groups = kPool ? (uint64_t)args_ptr()->pool_groups : 0;
  const uint64_t ng = ng_all - (pool_groups < ng_all ? pool_groups : ng_all);
  uint64_t g0, g1;
  const uint64_t nr = (uint64_t)nr32;
  // (unequal shares need many groups per workgroup: with a few each, their rounding unbalances
  // more than the ranks' rates do -- C2's 65,536 frames at N = 512 lost 6 %; and N = 256 lost 4 %)
  // (12 groups per workgroup: at 8-11 the rank shares' pair rounding cost more than the ranks'
  // rates gain -- 196,608 frames at N = 512 -5.0 %, 131,072 at 1024 -1.9 % with equal pairs instead;
  // below 8 equal pairs won by 2-16 %, profiles/r04_tuning.txt)
  const bool many = ng >= 12 * (uint64_t)grid;
  // Every boundary between two workgroups' ranges falls on an even group (32 frames): the
  // 4-byte scalar outputs of a workgroup then fill whole 128-byte lines (and the 52-byte MFCC
  // and 96-byte loudness records whole lines too), so no output line is written from two
  // XCDs' L2s. Shares ending on odd groups took WRITE_SIZE to 1.8x the outputs (12x for the
  // time-only set); ev() rounds a boundary down to even, the last range ends at ng.
  auto ev = [](uint64_t g) { return g & ~(uint64_t)1; };
  // [lo, hi) over q workgroups in pairs of groups, the remainder pairs one each to the first
  // workgroups (balanced to one pair; the last pair may be a single group at ng)
  auto split = [&](uint64_t lo, uint64_t hi, uint64_t q, uint64_t i) {
    const uint64_t np = (hi - lo + 1) / 2, base = np / q, rem = np % q;
    const uint64_t a = lo + 2 * (i * base + (i < rem ? i : rem)), b = a + 2 * (base + (i < rem ? 1 : 0));
    g0 = a < hi ? a : hi;
    g1 = b < hi ? b : hi;
  };
  if (N >= 512 && N != 1024 && many && nr >= 2 && nr <= 8 && grid % nr == 0) {
    // other N: rank r's weight 5 (R - 1) - 2 r, from 5:3 for the first rank to the last (round 4: 2:1
    // before; 5:3 measured -1.2 % at N = 2048 and -0.9..-1.7 % at 512, steeper and flatter ones slower)
    const uint64_t q = grid / nr, r = blockIdx.x / q, i = blockIdx.x % q;
    auto cum = [&](uint64_t k) { return k * 5 * (nr - 1) - k * (k - 1); };  // weights 5 (R - 1) - 2 r
    const uint64_t cs = cum(nr);
    split(ev(ng * cum(r) / cs), r + 1 == nr ? ng : ev(ng * cum(r + 1) / cs), q, i);
  } else if (N == 1024 && many && nr == 4 && (grid & 3) == 0) {
    // shares 22 / 18 / 14 / 10 of 64 for ranks 0..3 (linear, 2.2:1; 22 / 17 / 14 / 11 before
    // the pair granularity: a 262,144-frame batch's 17 / 64 is 8.5 pairs per workgroup)
    constexpr uint64_t c1 = 22, c2 = c1 + 18, c3 = c2 + 14, cs = c3 + 10;
    const uint64_t q = grid / 4, r = blockIdx.x / q, i = blockIdx.x % q;
    const uint64_t ca = r == 0 ? 0 : r == 1 ? c1 : r == 2 ? c2 : c3, cb = r == 0 ? c1 : r == 1 ? c2 : r == 2 ? c3 : cs;
    split(ev(ng * ca / cs), r == 3 ? ng : ev(ng * cb / cs), q, i);
  } else if (ng >= 2 * (uint64_t)grid) {
    // equal shares in pairs over every workgroup, with few groups each too: ceil(ng / grid) groups
    // per workgroup left the last workgroups idle -- C2's 65,536 frames at N = 512 (3.2 groups per
    // workgroup) ran 4 busy workgroups of 5 per CU, and 65,536 frames at N = 2048 (5.3) left 85 of
    // 768 idle and some CUs 18 groups against 16: -11 % and -14 % per launch, outputs identical
    split(0, ng, grid, blockIdx.x);
  } else {
    const uint64_t per = (ng + grid - 1) / grid;
    g0 = (uint64_t)blockIdx.x * per;
    g0 = g0 < ng ? g0 : ng;
    g1 = g0 + per < ng ? g0 + per : ng;
  }
  const uint64_t b0 = g0 * 4 + wave, bend = g1 * 4 < nb ? g1 * 4 : nb;
  // Loads are unconditional (the frame index is clamped; results of frames past the end
  // are never stored), so they issue back to back with no branches or waits between them.
  // With G::PREFETCH the next frame of the wave is loaded while this one is processed.
  const bool ntf = args_ptr()->nt_frames != 0;  // (one scalar register for the launch)
  auto frame_ptr = [&](uint64_t b, int j) {
    uint64_t f = b * FPW + j;
    f = f < nf ? f : nf - 1;
    // (wave-uniform, uniform_ptr: the lane's offset is added at each load)
    const float* base = INL ? inline_frame_ptr() : args_ptr()->frames;
    return (GF)uniform_ptr(gbl(base) + f * (uint64_t)N);
  };
  auto load = [&](float (&xv)[CH], uint64_t b, int j) {
    ld_frame<CHAIN>(xv, frame_ptr(b, j), (unsigned)lane, ntf);
  };

  // The workgroup's LDS tables, from the plan's image (lds_image_kernel) in one pass of 16-byte loads,
  // issued before the first frame's: a one-frame launch (the real-time path) waits for one round trip of
  // table loads, behind which its frame's loads are already in flight, instead of a chain of them.
  constexpr int kImgK = 4;  // chunks per thread in the first pass (16 KB: every plan's image at N <= 2048)
  const auto img = gbl(static_cast<const u32x4*>(img_p));
  u32x4* const limg = reinterpret_cast<u32x4*>(smem + LY::kc_off + 128);
  u32x4 iv[kImgK];
#pragma unroll
  for (int k = 0; k < kImgK; ++k) {
    const uint32_t i = (uint32_t)threadIdx.x + k * kThreads;
    iv[k] = img[i < nimg ? i : nimg - 1];
  }
  float wreg[CH];
  constexpr bool kWinReg = G::WIN_REG || RES;
  if constexpr (kWinReg) {
    const GF w = gbl(win_p);
#pragma unroll
    for (int c = 0; c < CH; ++c) wreg[c] = w[c * 64 + lane];
  }
  if constexpr (G::PREFETCH && !INL) {  // (load(xn, b0, 0) with the burst's frame pointer)
    const uint64_t f = b0 * FPW < nf ? b0 * FPW : nf - 1;
    ld_frame<CHAIN>(xn, (GF)uniform_ptr(gbl(frames_p) + f * (uint64_t)N), (unsigned)lane, ntf);
  }
  // the output pointers, then the image's chunks
  if (threadIdx.x < MGX_NUM_SCALARS) reinterpret_cast<void**>(smem + LY::kc_off)[threadIdx.x] = kp;
#pragma unroll
  for (int k = 0; k < kImgK; ++k) {
    const uint32_t i = (uint32_t)threadIdx.x + k * kThreads;
    if (i < nimg) limg[i] = iv[k];
  }
  for (uint32_t i = (uint32_t)threadIdx.x + kImgK * kThreads; i < nimg; i += kThreads) limg[i] = img[i];
  lds_barrier();
#if MGX_WAVE_TIMES
  const unsigned long long wt1 = wall_clock64();
  MGX_STAMP(1);
#endif

  KlTab<N> kl;  // spectrum bin held by each register after the last pass
#pragma unroll
  for (int r = 0; r < R; ++r) kl.set(r, pa(kraw[r]));
  // the band lane's prefix-row offsets pd(lim[b]) | pd(lim[b + 1]) << 16 (G::BLIM_REG)
  uint32_t blim = 0;
  if constexpr (G::BLIM_REG) {
    const int* kl = reinterpret_cast<const int*>(smem + LY::kc_off + 16 * 8);  // 8 pd(lim)
    const int lb = lane < kBark ? lane : 0;
    blim = (uint32_t)(kl[lb] >> 3) | ((uint32_t)(kl[lb + 1] >> 3) << 16);
  }

  MGX_STAMP(2);
  int it = 0;  // the wave's batch count (CHAIN with paired batches: the pair's second when odd)
  // The static batches (stride wstride from b0), then, with a tail pool, batches taken by ticket; a stolen
  // batch does not count in `it` (the scalar windows and pairs follow the static batches only).
  bool stolen = false;
  // RES: the request the resident launch waits for next, and its frame
  uint32_t rseq = RES ? args_ptr()->res_seq : 0;
  float xr[RES ? CH : 1];
  for (uint64_t b = b0;;) {
    if (!stolen && b >= bend) {
      if (!kPool || pool_groups == 0) break;
      if (kScalDefer && args_ptr()->scal_defer && (it & (kScalBatches - 1)) != 0) {
        // the wave's last window of static batches, before its batches from the pool
        KArgs* q = args_ptr();
        const int nbat = it & (kScalBatches - 1), l2 = opaque(lane);
        scalar_pass<N, SUB>(q, uniform_ptr(gbl(q->scal_rows) + ((uint64_t)blockIdx.x * 4 + wave) * (uint64_t)kScalWords),
                            reinterpret_cast<void* const*>(smem + LY::kc_off), (b0 + (uint64_t)(it - nbat) * wstride) * FPW,
                            wstride * FPW, nbat, l2);
        it = (it + kScalBatches) & ~(kScalBatches - 1);  // (the window is flushed: nothing left for the end)
      }
      stolen = true;
    }
    if (stolen) {
      // one ticket per batch (lane 0's vector atomic, the value to every lane); every wave ends on the first
      // ticket past the pool, so a launch hands out exactly pool batches + waves tickets, from 0. The wave that
      // draws the last of them resets the counter: every other ticket of the launch was drawn before it (the
      // counter's order), and no wave draws again, so the next launch on the stream -- or the next replay of
      // a captured one -- starts from 0 with no state kept on the host.
      KArgs* q = args_ptr();
      uint64_t t = 0;
      const uint64_t first = ng * 4, pool = nb - first, last = pool + (uint64_t)grid * 4 - 1;
      if (lane == 0) {
        t = __hip_atomic_fetch_add(gbl(q->pool_ctr), (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == last) __hip_atomic_store(gbl(q->pool_ctr), (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      t = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)t) |
          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(t >> 32)) << 32);
      if (t >= pool) break;
      b = first + t;
    }
    if constexpr (RES) {
      // the resident launch (one frame per request, wave 0; the others have no batch): the next request
      KArgs* q = args_ptr();
      if (!res_wait<CH>(q->res_mail, rseq, q->res_idle, q->res_light != 0, xr, (unsigned)lane)) break;
      MGX_STAMP(0);  // (the diagnostic build: the request's stamps count from here)
      MGX_CLOCK_STAMP(13);
    }
    const uint64_t f0 = b * FPW;
    // ------------------------------------------------------------- phase 1
    for (int j = 0; j < FPW; ++j) {
      const uint64_t f = f0 + j;
      // the last batch's frames past the end: nothing to compute (phase 2 stores nothing for them).
      // A launch of 1-3 frames would otherwise run 4 frames in its one wave (the real-time path's
      // one-frame launch: ~4x its serial time).
      if (f >= nf) break;
      float x[CH];
      GF next = nullptr;
      if constexpr (RES) {
        // (the frame from the mailbox; the mid-frame prefetch reads a valid table instead, ignored)
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = xr[c];
        next = frame_ptr(b, 0);
      } else if constexpr (G::PF == 1) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = xn[c];
        if (j + 1 < FPW) load(xn, b, j + 1);
        else load(xn, b + wstride, 0);
      } else if constexpr (G::PF == 2) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = xn[c];
        next = frame_ptr(j + 1 < FPW ? b : b + wstride, j + 1 < FPW ? j + 1 : 0);
      } else {
        load(x, b, j);
      }
      frame_phase1<N, FAITH, LITERAL, SUB, LIGHT, NOTIME, CHAIN, kWinReg>(args_ptr(), x, j, f, f < nf, lane, lp, kl, dc_lane, buf, mom, recs,
                                      reinterpret_cast<const int*>(smem + LY::kc_off + 16 * 8), xn, next,
                                      reinterpret_cast<const double2*>(smem + LY::twl_off), wreg, blim, rows, it, ntf);
    }
    wave_sync();

    // ------------------------------------------------------------- phase 2
    // Lane ids and the argument pointer are re-derived so that nothing phase 2 needs is
    // hoisted out of the batch loop (it would stay live across the FFT).
    MGX_STAMP(9);
    MGX_MARK(phase2_start);
    prio_hi<4>();
    // CHAIN: the mel chains, then the log and the DCT, every batch -- or with paired batches
    // (chain_pair) every second batch of the wave, for the pair (its first batch's energies in the
    // upper half of lm)
    bool mfcc_now = false;
    if constexpr (CHAIN) {
      KArgs* q = args_ptr();
      mfcc_now = q->need_spectrum && q->need_mfcc && (!q->chain_pair || (it & 1));
      if (mfcc_now) {
        // the rows' stores (every lane's) complete before any lane reads them: the ring is this
        // wave's alone and the CU's L1 is coherent for its own waves (workgroup scope)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (q->chain_pair) mel_chains<N, true>(q, opaque(lane), gbl(rows), recs, buf, true);
        else mel_chains<N, false>(q, opaque(lane), gbl(rows), recs, buf, true);
        wave_sync();  // the band energies are in the records: the log step reads them
      }
    }
    {
      KArgs* q = args_ptr();
      const int l2 = opaque(lane);
      if (!LIGHT && q->need_spectrum && q->need_loudness) {
        // 16 lanes per frame, two bands each (24 bands in lanes 0..11 of the row, 12..15 idle):
        // the four frames of the batch in one pass, a frame's reductions in one DPP row. The
        // lane's pair sum is the reduction tree's first level and the four row steps the rest,
        // so every partial sum is the one the 32-lane layout formed (same results).
        static_assert(FPW * 16 == 64, "one DPP row per frame of the batch");
        const int fb = (l2 >> 4) & 3, pr = l2 & 15;
        const uint64_t f = f0 + fb;
        const bool live = pr < kBark / 2;
        const int b0 = live ? 2 * pr : 0;
        FrameRec& rb = rec_at(recs, fb);
        const double sum0 = rb.band[b0], sum1 = rb.band[b0 + 1];
        // loudness.js:62 Math.pow(sum, 0.23), stored to Float32Array
        float sp0 = pow023(sum0), sp1 = pow023(sum1);
        if (!live) sp0 = sp1 = 0.0f;
        if (live && f < q->num_frames && q->out.loudness_specific)
          *reinterpret_cast<__attribute__((address_space(1))) f32x2*>(uniform_ptr(gbl(q->out.loudness_specific) + f0 * kBark) +
                                                                     __umul24((unsigned)fb, (unsigned)kBark) + b0) = f32x2{sp0, sp1};
        // loudness.js:67-69 total; perceptualSpread.js:7-12 max; perceptualSharpness.js:7-14
        // (off-by-one spec[i+1] for i < 15, then the constant 0.066 e^{0.171 (i+1)} tail).
        // total in double (perceptualSpread's (total - max) cancels); max exact in float32;
        // the sharpness weighted sum in float32 (a plain sum of positive terms).
        double tot = (double)sp0 + (double)sp1;
        // (the max on the float bits: every value is >= +0 or NaN, so unsigned order is float
        // order, and a NaN makes the total NaN either way; one DPP-fused max per step)
        uint32_t mx = max(__builtin_bit_cast(uint32_t, sp0), __builtin_bit_cast(uint32_t, sp1));
        float sh = ((b0 >= 1 && b0 <= 15) ? (float)b0 * sp0 : 0.0f) + ((b0 + 1 <= 15) ? (float)(b0 + 1) * sp1 : 0.0f);
        tot += dpp_d<0xB1>(tot); mx = max(mx, (uint32_t)dpp_i<0xB1>((int)mx)); sh += dpp_f<0xB1>(sh);
        tot += dpp_d<0x4E>(tot); mx = max(mx, (uint32_t)dpp_i<0x4E>((int)mx)); sh += dpp_f<0x4E>(sh);
        tot += dpp_d<0x141>(tot); mx = max(mx, (uint32_t)dpp_i<0x141>((int)mx)); sh += dpp_f<0x141>(sh);
        tot += dpp_d<0x140>(tot); mx = max(mx, (uint32_t)dpp_i<0x140>((int)mx)); sh += dpp_f<0x140>(sh);
        // (every lane of the row holds the frame's sums; the three quotients are formed in the
        // scalar step below, with the others)
        if (pr == 15) {
          rb.band[0] = tot;
          rb.loud_max = mx;
          rb.sharp_sum = sh;
        }
      }
      MGX_MARK(loud2_done);
      if (CHAIN ? mfcc_now : (q->need_spectrum && q->need_mfcc)) {
        mfcc_log<CHAIN, SUB>(q, l2, recs, 0);
        if (CHAIN && q->chain_pair) mfcc_log<CHAIN, SUB>(q, l2, recs, 32);  // the pair's first batch
      }
    }
    wave_sync();
    {
      KArgs* q = args_ptr();
      const int l2 = opaque(lane);
      MGX_MARK(ln_done);
      if (CHAIN ? mfcc_now : (q->need_spectrum && q->need_mfcc)) {
        mfcc_dct<CHAIN, SUB>(q, l2, recs, dct_lds, 0, f0);
        if (CHAIN && q->chain_pair) mfcc_dct<CHAIN, SUB>(q, l2, recs, dct_lds, 32, f0 - wstride * FPW);  // the pair's first batch
      }
      MGX_MARK(dct_done);
      const bool defer = kScalDefer && q->scal_defer && !stolen;
      if (defer) {
        // the batch's scalar inputs into the wave's window (10 words per frame, lanes 0..39: frame
        // l2 / 10, word l2 % 10), the scalars of the window once it is full (scalar_pass)
        const auto win = uniform_ptr(gbl(q->scal_rows) + ((uint64_t)blockIdx.x * 4 + wave) * (uint64_t)kScalWords);
        const int slot = it & (kScalBatches - 1);
        if (l2 < 10 * FPW) {
          const int fb = (int)(__umul24((unsigned)l2, 205u) >> 11);  // l2 / 10 for l2 < 40
          const int c = l2 - 10 * fb;
          const unsigned off = 8u * (unsigned)c + (c >= 8 ? 440u : 0u);  // words 0..7, then 63..64
          const uint64_t wv = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const unsigned char*>(&rec_at(recs, fb)) + off);
          win[__umul24((unsigned)c, 64u) + (unsigned)(4 * slot + fb)] = wv;
        }
      }
      // the scalar features: one lane per (feature, frame); the loudness total, perceptual
      // spread and sharpness from the loudness step's record entries (16 x 4 lanes at most)
      for (int i = l2; !defer && i < (MGX_PERCEPTUAL_SHARPNESS + 1) * FPW; i += 64) {
        const int sc = (int)((unsigned)i / FPW), fb = i & (FPW - 1);
        const uint64_t f = f0 + fb;
        void* dst = reinterpret_cast<void* const*>(smem + LY::kc_off)[sc];
        if (f >= q->num_frames || dst == nullptr) continue;
        const double v = scalar_value<N, SUB>(q, rec_at(recs, fb), sc);
        if (q->scalar_f64) gbl(static_cast<double*>(dst))[f] = v;
        else gbl(static_cast<float*>(dst))[f] = (float)v;
      }
    }
    prio_lo<4>();
    MGX_MARK(phase2_end);
    MGX_STAMP(10);
    wave_sync();  // records and slot buffer are reused by the next batch
    // The workgroup's four waves meet after every second group of 16 frames (G::GROUP_SYNC).
    // Left alone they drift apart by more than the L2's turnover time, so each wave's 16-byte piece
    // of a 64-byte scalar line was written back on its own: WRITE_SIZE 1.13x the outputs (time-only
    // set 1.40x). With the barrier: 1.016x (1.10x), all-feature launch +0.0 %, time-only -3.8 %,
    // outputs identical (profiles/r03_group_sync.txt). Every wave has a batch in a full group, so
    // all four reach the same barriers. N = 512 and 2048 lost 1.6 % and 2.3 % and keep none.
    if constexpr (G::GROUP_SYNC > 0) {
      const uint64_t g = (b - wave) / 4;
      if (!stolen && g * 4 + 3 < nb && g % G::GROUP_SYNC == G::GROUP_SYNC - 1) __builtin_amdgcn_s_barrier();
    }
    // A full scalar window: its pass right after the group barrier (a window ends on an odd group,
    // where the barrier is), so the workgroup's four waves write their 16-byte pieces of each
    // scalar output line together and the L2 merges them, as the per-batch form's writes.
    if (kScalDefer && !stolen && (it & (kScalBatches - 1)) == kScalBatches - 1) {
      KArgs* q = args_ptr();
      if (q->scal_defer) {
        prio_hi<4>();
        scalar_pass<N, SUB>(q, uniform_ptr(gbl(q->scal_rows) + ((uint64_t)blockIdx.x * 4 + wave) * (uint64_t)kScalWords),
                            reinterpret_cast<void* const*>(smem + LY::kc_off),
                            (b - (uint64_t)(kScalBatches - 1) * wstride) * FPW, wstride * FPW, kScalBatches, opaque(lane));
        prio_lo<4>();
      }
    }
    if constexpr (RES) {
      // the request answered: its number released to the completion word after the outputs (the launch does
      // not end, so its plain stores would otherwise stay in the L2: the host cannot wait on the output words)
      KArgs* q = args_ptr();
      MGX_STAMP(11);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      if (lane == 0) __hip_atomic_store(q->done_flag, rseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      MGX_STAMP(12);
      MGX_CLOCK_STAMP(14);
      ++rseq;
      continue;
    }
    if (!stolen) {
      b += wstride;
      ++it;
    }
  }
  if (kScalDefer && args_ptr()->scal_defer && (it & (kScalBatches - 1)) != 0) {
    // the wave's last window, with fewer than kScalBatches batches
    KArgs* q = args_ptr();
    const int nbat = it & (kScalBatches - 1), l2 = opaque(lane);
    prio_hi<4>();
    scalar_pass<N, SUB>(q, uniform_ptr(gbl(q->scal_rows) + ((uint64_t)blockIdx.x * 4 + wave) * (uint64_t)kScalWords),
                        reinterpret_cast<void* const*>(smem + LY::kc_off), (b0 + (uint64_t)(it - nbat) * wstride) * FPW,
                        wstride * FPW, nbat, l2);
    prio_lo<4>();
  }
  if constexpr (CHAIN) {
    // paired batches: a wave whose last batch opened a pair finishes that batch's mfcc alone
    KArgs* q = args_ptr();
    if (q->need_spectrum && q->need_mfcc && q->chain_pair && (it & 1)) {
      prio_hi<4>();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const int l2 = opaque(lane);
      mel_chains<N, true>(q, l2, gbl(rows), recs, buf, false);
      wave_sync();
      mfcc_log<CHAIN, SUB>(q, l2, recs, 32);
      wave_sync();
      mfcc_dct<CHAIN, SUB>(q, l2, recs, dct_lds, 32, (b0 + (uint64_t)(it - 1) * wstride) * FPW);
      prio_lo<4>();
    }
  }
  MGX_STAMP(11);
  if constexpr (RES) {
    // the resident launch ends (stop word or idle): wave 0 tells the host, after its last outputs
    if (wave == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      if (lane == 0) __hip_atomic_store(args_ptr()->res_exit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  } else if (args_ptr()->done_flag) {
    done_signal(args_ptr(), opaque(lane));
  }
  MGX_STAMP(12);
  MGX_CLOCK_STAMP(14);
#if MGX_WAVE_TIMES
  if (lane == 0 && blockIdx.x < 16384) {
    auto g = (__attribute__((address_space(1))) unsigned long long*)g_wave_times + ((uint64_t)blockIdx.x * 4 + wave) * 4;
    g[0] = wt0;
    g[1] = wt1;
    g[2] = wall_clock64();
    g[3] = __smid() | ((uint64_t)blockIdx.x << 32);
  }
#endif
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

// PCM -> float32 of one channel, decodeAudioData's scaling (include/meyda_gpu.h).
__global__ void pcm_decode_kernel(const unsigned char* __restrict__ pcm, uint64_t count, uint32_t format,
                                  uint32_t stride, uint32_t offset, float* __restrict__ out) {
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += step) {
    // samples are assembled from bytes: a caller's device pointer need not be aligned
    const unsigned char* b = pcm + i * stride + offset;
    auto w32 = [b]() { return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24; };
    float v;
    switch (format) {
      case MGX_PCM_S16: v = (float)(int16_t)(uint16_t)((uint32_t)b[0] | (uint32_t)b[1] << 8) * (1.0f / 32768.0f); break;
      case MGX_PCM_U8: v = (float)((int)b[0] - 128) * (1.0f / 128.0f); break;
      case MGX_PCM_S24: {
        const int32_t u = (int32_t)((uint32_t)b[0] << 8 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 24) >> 8;
        v = (float)u * (1.0f / 8388608.0f);
        break;
      }
      case MGX_PCM_S32: v = (float)((double)(int32_t)w32() * (1.0 / 2147483648.0)); break;
      default: v = __builtin_bit_cast(float, w32()); break;
    }
    out[i] = v;
  }
}

// Packed transfer buffer -> the root's structure-of-arrays outputs (group.cpp). One
// workgroup row per segment (blockIdx.y); dword copies: every field is a whole number of
// dwords per frame, and a shard's destination offset is only dword-aligned.
__global__ void unpack_kernel(UnpackArgs a) {
  const int s = blockIdx.y;
  if (s >= a.nseg) return;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(a.src + a.src_off[s]);
  uint32_t* dst = static_cast<uint32_t*>(a.dst[s]);
  const uint64_t n = a.dwords[s];
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

template <int N, bool FAITH, bool LITERAL, bool SUB = false, bool LIGHT = false, bool NOTIME = false, bool CHAIN = false>
hipError_t launch_n(const KernelArgs& a, int grid, hipStream_t stream, const float* inl = nullptr, bool res = false) {
  const size_t lds = Lds<N>::bytes(a.ncoef, a.nfilt);
  if constexpr (FAITH && !LITERAL && !CHAIN) {
    if (res) {  // MGX_FLAG_RESIDENT: the one-workgroup server of one-frame requests
      hipLaunchKernelGGL((extract_kernel<N, FAITH, LITERAL, SUB, LIGHT, NOTIME, CHAIN, false, true>), dim3(1), dim3(kThreads), lds,
                         stream, a);
      return hipGetLastError();
    }
  }
  if constexpr (N <= kInlineMaxN && FAITH && !LITERAL && !CHAIN) {
    if (inl) {  // the one frame in the kernel arguments (KernelArgsInline<N>)
      KernelArgsInline<N> x;
      x.a = a;
      memcpy(x.frame, inl, N * sizeof(float));
      hipLaunchKernelGGL((extract_kernel<N, FAITH, LITERAL, SUB, LIGHT, NOTIME, CHAIN, true>), dim3(grid), dim3(kThreads), lds,
                         stream, x);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((extract_kernel<N, FAITH, LITERAL, SUB, LIGHT, NOTIME, CHAIN>), dim3(grid), dim3(kThreads), lds, stream, a);
  return hipGetLastError();
}

template <int N, bool FAITH, bool LITERAL, bool SUB = false, bool LIGHT = false, bool NOTIME = false, bool CHAIN = false>
int occupancy_n(int ncoef, int nfilt) {
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, extract_kernel<N, FAITH, LITERAL, SUB, LIGHT, NOTIME, CHAIN>, kThreads,
                                                   Lds<N>::bytes(ncoef, nfilt)) != hipSuccess)
    return 0;
  return blocks;
}

// the instances a plan's launches use: MGX_FLAG_MFCC_REFERENCE takes the CHAIN pair
// (all features / any subset), every other faithful plan the four below
template <int N>
constexpr bool kChainN = N <= kChainMaxN;

template <int N>
int occupancy_prec(int precision, int mode, int ncoef, int nfilt, bool chain) {
  if (mode == MGX_MODE_LITERAL) return occupancy_n<N, true, true>(ncoef, nfilt);
  if (precision == MGX_PRECISION_FAST) return occupancy_n<N, false, false>(ncoef, nfilt);
  if constexpr (kChainN<N>) {
    if (chain) {
      const int m = occupancy_n<N, true, false, false, false, false, true>(ncoef, nfilt),
                o = occupancy_n<N, true, false, true, false, false, true>(ncoef, nfilt);
      return o < m ? o : m;
    }
  }
  // the grid serves the four faithful kernels (all features / without the time-domain ones /
  // a subset / a light subset)
  int m = occupancy_n<N, true, false>(ncoef, nfilt);
  for (int o : {occupancy_n<N, true, false, false, false, true>(ncoef, nfilt), occupancy_n<N, true, false, true>(ncoef, nfilt),
                occupancy_n<N, true, false, true, true>(ncoef, nfilt)})
    m = o < m ? o : m;
  return m;
}

template <int N>
hipError_t launch_prec(int precision, int mode, const KernelArgs& a, int grid, hipStream_t stream, const float* inl, bool res) {
  if (mode == MGX_MODE_LITERAL) return launch_n<N, true, true>(a, grid, stream);
  if (precision == MGX_PRECISION_FAST) return launch_n<N, false, false>(a, grid, stream);
  const bool every = a.need_mom == 2 && a.need_prefix && a.need_energy && a.need_zcr;
  if constexpr (kChainN<N>) {
    // MGX_FLAG_MFCC_REFERENCE: the mel sums as chains in the reference's order (mel_chains)
    if (a.chain_groups > 0 && a.need_spectrum && a.need_mfcc) {
      if (every) return launch_n<N, true, false, false, false, false, true>(a, grid, stream);
      return launch_n<N, true, false, true, false, false, true>(a, grid, stream);
    }
  }
  // a spectral feature subset that skips the moment / prefix / time-domain work takes the SUB kernel
  // (LIGHT: a subset reading neither the moments nor the prefix row, e.g. mfcc or the spectra
  // alone, compiled without that code: no runtime branches to keep its registers live)
  if (a.need_spectrum && a.need_mom == 0 && !a.need_prefix)
    return launch_n<N, true, false, true, true>(a, grid, stream, inl, res);
  // (NOTIME: every spectral sum but no rms / energy / zcr, e.g. C3: the all-feature schedule
  // with the time-domain reductions compiled out)
  if (a.need_spectrum && a.need_mom == 2 && a.need_prefix && !a.need_energy && !a.need_zcr)
    return launch_n<N, true, false, false, false, true>(a, grid, stream, inl, res);
  if (a.need_spectrum && !every)
    return launch_n<N, true, false, true>(a, grid, stream, inl, res);
  return launch_n<N, true, false>(a, grid, stream, inl, res);
}

template <int N>
size_t lds_image_bytes_n(int ncoef, int nfilt) {
  return (Lds<N>::bytes(ncoef, nfilt) - (Lds<N>::kc_off + 128) + 15) / 16 * 16;
}

template <int N>
hipError_t launch_image_n(int precision, int mode, const KernelArgs& a, void* image, hipStream_t stream) {
  auto* im = static_cast<unsigned char*>(image);
  if (mode == MGX_MODE_LITERAL) hipLaunchKernelGGL((lds_image_kernel<N, true, true>), dim3(1), dim3(kThreads), 0, stream, a, im);
  else if (precision == MGX_PRECISION_FAST) hipLaunchKernelGGL((lds_image_kernel<N, false, false>), dim3(1), dim3(kThreads), 0, stream, a, im);
  else hipLaunchKernelGGL((lds_image_kernel<N, true, false>), dim3(1), dim3(kThreads), 0, stream, a, im);
  return hipGetLastError();
}

}  // namespace

size_t lds_image_bytes(int n, int ncoef, int nfilt) {
  switch (n) {
    case 256: return lds_image_bytes_n<256>(ncoef, nfilt);
    case 512: return lds_image_bytes_n<512>(ncoef, nfilt);
    case 1024: return lds_image_bytes_n<1024>(ncoef, nfilt);
    case 2048: return lds_image_bytes_n<2048>(ncoef, nfilt);
    default: return 0;
  }
}

hipError_t launch_lds_image(int n, int precision, int mode, const KernelArgs& a, void* image, hipStream_t stream) {
  switch (n) {
    case 256: return launch_image_n<256>(precision, mode, a, image, stream);
    case 512: return launch_image_n<512>(precision, mode, a, image, stream);
    case 1024: return launch_image_n<1024>(precision, mode, a, image, stream);
    case 2048: return launch_image_n<2048>(precision, mode, a, image, stream);
    default: return hipErrorInvalidValue;
  }
}

size_t extract_lds_bytes(int n, int ncoef, int nfilt, bool chain) {
  switch (n) {
    case 256: return Lds<256>::bytes(ncoef, nfilt);
    case 512: return Lds<512>::bytes(ncoef, nfilt);
    case 1024: return Lds<1024>::bytes(ncoef, nfilt);
    case 2048: return Lds<2048>::bytes(ncoef, nfilt);
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

int extract_blocks_per_cu(int n, int precision, int mode, int ncoef, int nfilt, bool chain) {
  switch (n) {
    case 256: return occupancy_prec<256>(precision, mode, ncoef, nfilt, chain);
    case 512: return occupancy_prec<512>(precision, mode, ncoef, nfilt, chain);
    case 1024: return occupancy_prec<1024>(precision, mode, ncoef, nfilt, chain);
    case 2048: return occupancy_prec<2048>(precision, mode, ncoef, nfilt, false);
    default: return 0;
  }
}

hipError_t launch_extract(int n, int precision, int mode, const KernelArgs& a, int grid,
                          hipStream_t stream, const float* inline_frame, bool resident) {
  if (a.num_frames != 1) inline_frame = nullptr;
  if (resident && (a.num_frames != 1 || grid != 1 || a.res_mail == nullptr || a.res_exit == nullptr ||
                   a.done_flag == nullptr))
    return hipErrorInvalidValue;
  switch (n) {
    case 256: return launch_prec<256>(precision, mode, a, grid, stream, inline_frame, resident);
    case 512: return launch_prec<512>(precision, mode, a, grid, stream, inline_frame, resident);
    case 1024: return launch_prec<1024>(precision, mode, a, grid, stream, inline_frame, resident);
    case 2048: return launch_prec<2048>(precision, mode, a, grid, stream, nullptr, resident);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_pcm_decode(const void* pcm, uint64_t count, uint32_t format, uint32_t channels,
                             uint32_t channel, float* out, hipStream_t stream) {
  const uint32_t bps = format == MGX_PCM_S16 ? 2 : format == MGX_PCM_U8 ? 1 : format == MGX_PCM_S24 ? 3 : 4;
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(pcm_decode_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     static_cast<const unsigned char*>(pcm), count, format, bps * channels, bps * channel, out);
  return hipGetLastError();
}

hipError_t launch_unpack(const UnpackArgs& a, hipStream_t stream) {
  uint64_t most = 0;
  for (int i = 0; i < a.nseg; ++i) most = a.dwords[i] > most ? a.dwords[i] : most;
  if (a.nseg == 0 || most == 0) return hipSuccess;
  uint64_t bx = (most + 1023) / 1024;
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)bx, (unsigned)a.nseg), dim3(256), 0, stream, a);
  return hipGetLastError();
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

#if MGX_WAVE_TIMES
extern "C" int mgx_debug_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mgx::g_stamps), 16 * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int mgx_debug_wave_times(unsigned long long* host, int count) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mgx::g_wave_times), (size_t)count * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
