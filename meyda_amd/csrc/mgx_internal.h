// Internal definitions shared by the host plan code and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/meyda_gpu.h"

namespace mgx {

constexpr int kMaxMel = 64;
// The scalar features run once per window of kScalBatches batches of a wave (kernels.hip
// scalar_pass), one lane per frame: the window's per-frame inputs (10 8-byte words each, the
// record's S[0..4], ln2sum, energy, loudness total, zcr | roll_m, loud_max | sharp_sum) wait in
// device memory, kScalWords words per wave.
// (a constant: the round-4 override macro built window lengths that no test covered)
constexpr int kScalBatches = 16;
// word c of the window's frame l (l = 4 batch + frame, < 4 kScalBatches) at c * 64 + l
static_assert(4 * kScalBatches <= 64, "a window's frames are lanes of one wave");
constexpr int kScalWords = 10 * 64;
constexpr int kBark = 24;
constexpr int kMaxCoeffs = 32;
constexpr int kThreads = 256;  // 4 waves per workgroup
// Mel band chains in the reference's own order (MGX_FLAG_MFCC_REFERENCE, every N): F frames x
// nfilt chains on 64 / F packed tracks (F = 8 for nfilt <= 31, else F = 4; plan.cpp chain_schedule).
constexpr int kRecBytes = 520;  // sizeof(FrameRec) (kernels.hip)
constexpr int kRecLmOff = 248;  // offsetof(FrameRec, lm)
constexpr int kChainPairMaxMel = 31;  // paired batches keep two halves of FrameRec::lm (flag at 31)
constexpr int kChainMaxN = 2048;
constexpr int kChainSkip = 1 << 30;  // FrameRec.zcr flag bit: a non-finite frame keeps its phase-1 mel sums
// dwords of one lane's mel record for R bins per lane (R weights, R slot bytes, R keep bytes,
// 8 bytes of scan keeps and slots), padded to whole 16-byte loads
// The lane's mel record (plan.cpp mel_lane_tables): the bin weights -- (rise, 1 - rise) pairs
// up to R = 8 slots per lane, the rising weight alone above --, the keep bytes, the scan keeps
// (2 words) and the four assembly offsets (2 words).
__host__ __device__ constexpr int mel_weight_words(int R) { return R <= 8 ? 2 * R : R; }
__host__ __device__ constexpr int mel_rec_words(int R) { return (mel_weight_words(R) + (R + 3) / 4 + 4 + 3) / 4 * 4; }
// Device-resident, read-only tables of a plan (one allocation, see plan.cpp).
struct DevTables {
  const float* window;       // N, the selected window (src/meyda.js:116-138)
  const double2* tw;         // N/2 - 1 faithful twiddles, stage q at offset 2^q - 1
  const float2* twf;         // same, float32 (MGX_PRECISION_FAST)
  const double2* twm;        // like tw, two per entry: (b, c0), (t4, kL) of the mixed butterflies (plan.cpp mixed_coeffs)
  const int* klist;          // N/2: slot location -> spectrum bin
  const int* bblim;          // 25 bark band limits (loudness.js:24-45)
  const uint32_t* mel_rec;   // 64 per-lane records of the mel segment tables (plan.cpp mel_lane_tables)
  const int* mel_bins;       // nfilt + 2 filter edges (mfcc.js:15-38), for the non-finite-frame path
  const float* dct;          // ncoef * nfilt, dct[c + j*ncoef] (mfcc.js:67-83)
  // MGX_FLAG_MFCC_REFERENCE (plan.cpp chain_schedule, kernels.hip mel_chains):
  const uint32_t* chain_ctl; // per 8-step group and lane: row offset, chain start, the finished chain's store
  const double* chain_w;     // per track, the weights of its chains' steps back to back
  const double2* log_tab;    // 64 x (1/c_k, -ln(1/c_k)), c_k = 1 + (2k + 1)/128: the reference-order MFCC's ln (kernels.hip ref_ln)
  // The workgroup's LDS tables as one image (kernels.hip lds_image_kernel, built once per plan): the bark
  // limits' prefix-row offsets, the staged twiddles and the DCT table, byte for byte as they sit in LDS
  // from Lds<N>::kc_off + 128 on; each launch's prologue copies it in one pass of 16-byte loads.
  const void* lds_image;
  uint32_t lds_image_chunks; // 16-byte chunks of the image
};

struct KernelArgs {
  const float* frames;
  uint64_t num_frames;
  DevTables t;
  mgx_outputs out;
  double sample_rate;
  double freq_sum;       // spectralSlope.js: sum of i*sr/N, i < N/2 (input independent)
  double pow_freq_sum;   // spectralSlope.js: sum of (i*sr/N)^2
  double nyq_bin;        // spectralRolloff.js:4: sr / (2 (N/2 - 1))
  double sharp_tail_sum; // perceptualSharpness.js:10: sum_{i=15}^{23} 0.066 e^{0.171 (i+1)}
  double rcp_ncoef;      // 1 / ncoef, correctly rounded: the DCT's scale as Markstein quotients (div_by)
  int nfilt;
  int ncoef;
  int scalar_f64;
  int need_spectrum;     // any spectral output requested
  int need_loudness;     // loudness / perceptual outputs requested
  int need_mfcc;
  int need_mom;          // 2: flatness / spread / skewness / kurtosis (S1..S4, sum log2 a); 1: centroid / slope (S1); 0
  int need_prefix;       // rolloff or loudness: the prefix row (rolloff count, bark band sums)
  int need_energy;       // rms or energy: the wave sum of the squares (SUB kernel)
  int need_zcr;          // zcr: the sign-change ballots (SUB kernel)
  int scal_defer;        // the scalars by windows (scalar_pass): a spectrum is computed and a scalar requested
  int nt_frames;         // the frames read with non-temporal loads: the batch is larger than the MALL (kernels.hip ld_frame)
  // Small host batches (plan.cpp extract_host_small): every wave counts itself in done_count at
  // its end, after its output stores are visible to the host, and the last one sets the mapped
  // host word done_flag to done_seq, which the host polls instead of synchronising the stream.
  uint32_t* done_flag;   // null: no completion word
  uint32_t* done_count;  // device memory, 0 between launches (the last wave resets it)
  uint32_t done_seq;
  uint32_t done_waves;   // waves in the grid
  int dct_sequential;    // MGX_FLAG_DCT_SEQUENTIAL: the DCT as VALU FMAs in the reference's order
  int wg_ranks;          // workgroups per CU when the grid is the resident one (else 1): their work shares
  int chain_groups;      // 8-step groups of the mel chain tracks (0: the segmented scan)
  int chain_pair;        // the chains of two consecutive batches of a wave run together (8 frames, nfilt <= 31)
  float* chain_rows;     // the chains' power rows: 2 FPW x N/2 floats per wave of the grid (kernels.hip mel_chains)
  uint64_t* scal_rows;   // the scalar window: kScalWords 8-byte words per wave of the grid (kernels.hip scalar_pass)
  // The tail pool (kernels without a frame prefetch, i.e. N = 2048; 0 groups = off): the last pool_groups
  // groups of 4 batches are left out of the static shares and taken one batch per ticket by the waves
  // that finish their share first. pool_ctr is the launching stream's ticket counter: 0 when a launch starts,
  // and reset to 0 on the device by the wave that draws the launch's last ticket (kernels.hip), so a launch
  // captured into a graph replays with no host state.
  uint64_t* pool_ctr;
  uint32_t pool_groups;
  // MGX_FLAG_RESIDENT (plan.cpp resident_*): a one-workgroup launch that stays on the device and serves
  // one-frame requests from a mailbox in mapped host memory, until the host's stop word or res_idle ticks
  // of the 100 MHz clock without a request. res_mail: N words, (float32 sample bits) | request << 32, each
  // written by the host with one 8-byte store and read with one 8-byte system-scope load, so a frame is
  // complete when every word carries the request's number; word 0 carrying kResStop ends the launch.
  // After each request's outputs the launch releases its number to done_flag (a launch that does not end
  // leaves plain stores in the L2 until a release writes them back). res_exit: the host word the launch
  // sets to 1 as it ends.
  const uint64_t* res_mail;
  uint32_t* res_exit;
  uint32_t res_seq;      // the first request number the launch serves
  uint32_t res_idle;     // idle timeout, ticks of the 100 MHz real-time clock
  uint32_t res_light;    // poll the mailbox's first word only, then read the frame (MGX_RESIDENT_POLL=light)
};
constexpr uint32_t kResStop = 0xFFFFFFFFu;  // a request number that stops the resident launch

// A one-frame launch at N <= kInlineMaxN (the real-time path: extract_host_small with one frame) carries
// its frame in the kernel arguments, after the KernelArgs: the kernel's first loads read it from the
// kernarg segment, whose address the wave holds from its first instruction, instead of waiting for the
// arguments before it can issue the frame's read of pinned host memory over PCIe.
constexpr int kInlineMaxN = 1024;  // (4,528 bytes of arguments at N = 1024: tools/ubench/kernarg_size.hip runs 4.8 KB)
template <int N>
struct KernelArgsInline {
  KernelArgs a;
  alignas(16) float frame[N];
};
// (the frame's offset in the kernel arguments, the same for every N)
constexpr size_t kInlineFrameOff = (sizeof(KernelArgs) + 15) / 16 * 16;
static_assert(offsetof(KernelArgsInline<256>, frame) == kInlineFrameOff && offsetof(KernelArgsInline<2048>, frame) == kInlineFrameOff,
              "inline frame offset");

// Last-error reporting (plan.cpp): set mgx_last_error() and return `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_fail(hipError_t e, const char* what);

// Launchers (kernels.hip).
// inline_frame (host memory, N floats): a one-frame launch at N <= kInlineMaxN passes its frame in the
// kernel arguments (KernelArgsInline) when a faithful per-buffer kernel without the reference-order
// chains runs it; a.frames is then not read. Otherwise ignored.
// resident (MGX_FLAG_RESIDENT, one frame, grid 1, a.res_* set): the launch stays on the
// device serving requests from a.res_mail until the stop word or the idle timeout (kernels.hip res_wait);
// the literal, fast and reference-order plans have no resident form (an error).
hipError_t launch_extract(int n, int precision, int mode, const KernelArgs& a, int grid,
                          hipStream_t stream, const float* inline_frame = nullptr, bool resident = false);
hipError_t launch_synth(float* out, uint64_t count, uint64_t seed, uint64_t first_index,
                        hipStream_t stream);
hipError_t launch_pcm_decode(const void* pcm, uint64_t count, uint32_t format, uint32_t channels,
                             uint32_t channel, float* out, hipStream_t stream);
// Scatter of one packed transfer buffer into the root's outputs (group.cpp): segment i
// copies dwords[i] dwords from src + src_off[i] to dst[i].
constexpr int kMaxSegs = 19;
struct UnpackArgs {
  const unsigned char* src;
  uint64_t src_off[kMaxSegs];
  void* dst[kMaxSegs];
  uint64_t dwords[kMaxSegs];
  int nseg;
};
hipError_t launch_unpack(const UnpackArgs& a, hipStream_t stream);
size_t extract_lds_bytes(int n, int ncoef, int nfilt, bool chain);
size_t lds_image_bytes(int n, int ncoef, int nfilt);  // DevTables::lds_image, a multiple of 16
hipError_t launch_lds_image(int n, int precision, int mode, const KernelArgs& a, void* image, hipStream_t stream);
int frames_per_batch(int n);
int extract_blocks_per_cu(int n, int precision, int mode, int ncoef, int nfilt, bool chain);  // resident workgroups per CU

}  // namespace mgx
