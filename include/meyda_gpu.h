/*
 * meyda_gpu.h — C ABI of the MI355X (gfx950) meyda feature-extraction engine.
 *
 * This is the drop-in boundary for the reference's per-buffer hot path. In the
 * reference (kirbysayshi/meyda), one call of the path is:
 *
 *   src/meyda.js:69-91    onaudioprocess: window -> (FFT) -> amplitude spectrum
 *   src/meyda.js:244-261  Meyda.get(feature | features[]) -> extractor modules
 *   src/extractors/NAME.js  the 18 extractor plugins, signature (bufferSize, m)
 *
 * The engine batches that path: many frames of `buffer_size` Float32 samples are
 * processed by one fused HIP launch. A host binding (the N-API addon under
 * meyda_amd/addon/, or ctypes) maps Meyda's get()/start()/stop() onto it.
 *
 * Entry points and the reference interface each one replaces:
 *   mgx_plan_create      new Meyda(audioContext, src, bufferSize)   src/meyda.js:17-97
 *                        (power-of-two check src/meyda.js:20-22, tables :44-48,
 *                         extractor init :208-225)
 *   mgx_extract_device   onaudioprocess + get(features)             src/meyda.js:69-91,244-261
 *   mgx_extract_host     same, for host (pageable) buffers
 *   mgx_wav_parse,       decodeAudioData + getChannelData(0)        lib/bufferLoader.js:23,
 *   mgx_pcm_decode_device,                                          src/meyda.js:72
 *   mgx_extract_host_pcm
 *   mgx_group_*          several devices, RCCL gather of the        src/meyda.js:17-97 (one plan
 *                        per-frame records to the root device       per device), :69-91 (buffers
 *                                                                   are independent: shardable)
 *   mgx_feature_index    the extractor registry by name             src/extractors/index.js:1-20
 *   mgx_feature_info     featureInfo[name].type                     src/feature-info.js:1-65
 *   mgx_last_error       console.error / thrown Error text          src/meyda.js:20-26,249-253
 *
 * Conventions: every function returns an int status (MGX_OK = 0, negative =
 * MGX_E_*); the message of the last failure on the calling thread is returned
 * by mgx_last_error(). Plans are not thread-safe; distinct plans are
 * independent. No torch or HIP types appear in these signatures: streams are
 * passed as `void*` (a hipStream_t, or NULL for the default stream).
 */
#ifndef MEYDA_GPU_H
#define MEYDA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGX_ABI_VERSION 2  /* 2: mgx_extract_host_pcm takes the PCM byte count; mgx_plan_desc.flags;
                              multi-device groups */

typedef enum mgx_status {
  MGX_OK = 0,
  MGX_E_INVALID_ARGUMENT = -1,   /* NULL pointer, bad enum, bad struct_size */
  MGX_E_NOT_POWER_OF_TWO = -2,   /* "Buffer size is not a power of two" (src/meyda.js:20-22) */
  MGX_E_UNSUPPORTED = -3,        /* valid request this build does not implement */
  MGX_E_DEVICE = -4,             /* a HIP runtime call failed */
  MGX_E_OUT_OF_MEMORY = -5,
  MGX_E_NO_DEVICE = -6           /* no usable gfx950 device */
} mgx_status;

/* Feature indices. The first 13 are the per-frame scalar record, in this order. */
typedef enum mgx_feature {
  MGX_RMS = 0,                  /* src/extractors/rms.js */
  MGX_ENERGY = 1,               /* energy.js */
  MGX_ZCR = 2,                  /* zcr.js (exact integer count) */
  MGX_SPECTRAL_CENTROID = 3,    /* spectralCentroid.js (bin units, as the reference) */
  MGX_SPECTRAL_FLATNESS = 4,    /* spectralFlatness.js */
  MGX_SPECTRAL_SLOPE = 5,       /* spectralSlope.js */
  MGX_SPECTRAL_ROLLOFF = 6,     /* spectralRolloff.js (Hz) */
  MGX_SPECTRAL_SPREAD = 7,      /* spectralSpread.js */
  MGX_SPECTRAL_SKEWNESS = 8,    /* spectralSkewness.js */
  MGX_SPECTRAL_KURTOSIS = 9,    /* spectralKurtosis.js */
  MGX_LOUDNESS_TOTAL = 10,      /* loudness.js .total */
  MGX_PERCEPTUAL_SPREAD = 11,   /* perceptualSpread.js */
  MGX_PERCEPTUAL_SHARPNESS = 12,/* perceptualSharpness.js */
  MGX_NUM_SCALARS = 13,
  /* vector features (pointer fields of mgx_outputs) */
  MGX_LOUDNESS = 13,            /* loudness.js: {specific: Float32Array(24), total} */
  MGX_MFCC = 14,                /* mfcc.js: Float32Array(13) */
  MGX_AMPLITUDE_SPECTRUM = 15,  /* amplitudeSpectrum.js */
  MGX_POWER_SPECTRUM = 16,      /* powerSpectrum.js */
  MGX_COMPLEX_SPECTRUM = 17,    /* complexSpectrum.js: {real, imag} */
  MGX_BUFFER = 18,              /* buffer (declared in feature-info.js:3-5): the frame itself */
  MGX_NUM_FEATURES = 19
} mgx_feature;

typedef enum mgx_window { MGX_WINDOW_HANNING = 0, MGX_WINDOW_HAMMING = 1 } mgx_window;

typedef enum mgx_precision {
  /* FP64 butterflies, every radix-2 stage rounded to float32 as jsfft stores it
   * (lib/jsfft/fft.js:153-161 + Float32Array storage). Parity default. */
  MGX_PRECISION_FAITHFUL = 0,
  /* float32 butterflies: HBM-bound, matches the reference only on broadband input. */
  MGX_PRECISION_FAST = 1
} mgx_precision;

typedef enum mgx_mode {
  MGX_MODE_PER_BUFFER_FFT = 0,  /* the intended path: FFT of every buffer */
  MGX_MODE_LITERAL = 1          /* the snapshot's behaviour: ampSpectrum = |window * x|,
                                   no per-buffer FFT (src/meyda.js:79-84,184-197) */
} mgx_mode;

typedef enum mgx_info_type { MGX_TYPE_NUMBER = 0, MGX_TYPE_ARRAY = 1, MGX_TYPE_MULTIPLE_ARRAYS = 2 } mgx_info_type;

typedef struct mgx_plan_desc {
  uint32_t struct_size;      /* = sizeof(mgx_plan_desc) */
  uint32_t buffer_size;      /* N: power of two; the GPU path supports 256 <= N <= 2048 */
  double sample_rate;        /* audioContext.sampleRate */
  uint32_t window;           /* mgx_window (Meyda.windowingFunction) */
  uint32_t precision;        /* mgx_precision */
  uint32_t mode;             /* mgx_mode */
  uint32_t num_bark_bands;   /* 24 (loudness.js NUM_BARK_BANDS) */
  uint32_t num_mel_bands;    /* 26 in the reference (mfcc.js:15); 1..64 supported */
  uint32_t num_mfcc_coeffs;  /* 13 (mfcc.js:71) */
  uint32_t scalar_f64;       /* 0: scalar outputs are float32 arrays, 1: float64 */
  int32_t device;            /* HIP device ordinal */
  uint32_t flags;            /* MGX_FLAG_* */
} mgx_plan_desc;

/* mgx_plan_desc.flags */
#define MGX_FLAG_DCT_SEQUENTIAL 1u  /* mfcc.js:85-93 DCT as VALU FMAs in the reference's sequential
                                        order instead of the FP64 matrix cores (the default: same
                                        exact products, f64 sums in 4-band blocks) */
#define MGX_FLAG_MFCC_REFERENCE 2u  /* mfcc.js:53-93 in the reference's own order: each mel band summed
                                        over its bins in ascending order into a float32 accumulator of
                                        double products, Math.log in double, the sequential DCT (MFCC
                                        bit-identical wherever the power spectrum is; slower, see
                                        DESIGN.md §5.3). Default off: segmented-scan mel sums, float32
                                        hardware log, the matrix-core DCT, all within 1e-5. */
#define MGX_FLAG_RESIDENT 4u        /* the real-time path (src/meyda.js:69-91, one buffer per call): one-frame
                                        mgx_extract_host calls are served by one workgroup that stays on the
                                        device between calls, polling a mailbox in pinned host memory, instead
                                        of one launch per call. It holds one CU slot and reads the
                                        mailbox over PCIe (about N x 16 bytes per microsecond; with
                                        MGX_RESIDENT_POLL=light its first word only, ~1 us more per call)
                                        while it waits,
                                        and ends itself 20 ms after its last call (MGX_RESIDENT_IDLE_MS), on
                                        the plan's next call of any other kind, or at mgx_plan_destroy. A device
                                        synchronisation made meanwhile waits for that end. mgx_plan_create
                                        pays the path's one-time set-up (~13 ms: pinned buffers, a hardware
                                        queue, one warm-up call), not the first real-time call. Faithful per-buffer
                                        plans without MGX_FLAG_MFCC_REFERENCE only (MGX_E_UNSUPPORTED
                                        otherwise). */

typedef struct mgx_plan mgx_plan;

/* Output arrays, structure of arrays over frames. Any pointer may be NULL: the
 * corresponding feature is then not written (and, where possible, not computed).
 * scalars[i] points to num_frames floats (or doubles if scalar_f64). */
typedef struct mgx_outputs {
  void* scalars[MGX_NUM_SCALARS];
  float* loudness_specific;   /* num_frames x num_bark_bands */
  float* mfcc;                /* num_frames x num_mfcc_coeffs */
  float* amplitude_spectrum;  /* num_frames x N/2 */
  float* power_spectrum;      /* num_frames x N/2 */
  float* complex_real;        /* num_frames x N */
  float* complex_imag;        /* num_frames x N */
} mgx_outputs;

/* Host-side tables of a plan (no device needed): used by tests and by bindings
 * that want to show the same tables Meyda exposes (hanning, hamming, barkScale). */
typedef struct mgx_host_tables {
  float* window;        /* N */
  float* hanning;       /* N */
  float* hamming;       /* N */
  float* bark_scale;    /* N */
  int32_t* bark_limits; /* num_bark_bands + 1 */
  int32_t* mel_bins;    /* num_mel_bands + 2 */
  float* dct;           /* num_mfcc_coeffs * num_mel_bands, layout dct[c + j*num_mfcc_coeffs] */
} mgx_host_tables;

void mgx_plan_desc_init(mgx_plan_desc* desc);
int mgx_plan_create(const mgx_plan_desc* desc, mgx_plan** out_plan);
int mgx_plan_destroy(mgx_plan* plan);
int mgx_plan_get_desc(const mgx_plan* plan, mgx_plan_desc* out_desc);

/* Device-resident batch: frames and every non-NULL output are device pointers.
 * Asynchronous on `stream` (hipStream_t or NULL). The launch uses per-stream device scratch,
 * one set per distinct stream the plan launches on: the scalar features' windows (5 KB per
 * resident wave, ~20 MB), for a plan with MGX_FLAG_MFCC_REFERENCE the power-row ring of its mel
 * chains (~2 KB x 8 per resident wave, tens of MB), and at N = 2048 the tail pool's ticket
 * counter (8 bytes). The whole set is allocated by the first call on its stream, whatever that
 * call's size or outputs (hipMalloc, which may synchronise the device: make one untimed call per
 * stream first, outside any stream capture), and kept until mgx_plan_destroy, which waits for
 * the launches that used it. After that first call a launch keeps no host-side state between
 * calls: it may be captured into a HIP graph and replayed any number of times. */
int mgx_extract_device(mgx_plan* plan, const float* frames, uint64_t num_frames,
                       const mgx_outputs* outputs, void* stream);

/* Host batch: frames and outputs in host memory; returns when the outputs are
 * written. Up to 512 frames run one launch over plan-owned pinned host memory
 * (a single frame of N <= 1024 samples inside the kernel arguments, or with
 * MGX_FLAG_RESIDENT handed to the plan's resident workgroup); larger
 * batches stage through plan-owned device buffers in chunks. A one-frame call
 * without spectrum outputs may return while the tail of its launch still runs
 * on the plan's stream: later calls on the plan are ordered after it, and
 * mgx_plan_destroy waits for it. */
int mgx_extract_host(mgx_plan* plan, const float* frames, uint64_t num_frames,
                     const mgx_outputs* outputs);

/* Synthetic PCM written straight into HBM:
 * x[i] = (splitmix64(seed + (i+1)*0x9E3779B97F4A7C15) >> 40) * 2^-23 - 1,
 * i = first_frame*N + t for t < num_frames*N. */
int mgx_synth_frames_device(float* frames, uint64_t num_frames, uint32_t buffer_size,
                            uint64_t seed, uint64_t first_frame, void* stream);

int mgx_get_host_tables(const mgx_plan_desc* desc, const mgx_host_tables* out);

/* ---- PCM / WAV ingest ---------------------------------
 * Replaces the browser's decodeAudioData + getChannelData(0) that feed the
 * reference (lib/bufferLoader.js:23, index.html:182, src/meyda.js:72): samples of
 * one channel become float32 exactly as decodeAudioData scales them
 * (u8: (v-128)/128, s16: v/32768, s24: v/2^23, s32: v/2^31, f32: as stored), and
 * are cut into non-overlapping buffer_size frames (a trailing partial frame is
 * dropped, as a ScriptProcessor only delivers full buffers). */
typedef enum mgx_pcm_format {
  MGX_PCM_F32 = 0,
  MGX_PCM_S16 = 1,
  MGX_PCM_U8 = 2,
  MGX_PCM_S24 = 3,   /* packed, 3 bytes little-endian */
  MGX_PCM_S32 = 4
} mgx_pcm_format;

typedef struct mgx_wav_info {
  uint32_t struct_size;     /* = sizeof(mgx_wav_info) */
  uint32_t pcm_format;      /* mgx_pcm_format */
  uint32_t channels;
  uint32_t sample_rate;
  uint32_t bits_per_sample;
  uint32_t block_align;     /* bytes per sample frame (all channels) */
  uint64_t data_offset;     /* byte offset of the first sample in the file */
  uint64_t data_bytes;      /* sample bytes present (the data chunk, clipped to the file) */
  uint64_t sample_frames;   /* data_bytes / block_align */
} mgx_wav_info;

/* RIFF/WAVE header walk: 'fmt ' chunk of 16, 18 or 40 (WAVE_FORMAT_EXTENSIBLE)
 * bytes, PCM (1) or IEEE float (3), chunks in any order, odd sizes padded. Host
 * only (no device). info->struct_size must be set by the caller. */
int mgx_wav_parse(const void* bytes, uint64_t num_bytes, mgx_wav_info* info);

/* Device decode: `sample_frames` interleaved frames of `channels` samples at
 * `pcm` (device memory, any byte alignment) -> float32 samples of channel `channel` at `out`. */
int mgx_pcm_decode_device(const void* pcm, uint64_t sample_frames, uint32_t format, uint32_t channels,
                          uint32_t channel, float* out, void* stream);

/* Host PCM in, host outputs: floor(sample_frames / buffer_size) buffers of channel
 * `channel`. The raw PCM (not float32) crosses PCIe and is decoded on the device;
 * outputs are laid out as for mgx_extract_host. `pcm_bytes` is the size of the buffer at
 * `pcm`: sample_frames * channels * bytes-per-sample beyond it is MGX_E_INVALID_ARGUMENT
 * (no read past the caller's buffer). `pcm` needs no alignment. */
int mgx_extract_host_pcm(mgx_plan* plan, const void* pcm, uint64_t pcm_bytes, uint64_t sample_frames,
                         uint32_t format, uint32_t channels, uint32_t channel, const mgx_outputs* outputs);

/* ---- Multi-device groups -------------------------------
 * Replaces nothing in the reference (single-threaded browser code); it exists because
 * buffers are independent (src/meyda.js:69-91 keeps no cross-buffer state), so a batch
 * is cut into contiguous shards, one per device, each extracted by that device's plan
 * (the plan of `new Meyda(...)`, src/meyda.js:17-97), and the per-frame feature records
 * are gathered to the root device (rank 0) over xGMI by RCCL point-to-point transfers.
 * The gather is chunked: chunk i of every shard is sent while chunk i+1 is extracted.
 * RCCL (librccl.so.1, or $MGX_RCCL_LIB) is loaded when a group of more than one rank is
 * created; a one-rank group needs no RCCL. */
typedef struct mgx_group mgx_group;

#define MGX_COMM_ID_BYTES 128  /* an RCCL unique id (ncclUniqueId) */

/* Output selection of a group extraction (every rank passes the same mask). */
#define MGX_OUT_SCALAR(i) (1u << (i))       /* i < MGX_NUM_SCALARS */
#define MGX_OUT_LOUDNESS_SPECIFIC (1u << 13)
#define MGX_OUT_MFCC (1u << 14)
#define MGX_OUT_AMPLITUDE_SPECTRUM (1u << 15)
#define MGX_OUT_POWER_SPECTRUM (1u << 16)
#define MGX_OUT_COMPLEX_SPECTRUM (1u << 17)   /* real and imag */
#define MGX_OUT_ALL_MASK ((1u << 18) - 1)

/* Contiguous shard [*start, *start + *count) of `total` frames for `rank` of `nranks`:
 * the first total % nranks ranks get one frame more. Host only. */
int mgx_shard_range(uint64_t total, uint32_t nranks, uint32_t rank, uint64_t* start, uint64_t* count);

/* Byte offsets of the outputs of `num_frames` frames packed into one transfer buffer
 * (structure of arrays, each array 256-byte aligned, in mgx_outputs order: 13 scalars,
 * loudness_specific, mfcc, amplitude, power, complex real, complex imag). offsets[i] is
 * the offset of field i (MGX_OUT_* bit i; the complex field has two arrays: offsets[17]
 * real, offsets[18] imag), or UINT64_MAX when not in `mask`. Returns the total bytes.
 * Host only; the root unpacks each peer's chunk with the same arithmetic. */
uint64_t mgx_packed_layout(const mgx_plan_desc* desc, uint32_t mask, uint64_t num_frames, uint64_t offsets[19]);

/* Single process, several devices (RCCL ncclCommInitAll): devices[0] is the root. */
int mgx_group_create(const mgx_plan_desc* desc, const int32_t* devices, uint32_t num_devices, mgx_group** out);

/* One process per device (e.g. torchrun): rank 0 calls mgx_comm_unique_id and the caller
 * broadcasts the bytes; every rank then calls mgx_group_create_rank with its rank.
 * desc->device is this rank's device. Rank 0 is the root.
 * Test transport across processes: with MGX_GROUP_TRANSPORT=ipc in the environment of every
 * rank, the id names a POSIX shared-memory mailbox instead of an RCCL communicator, and each
 * peer chunk reaches the root through hipIpcGetMemHandle / hipIpcOpenMemHandle of the peer's
 * transfer buffer (a device copy on the root's communication stream, handed over through the
 * mailbox's per-slot sequence numbers) -- the multi-rank data path across a process boundary,
 * runnable with every rank on one GPU (RCCL refuses that). $MGX_IPC_TIMEOUT_S (default 60)
 * bounds each wait for a peer; a missing peer is an MGX_E_DEVICE error, not a hang. */
int mgx_comm_unique_id(void* id, uint64_t id_bytes);
int mgx_group_create_rank(const mgx_plan_desc* desc, const void* unique_id, uint32_t nranks, uint32_t rank,
                          mgx_group** out);
/* Test transport: nranks ranks in this process, all on desc->device, whose chunk transfers
 * are device copies into the root's staging slots instead of RCCL messages. Everything
 * else -- shards, chunks, transfer slots, the two compute streams, the root's unpack -- is
 * the multi-device path's own code, so one GPU can check the gather byte for byte. */
int mgx_group_create_loopback(const mgx_plan_desc* desc, uint32_t nranks, mgx_group** out);
/* The same test group with the RCCL transport: the root holds a one-rank RCCL
 * communicator on desc->device, and each peer chunk crosses as an ncclSend to self matched
 * by an ncclRecv from self (one ncclGroupStart/End each) on the root's communication
 * stream -- the RCCL calls, message sizes, slot ordering and unpack of the multi-rank
 * path, runnable on one GPU (RCCL refuses two ranks on one device). */
int mgx_group_create_loopback_rccl(const mgx_plan_desc* desc, uint32_t nranks, mgx_group** out);
int mgx_group_destroy(mgx_group* group);
/* Ranks of the group, and the ranks this process drives (num_local = 1 per process, or
 * all of them in single-process mode, first_local = their first rank). */
int mgx_group_info(const mgx_group* group, uint32_t* nranks, uint32_t* first_local, uint32_t* num_local);
/* What the RCCL communicator of this process's first local rank reports: ranks in the
 * communicator (ncclCommCount), this rank in it (ncclCommUserRank) and its device
 * (ncclCommCuDevice); all -1 when the group has no communicator (one rank, or device copies).
 * MGX_E_UNSUPPORTED when the loaded RCCL lacks those three queries (the data path does not
 * need them). */
int mgx_group_comm_info(const mgx_group* group, int32_t* comm_ranks, int32_t* comm_rank, int32_t* comm_device);

/* Device-resident batch. frames[i]: device pointer of the shard of local rank
 * first_local + i (on that rank's device); counts: frames of every rank (nranks
 * entries, the same on every rank; shard r holds global frames [sum counts[<r],
 * + counts[r])). root_out: device pointers on the root device sized for sum(counts)
 * frames (read on the root only; may be NULL elsewhere); every field in `mask` must be
 * non-NULL there. num_chunks: pipeline depth (0 = automatic). streams: NULL for the
 * group's own streams, else streams[i] is local rank i's stream (a NULL entry is that
 * device's default stream): the work is ordered after what is enqueued on it, and it
 * waits for the work's completion (gather included). Asynchronous. */
int mgx_group_extract_device(mgx_group* group, const float* const* frames, const uint64_t* counts,
                             const mgx_outputs* root_out, uint32_t mask, uint32_t num_chunks,
                             void* const* streams);

/* Host batch in, host outputs (single-process groups): the frames are cut into one
 * shard per device (mgx_shard_range), copied to the devices in parallel, extracted,
 * gathered to the root device by RCCL and copied back. Output layout as mgx_extract_host. */
int mgx_group_extract_host(mgx_group* group, const float* frames, uint64_t num_frames, const mgx_outputs* outputs);

int mgx_is_power_of_two(double n);           /* src/utils.js:13-19 */
int mgx_feature_index(const char* name);     /* -1 if unknown */
const char* mgx_feature_name(int feature);   /* NULL if out of range */
int mgx_feature_info(int feature);           /* mgx_info_type, or -1 */
int mgx_device_count(int* count);
int mgx_abi_version(void);
const char* mgx_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MEYDA_GPU_H */
