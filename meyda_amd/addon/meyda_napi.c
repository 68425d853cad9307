/*
 * meyda_napi.c — N-API bridge between JavaScript typed arrays and the C ABI
 * (include/meyda_gpu.h). Thin by design: argument marshalling, typed-array
 * allocation and error translation; all compute is in libmeyda_gpu.so.
 *
 * Exports:
 *   createPlan(opts)                     -> plan handle (external; destroyed by GC or destroyPlan);
 *                                           opts.devices = [d0, d1, ...] makes a multi-device
 *                                           plan: batches are sharded over the devices and the
 *                                           features gathered to d0 by RCCL (mgx_group_*)
 *   destroyPlan(plan)
 *   planBusy(plan)                       -> true while an async extraction owns the plan
 *   extract(plan, frames, features)      -> { name: TypedArray }   (synchronous)
 *   extractAsync(plan, frames, features) -> Promise<{ name: TypedArray }>  (napi_async_work)
 *   extractWav(plan, wavBytes, features[, channel]) / extractWavAsync(...)
 *                                        -> the features of every full buffer of a .wav file;
 *                                           the raw PCM is decoded on the device
 *   wavParse(wavBytes)                   -> { pcmFormat, channels, sampleRate, bitsPerSample, ... }
 *   hostTables(opts)                     -> { hanning, hamming, window, barkScale, barkLimits, melBins, dct }
 *   isPowerOfTwo(n), deviceCount(), featureNames(), featureInfo(name), abiVersion()
 * Feature names are the reference extractor names (src/extractors/index.js).
 * Scalars come back as Float64Array (JS numbers are doubles), vectors as Float32Array.
 */
#define NAPI_VERSION 4
#include <node_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/meyda_gpu.h"

#define CHECK(call)                                                       \
  do {                                                                    \
    if ((call) != napi_ok) {                                              \
      napi_throw_error(env, NULL, "meyda_napi: N-API call failed: " #call); \
      return NULL;                                                        \
    }                                                                     \
  } while (0)

static napi_value throw_mgx(napi_env env, int rc) {
  char code[16];
  snprintf(code, sizeof code, "%d", rc);
  napi_throw_error(env, code, mgx_last_error());
  return NULL;
}

typedef struct {
  mgx_plan* plan;
  mgx_group* group;  /* createPlan({devices: [...]}): a multi-device group */
  mgx_plan_desc desc;
  int busy;       /* an async extraction owns the plan */
  int finalized;  /* the JS handle was collected while busy: async_complete frees the box */
} plan_box;

static void plan_box_free(plan_box* b) {
  if (b->plan) mgx_plan_destroy(b->plan);
  if (b->group) mgx_group_destroy(b->group);
  free(b);
}

/* A queued or running async job holds a reference to the plan's external, so the GC
 * cannot collect it mid-job; `finalized` covers a finalizer that runs anyway while the
 * job is in flight (environment teardown): the box is then freed by async_complete. */
static void plan_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  plan_box* b = (plan_box*)data;
  if (b->busy) {
    b->finalized = 1;
    return;
  }
  plan_box_free(b);
}

static int get_u32_prop(napi_env env, napi_value obj, const char* name, uint32_t* out) {
  bool has = false;
  if (napi_has_named_property(env, obj, name, &has) != napi_ok || !has) return 0;
  napi_value v;
  napi_valuetype t;
  if (napi_get_named_property(env, obj, name, &v) != napi_ok) return 0;
  napi_typeof(env, v, &t);
  if (t != napi_number) return 0;
  napi_get_value_uint32(env, v, out);
  return 1;
}

static int get_f64_prop(napi_env env, napi_value obj, const char* name, double* out) {
  bool has = false;
  if (napi_has_named_property(env, obj, name, &has) != napi_ok || !has) return 0;
  napi_value v;
  napi_valuetype t;
  if (napi_get_named_property(env, obj, name, &v) != napi_ok) return 0;
  napi_typeof(env, v, &t);
  if (t != napi_number) return 0;
  napi_get_value_double(env, v, out);
  return 1;
}

static int get_str_prop(napi_env env, napi_value obj, const char* name, char* buf, size_t cap) {
  bool has = false;
  if (napi_has_named_property(env, obj, name, &has) != napi_ok || !has) return 0;
  napi_value v;
  napi_valuetype t;
  if (napi_get_named_property(env, obj, name, &v) != napi_ok) return 0;
  napi_typeof(env, v, &t);
  if (t != napi_string) return 0;
  size_t len = 0;
  napi_get_value_string_utf8(env, v, buf, cap, &len);
  return 1;
}

/* opts: { bufferSize, sampleRate, windowingFunction, precision, mode, numMelBands,
 *         numMfccCoeffs, device, scalarF64, dctSequential, mfccReferenceOrder, resident, devices } */
static int desc_from_opts(napi_env env, napi_value opts, mgx_plan_desc* d) {
  mgx_plan_desc_init(d);
  d->scalar_f64 = 1;
  double dv;
  uint32_t u;
  char s[64];
  if (get_f64_prop(env, opts, "bufferSize", &dv)) {
    if (!mgx_is_power_of_two(dv)) d->buffer_size = 3; /* reported as not-a-power-of-two */
    else d->buffer_size = (uint32_t)dv;
  }
  if (get_f64_prop(env, opts, "sampleRate", &dv)) d->sample_rate = dv;
  if (get_str_prop(env, opts, "windowingFunction", s, sizeof s)) {
    if (strcmp(s, "hanning") == 0) d->window = MGX_WINDOW_HANNING;
    else if (strcmp(s, "hamming") == 0) d->window = MGX_WINDOW_HAMMING;
    else d->window = 99;
  }
  if (get_str_prop(env, opts, "precision", s, sizeof s)) d->precision = strcmp(s, "fast") == 0 ? MGX_PRECISION_FAST : MGX_PRECISION_FAITHFUL;
  if (get_str_prop(env, opts, "mode", s, sizeof s)) d->mode = strcmp(s, "literal") == 0 ? MGX_MODE_LITERAL : MGX_MODE_PER_BUFFER_FFT;
  if (get_u32_prop(env, opts, "numMelBands", &u)) d->num_mel_bands = u;
  if (get_u32_prop(env, opts, "numMfccCoeffs", &u)) d->num_mfcc_coeffs = u;
  if (get_u32_prop(env, opts, "device", &u)) d->device = (int32_t)u;
  if (get_u32_prop(env, opts, "scalarF64", &u)) d->scalar_f64 = u ? 1 : 0;
  if (get_u32_prop(env, opts, "dctSequential", &u) && u) d->flags |= MGX_FLAG_DCT_SEQUENTIAL;
  if (get_u32_prop(env, opts, "mfccReferenceOrder", &u) && u) d->flags |= MGX_FLAG_MFCC_REFERENCE;
  if (get_u32_prop(env, opts, "resident", &u) && u) d->flags |= MGX_FLAG_RESIDENT;
  return 1;
}

static napi_value create_plan(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 1) {
    napi_throw_type_error(env, NULL, "createPlan(opts) expects an options object");
    return NULL;
  }
  mgx_plan_desc d;
  desc_from_opts(env, argv[0], &d);
  /* devices: [d0, d1, ...] shards every batch over those devices (d0 is the root) */
  int32_t devs[64];
  uint32_t ndev = 0;
  bool has = false, is_arr = false;
  napi_has_named_property(env, argv[0], "devices", &has);
  if (has) {
    napi_value arr;
    CHECK(napi_get_named_property(env, argv[0], "devices", &arr));
    napi_is_array(env, arr, &is_arr);
    if (is_arr) {
      napi_get_array_length(env, arr, &ndev);
      if (ndev == 0 || ndev > 64) {
        napi_throw_range_error(env, NULL, "devices must list 1 to 64 device ordinals");
        return NULL;
      }
      for (uint32_t i = 0; i < ndev; ++i) {
        napi_value v;
        int32_t dv = -1;
        napi_get_element(env, arr, i, &v);
        if (napi_get_value_int32(env, v, &dv) != napi_ok) {
          napi_throw_type_error(env, NULL, "devices must be numbers");
          return NULL;
        }
        devs[i] = dv;
      }
      d.device = devs[0];
    }
  }
  mgx_plan* p = NULL;
  mgx_group* grp = NULL;
  int rc = ndev > 0 ? mgx_group_create(&d, devs, ndev, &grp) : mgx_plan_create(&d, &p);
  if (rc) return throw_mgx(env, rc);
  plan_box* b = (plan_box*)calloc(1, sizeof *b);
  b->plan = p;
  b->group = grp;
  b->desc = d;
  napi_value ext;
  CHECK(napi_create_external(env, b, plan_finalize, NULL, &ext));
  return ext;
}

static plan_box* get_plan(napi_env env, napi_value v) {
  void* data = NULL;
  if (napi_get_value_external(env, v, &data) != napi_ok || !data) {
    napi_throw_type_error(env, NULL, "expected a plan created by createPlan()");
    return NULL;
  }
  plan_box* b = (plan_box*)data;
  if (!b->plan && !b->group) {
    napi_throw_error(env, NULL, "plan was destroyed");
    return NULL;
  }
  return b;
}

static napi_value plan_busy(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], r;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  plan_box* b = argc ? get_plan(env, argv[0]) : NULL;
  if (!b) return NULL;
  CHECK(napi_get_boolean(env, b->busy != 0, &r));
  return r;
}

static napi_value destroy_plan(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  plan_box* b = argc ? get_plan(env, argv[0]) : NULL;
  if (!b) return NULL;
  if (b->busy) {
    napi_throw_error(env, NULL, "plan is busy with an async extraction");
    return NULL;
  }
  if (b->plan) mgx_plan_destroy(b->plan);
  if (b->group) mgx_group_destroy(b->group);
  b->plan = NULL;
  b->group = NULL;
  return NULL;
}

/* ------------------------------------------------------------ extraction job */
enum { SLOT_SCALAR0 = 0, SLOT_LOUD = MGX_NUM_SCALARS, SLOT_MFCC, SLOT_AMP, SLOT_POW, SLOT_CRE, SLOT_CIM, NSLOTS };

typedef struct {
  plan_box* box;
  const float* frames;
  uint64_t nframes;
  /* PCM input (extractWav): interleaved samples, decoded on the device */
  const unsigned char* pcm;
  uint64_t pcm_bytes;
  uint64_t pcm_frames;
  uint32_t pcm_format, pcm_channels, pcm_channel;
  mgx_outputs out;
  /* The outputs are written straight into JS ArrayBuffers (napi_create_arraybuffer), held by
   * references until the result object takes them. (External ArrayBuffers over malloc'd memory
   * with a free finalizer made Node 12 abort at exit: v8impl ArrayBufferReference::Finalize's
   * assertion during the environment's teardown.) */
  napi_ref refs[NSLOTS];
  void* bufs[NSLOTS];
  size_t bytes[NSLOTS];
  int want[NSLOTS];
  napi_ref frames_ref;
  napi_ref plan_ref;  /* keeps the plan's external alive while the job is queued or running */
  napi_deferred deferred;
  napi_async_work work;
  int rc;
  char err[512];
} job;

static void job_free_buffers(napi_env env, job* j) {
  for (int i = 0; i < NSLOTS; ++i)
    if (j->refs[i]) {
      napi_delete_reference(env, j->refs[i]);
      j->refs[i] = NULL;
      j->bufs[i] = NULL;
    }
}

/* Parse the features argument (string or array of strings) into wanted output slots. */
static int parse_features(napi_env env, napi_value feats, job* j) {
  bool is_arr = false;
  napi_is_array(env, feats, &is_arr);
  uint32_t n = 1;
  if (is_arr) napi_get_array_length(env, feats, &n);
  for (uint32_t i = 0; i < n; ++i) {
    napi_value v = feats;
    if (is_arr) napi_get_element(env, feats, i, &v);
    char name[64];
    size_t len = 0;
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t != napi_string) {
      napi_throw_type_error(env, NULL, "feature names must be strings");
      return 0;
    }
    napi_get_value_string_utf8(env, v, name, sizeof name, &len);
    int f = mgx_feature_index(name);
    if (f < 0) {
      char msg[128];
      snprintf(msg, sizeof msg, "unknown feature '%s'", name);
      napi_throw_type_error(env, NULL, msg);
      return 0;
    }
    if (f < MGX_NUM_SCALARS) j->want[f] = 1;
    else if (f == MGX_LOUDNESS) { j->want[SLOT_LOUD] = 1; j->want[MGX_LOUDNESS_TOTAL] = 1; }
    else if (f == MGX_MFCC) j->want[SLOT_MFCC] = 1;
    else if (f == MGX_AMPLITUDE_SPECTRUM) j->want[SLOT_AMP] = 1;
    else if (f == MGX_POWER_SPECTRUM) j->want[SLOT_POW] = 1;
    else if (f == MGX_COMPLEX_SPECTRUM) { j->want[SLOT_CRE] = 1; j->want[SLOT_CIM] = 1; }
    /* MGX_BUFFER is the input itself: handled by the JS facade */
  }
  return 1;
}

static int job_alloc(napi_env env, job* j, napi_value feats);

static int job_prepare(napi_env env, job* j, napi_value frames_v, napi_value feats) {
  bool is_ta = false;
  napi_is_typedarray(env, frames_v, &is_ta);
  if (!is_ta) {
    napi_throw_type_error(env, NULL, "frames must be a Float32Array");
    return 0;
  }
  napi_typedarray_type tt;
  size_t len = 0;
  void* data = NULL;
  napi_value ab;
  size_t off = 0;
  napi_get_typedarray_info(env, frames_v, &tt, &len, &data, &ab, &off);
  if (tt != napi_float32_array) {
    napi_throw_type_error(env, NULL, "frames must be a Float32Array");
    return 0;
  }
  const uint32_t n = j->box->desc.buffer_size;
  if (len % n) {
    napi_throw_range_error(env, NULL, "frames.length must be a multiple of bufferSize");
    return 0;
  }
  j->frames = (const float*)data;
  j->nframes = len / n;
  return job_alloc(env, j, feats);
}

/* Wanted outputs for j->nframes frames. */
static int job_alloc(napi_env env, job* j, napi_value feats) {
  const uint32_t n = j->box->desc.buffer_size;
  if (!parse_features(env, feats, j)) return 0;
  const size_t F = j->nframes, L = n / 2;
  const size_t ss = j->box->desc.scalar_f64 ? 8 : 4;
  for (int i = 0; i < NSLOTS; ++i) {
    if (!j->want[i]) continue;
    size_t b = 0;
    if (i < MGX_NUM_SCALARS) b = F * ss;
    else if (i == SLOT_LOUD) b = F * 24 * 4;
    else if (i == SLOT_MFCC) b = F * j->box->desc.num_mfcc_coeffs * 4;
    else if (i == SLOT_AMP || i == SLOT_POW) b = F * L * 4;
    else b = F * n * 4;
    j->bytes[i] = b;
    napi_value abv;
    void* data = NULL;
    if (napi_create_arraybuffer(env, b, &data, &abv) != napi_ok || napi_create_reference(env, abv, 1, &j->refs[i]) != napi_ok) {
      napi_throw_error(env, NULL, "out of host memory");
      return 0;
    }
    j->bufs[i] = data;
  }
  for (int i = 0; i < MGX_NUM_SCALARS; ++i) j->out.scalars[i] = j->bufs[i];
  j->out.loudness_specific = (float*)j->bufs[SLOT_LOUD];
  j->out.mfcc = (float*)j->bufs[SLOT_MFCC];
  j->out.amplitude_spectrum = (float*)j->bufs[SLOT_AMP];
  j->out.power_spectrum = (float*)j->bufs[SLOT_POW];
  j->out.complex_real = (float*)j->bufs[SLOT_CRE];
  j->out.complex_imag = (float*)j->bufs[SLOT_CIM];
  return 1;
}

/* wavBytes: a Buffer / Uint8Array / ArrayBuffer holding a whole .wav file. */
static int bytes_of(napi_env env, napi_value v, const unsigned char** data, size_t* len) {
  bool is = false;
  void* d = NULL;
  napi_is_buffer(env, v, &is);
  if (is) {
    napi_get_buffer_info(env, v, &d, len);
    *data = (const unsigned char*)d;
    return 1;
  }
  napi_is_typedarray(env, v, &is);
  if (is) {
    napi_typedarray_type tt;
    size_t n = 0, off = 0;
    napi_value ab;
    napi_get_typedarray_info(env, v, &tt, &n, &d, &ab, &off);
    if (tt == napi_uint8_array || tt == napi_int8_array || tt == napi_uint8_clamped_array) {
      *data = (const unsigned char*)d;
      *len = n;
      return 1;
    }
  }
  napi_is_arraybuffer(env, v, &is);
  if (is) {
    napi_get_arraybuffer_info(env, v, &d, len);
    *data = (const unsigned char*)d;
    return 1;
  }
  napi_throw_type_error(env, NULL, "expected the bytes of a .wav file (Buffer, Uint8Array or ArrayBuffer)");
  return 0;
}

static int job_prepare_wav(napi_env env, job* j, napi_value wav_v, napi_value feats, napi_value chan_v) {
  const unsigned char* data = NULL;
  size_t len = 0;
  if (!bytes_of(env, wav_v, &data, &len)) return 0;
  mgx_wav_info wi;
  memset(&wi, 0, sizeof wi);
  wi.struct_size = sizeof wi;
  int rc = mgx_wav_parse(data, len, &wi);
  if (rc) {
    throw_mgx(env, rc);
    return 0;
  }
  uint32_t ch = 0;
  if (chan_v) {
    napi_valuetype t;
    napi_typeof(env, chan_v, &t);
    if (t == napi_number) napi_get_value_uint32(env, chan_v, &ch);
  }
  if (ch >= wi.channels) {
    napi_throw_range_error(env, NULL, "channel out of range for this file");
    return 0;
  }
  j->pcm = data + wi.data_offset;
  j->pcm_bytes = wi.data_bytes;
  j->pcm_frames = wi.sample_frames;
  j->pcm_format = wi.pcm_format;
  j->pcm_channels = wi.channels;
  j->pcm_channel = ch;
  j->nframes = wi.sample_frames / j->box->desc.buffer_size;
  return job_alloc(env, j, feats);
}

static void job_run(job* j) {
  if (j->box->group && j->pcm) {
    j->rc = MGX_E_UNSUPPORTED;
    snprintf(j->err, sizeof j->err, "extractWav on a multi-device plan: use a single-device plan");
    return;
  }
  if (j->box->group)
    j->rc = mgx_group_extract_host(j->box->group, j->frames, j->nframes, &j->out);
  else if (j->pcm)
    j->rc = mgx_extract_host_pcm(j->box->plan, j->pcm, j->pcm_bytes, j->pcm_frames, j->pcm_format, j->pcm_channels,
                                 j->pcm_channel, &j->out);
  else
    j->rc = mgx_extract_host(j->box->plan, j->frames, j->nframes, &j->out);
  if (j->rc) snprintf(j->err, sizeof j->err, "%s", mgx_last_error());
}

static napi_value typed(napi_env env, job* j, int slot, napi_typedarray_type t, size_t elem) {
  napi_value ab, ta;
  if (napi_get_reference_value(env, j->refs[slot], &ab) != napi_ok) return NULL;
  if (napi_create_typedarray(env, t, j->bytes[slot] / elem, ab, 0, &ta) != napi_ok) return NULL;
  return ta;
}

static napi_value job_result(napi_env env, job* j) {
  static const char* names[MGX_NUM_SCALARS] = {
      "rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope", "spectralRolloff",
      "spectralSpread", "spectralSkewness", "spectralKurtosis", "loudness.total", "perceptualSpread",
      "perceptualSharpness"};
  napi_value obj;
  if (napi_create_object(env, &obj) != napi_ok) return NULL;
  const int f64 = j->box->desc.scalar_f64;
  for (int i = 0; i < MGX_NUM_SCALARS; ++i)
    if (j->want[i]) napi_set_named_property(env, obj, names[i], typed(env, j, i, f64 ? napi_float64_array : napi_float32_array, f64 ? 8 : 4));
  if (j->want[SLOT_LOUD]) napi_set_named_property(env, obj, "loudness.specific", typed(env, j, SLOT_LOUD, napi_float32_array, 4));
  if (j->want[SLOT_MFCC]) napi_set_named_property(env, obj, "mfcc", typed(env, j, SLOT_MFCC, napi_float32_array, 4));
  if (j->want[SLOT_AMP]) napi_set_named_property(env, obj, "amplitudeSpectrum", typed(env, j, SLOT_AMP, napi_float32_array, 4));
  if (j->want[SLOT_POW]) napi_set_named_property(env, obj, "powerSpectrum", typed(env, j, SLOT_POW, napi_float32_array, 4));
  if (j->want[SLOT_CRE]) napi_set_named_property(env, obj, "complexSpectrum.real", typed(env, j, SLOT_CRE, napi_float32_array, 4));
  if (j->want[SLOT_CIM]) napi_set_named_property(env, obj, "complexSpectrum.imag", typed(env, j, SLOT_CIM, napi_float32_array, 4));
  return obj;
}

static napi_value extract_common(napi_env env, napi_callback_info info, int wav) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) {
    napi_throw_type_error(env, NULL, wav ? "extractWav(plan, wavBytes, features[, channel])" : "extract(plan, frames, features)");
    return NULL;
  }
  job j;
  memset(&j, 0, sizeof j);
  j.box = get_plan(env, argv[0]);
  if (!j.box) return NULL;
  if (j.box->busy) {
    napi_throw_error(env, NULL, "plan is busy with an async extraction");
    return NULL;
  }
  if (!(wav ? job_prepare_wav(env, &j, argv[1], argv[2], argc > 3 ? argv[3] : NULL)
            : job_prepare(env, &j, argv[1], argv[2]))) {
    job_free_buffers(env, &j);
    return NULL;
  }
  job_run(&j);
  if (j.rc) {
    job_free_buffers(env, &j);
    char code[16];
    snprintf(code, sizeof code, "%d", j.rc);
    napi_throw_error(env, code, j.err);
    return NULL;
  }
  napi_value r = job_result(env, &j);
  job_free_buffers(env, &j);
  return r;
}

/* extractInto(plan, frames, offsets, out): the same synchronous extraction into ONE caller-provided
 * ArrayBuffer. offsets: a Float64Array of the 19 output fields' byte offsets in `out` (mgx_outputs
 * order: the 13 scalars, loudness_specific, mfcc, amplitude, power, complex real, complex imag; a
 * negative entry = not requested). The facade's real-time paths (get(), batched streaming) lay the
 * outputs of a feature list out once and call this per buffer or batch: one allocation and a handful of
 * N-API calls instead of an ArrayBuffer, a reference and a typed array per output. */
static napi_value extract_into(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 4) {
    napi_throw_type_error(env, NULL, "extractInto(plan, frames, offsets, out)");
    return NULL;
  }
  plan_box* box = get_plan(env, argv[0]);
  if (!box) return NULL;
  if (box->busy) {
    napi_throw_error(env, NULL, "plan is busy with an async extraction");
    return NULL;
  }
  napi_typedarray_type tt;
  size_t len = 0, off = 0, olen = 0;
  void* data = NULL;
  void* offs = NULL;
  napi_value ab;
  bool is = false;
  napi_is_typedarray(env, argv[1], &is);
  if (is) napi_get_typedarray_info(env, argv[1], &tt, &len, &data, &ab, &off);
  if (!is || tt != napi_float32_array) {
    napi_throw_type_error(env, NULL, "frames must be a Float32Array");
    return NULL;
  }
  napi_is_typedarray(env, argv[2], &is);
  if (is) napi_get_typedarray_info(env, argv[2], &tt, &olen, &offs, &ab, &off);
  if (!is || tt != napi_float64_array || olen != 19) {
    napi_throw_type_error(env, NULL, "offsets must be a Float64Array of 19 byte offsets");
    return NULL;
  }
  void* out = NULL;
  size_t out_bytes = 0;
  napi_is_arraybuffer(env, argv[3], &is);
  if (is) napi_get_arraybuffer_info(env, argv[3], &out, &out_bytes);
  if (!is) {
    napi_throw_type_error(env, NULL, "out must be an ArrayBuffer");
    return NULL;
  }
  const uint32_t n = box->desc.buffer_size;
  if (len % n) {
    napi_throw_range_error(env, NULL, "frames.length must be a multiple of bufferSize");
    return NULL;
  }
  const uint64_t F = len / n;
  const size_t ss = box->desc.scalar_f64 ? 8 : 4;
  size_t per[19];
  for (int i = 0; i < 19; ++i)
    per[i] = i < MGX_NUM_SCALARS ? ss : i == 13 ? 24 * 4 : i == 14 ? (size_t)box->desc.num_mfcc_coeffs * 4
           : i < 17 ? (size_t)(n / 2) * 4 : (size_t)n * 4;
  void* ptr[19];
  const double* o = (const double*)offs;
  for (int i = 0; i < 19; ++i) {
    ptr[i] = NULL;
    if (!(o[i] >= 0)) continue;
    const double end = o[i] + (double)(per[i] * F);
    if (o[i] != (double)(uint64_t)o[i] || end > (double)out_bytes || ((uint64_t)o[i] % (i < MGX_NUM_SCALARS ? ss : 4))) {
      napi_throw_range_error(env, NULL, "an output's offset is misaligned or runs past the end of out");
      return NULL;
    }
    ptr[i] = (unsigned char*)out + (uint64_t)o[i];
  }
  if ((ptr[17] == NULL) != (ptr[18] == NULL)) {
    napi_throw_range_error(env, NULL, "complex real and imag go together");
    return NULL;
  }
  mgx_outputs mo;
  memset(&mo, 0, sizeof mo);
  for (int i = 0; i < MGX_NUM_SCALARS; ++i) mo.scalars[i] = ptr[i];
  mo.loudness_specific = (float*)ptr[13];
  mo.mfcc = (float*)ptr[14];
  mo.amplitude_spectrum = (float*)ptr[15];
  mo.power_spectrum = (float*)ptr[16];
  mo.complex_real = (float*)ptr[17];
  mo.complex_imag = (float*)ptr[18];
  const int rc = box->group ? mgx_group_extract_host(box->group, (const float*)data, F, &mo)
                            : mgx_extract_host(box->plan, (const float*)data, F, &mo);
  if (rc) return throw_mgx(env, rc);
  return argv[3];
}

static napi_value extract_sync(napi_env env, napi_callback_info info) { return extract_common(env, info, 0); }
static napi_value extract_wav_sync(napi_env env, napi_callback_info info) { return extract_common(env, info, 1); }

static void async_execute(napi_env env, void* data) {
  (void)env;
  job_run((job*)data);
}

static void async_complete(napi_env env, napi_status status, void* data) {
  job* j = (job*)data;
  plan_box* box = j->box;
  box->busy = 0;
  if (status != napi_ok || j->rc) {
    napi_value msg, err;
    napi_create_string_utf8(env, j->rc ? j->err : "async extraction cancelled", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, j->deferred, err);
  } else {
    napi_resolve_deferred(env, j->deferred, job_result(env, j));
  }
  napi_delete_reference(env, j->frames_ref);
  napi_delete_reference(env, j->plan_ref);
  napi_delete_async_work(env, j->work);
  job_free_buffers(env, j);
  free(j);
  if (box->finalized) plan_box_free(box);
}

static napi_value extract_async_common(napi_env env, napi_callback_info info, int wav) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) {
    napi_throw_type_error(env, NULL, wav ? "extractWavAsync(plan, wavBytes, features[, channel])"
                                         : "extractAsync(plan, frames, features)");
    return NULL;
  }
  job* j = (job*)calloc(1, sizeof *j);
  j->box = get_plan(env, argv[0]);
  if (!j->box) { free(j); return NULL; }
  if (j->box->busy) {
    free(j);
    napi_throw_error(env, NULL, "plan is busy with an async extraction");
    return NULL;
  }
  if (!(wav ? job_prepare_wav(env, j, argv[1], argv[2], argc > 3 ? argv[3] : NULL)
            : job_prepare(env, j, argv[1], argv[2]))) {
    job_free_buffers(env, j);
    free(j);
    return NULL;
  }
  napi_value promise, name;
  CHECK(napi_create_reference(env, argv[1], 1, &j->frames_ref));  /* keep the input alive */
  CHECK(napi_create_reference(env, argv[0], 1, &j->plan_ref));    /* and the plan */
  CHECK(napi_create_promise(env, &j->deferred, &promise));
  CHECK(napi_create_string_utf8(env, "meyda_extract", NAPI_AUTO_LENGTH, &name));
  CHECK(napi_create_async_work(env, NULL, name, async_execute, async_complete, j, &j->work));
  j->box->busy = 1;
  CHECK(napi_queue_async_work(env, j->work));
  return promise;
}

static napi_value extract_async(napi_env env, napi_callback_info info) { return extract_async_common(env, info, 0); }
static napi_value extract_wav_async(napi_env env, napi_callback_info info) { return extract_async_common(env, info, 1); }

static napi_value wav_parse(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  const unsigned char* data = NULL;
  size_t len = 0;
  if (argc < 1 || !bytes_of(env, argv[0], &data, &len)) return NULL;
  mgx_wav_info wi;
  memset(&wi, 0, sizeof wi);
  wi.struct_size = sizeof wi;
  int rc = mgx_wav_parse(data, len, &wi);
  if (rc) return throw_mgx(env, rc);
  static const char* fmts[] = {"f32", "s16", "u8", "s24", "s32"};
  napi_value obj, v;
  CHECK(napi_create_object(env, &obj));
  CHECK(napi_create_string_utf8(env, fmts[wi.pcm_format], NAPI_AUTO_LENGTH, &v));
  CHECK(napi_set_named_property(env, obj, "pcmFormat", v));
  const struct { const char* k; double v; } nums[] = {
      {"channels", wi.channels}, {"sampleRate", wi.sample_rate}, {"bitsPerSample", wi.bits_per_sample},
      {"blockAlign", wi.block_align}, {"dataOffset", (double)wi.data_offset}, {"dataBytes", (double)wi.data_bytes},
      {"sampleFrames", (double)wi.sample_frames}};
  for (size_t i = 0; i < sizeof nums / sizeof nums[0]; ++i) {
    CHECK(napi_create_double(env, nums[i].v, &v));
    CHECK(napi_set_named_property(env, obj, nums[i].k, v));
  }
  return obj;
}

/* ---------------------------------------------------------------- host tables */
static napi_value host_tables(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  mgx_plan_desc d;
  if (argc) desc_from_opts(env, argv[0], &d);
  else mgx_plan_desc_init(&d);
  const size_t n = d.buffer_size, nf = d.num_mel_bands, nc = d.num_mfcc_coeffs;
  if (n > (1u << 20) || nf > 64 || nc > 64) {
    napi_throw_range_error(env, NULL, "hostTables: size out of range");
    return NULL;
  }
  napi_value ab[7];
  void* p[7];
  size_t sz[7] = {n * 4, n * 4, n * 4, n * 4, 25 * 4, (nf + 2) * 4, nc * nf * 4};
  for (int i = 0; i < 7; ++i) CHECK(napi_create_arraybuffer(env, sz[i], &p[i], &ab[i]));
  mgx_host_tables t = {(float*)p[0], (float*)p[1], (float*)p[2], (float*)p[3], (int32_t*)p[4], (int32_t*)p[5], (float*)p[6]};
  int rc = mgx_get_host_tables(&d, &t);
  if (rc) return throw_mgx(env, rc);
  static const char* keys[7] = {"window", "hanning", "hamming", "barkScale", "barkLimits", "melBins", "dct"};
  napi_value obj;
  CHECK(napi_create_object(env, &obj));
  for (int i = 0; i < 7; ++i) {
    napi_value ta;
    const int is_int = (i == 4 || i == 5);
    CHECK(napi_create_typedarray(env, is_int ? napi_int32_array : napi_float32_array, sz[i] / 4, ab[i], 0, &ta));
    CHECK(napi_set_named_property(env, obj, keys[i], ta));
  }
  return obj;
}

static napi_value is_pow2(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], r;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  double v = 0;
  napi_valuetype t = napi_undefined;
  if (argc) napi_typeof(env, argv[0], &t);
  if (t == napi_number) napi_get_value_double(env, argv[0], &v);
  else v = 0; /* undefined % 2 is NaN in JS: not a power of two */
  CHECK(napi_get_boolean(env, t == napi_number && mgx_is_power_of_two(v), &r));
  return r;
}

static napi_value device_count(napi_env env, napi_callback_info info) {
  (void)info;
  int c = 0;
  mgx_device_count(&c);
  napi_value r;
  CHECK(napi_create_int32(env, c, &r));
  return r;
}

static napi_value feature_names(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value arr;
  CHECK(napi_create_array(env, &arr));
  for (int i = 0; i < MGX_NUM_FEATURES; ++i) {
    napi_value s;
    CHECK(napi_create_string_utf8(env, mgx_feature_name(i), NAPI_AUTO_LENGTH, &s));
    CHECK(napi_set_element(env, arr, i, s));
  }
  return arr;
}

static napi_value feature_info(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], r;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  char name[64] = {0};
  size_t len = 0;
  if (argc) napi_get_value_string_utf8(env, argv[0], name, sizeof name, &len);
  CHECK(napi_create_int32(env, mgx_feature_info(mgx_feature_index(name)), &r));
  return r;
}

static napi_value abi_version(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value r;
  CHECK(napi_create_int32(env, mgx_abi_version(), &r));
  return r;
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"createPlan", NULL, create_plan, NULL, NULL, NULL, napi_enumerable, NULL},
      {"destroyPlan", NULL, destroy_plan, NULL, NULL, NULL, napi_enumerable, NULL},
      {"planBusy", NULL, plan_busy, NULL, NULL, NULL, napi_enumerable, NULL},
      {"extract", NULL, extract_sync, NULL, NULL, NULL, napi_enumerable, NULL},
      {"extractInto", NULL, extract_into, NULL, NULL, NULL, napi_enumerable, NULL},
      {"extractAsync", NULL, extract_async, NULL, NULL, NULL, napi_enumerable, NULL},
      {"extractWav", NULL, extract_wav_sync, NULL, NULL, NULL, napi_enumerable, NULL},
      {"extractWavAsync", NULL, extract_wav_async, NULL, NULL, NULL, napi_enumerable, NULL},
      {"wavParse", NULL, wav_parse, NULL, NULL, NULL, napi_enumerable, NULL},
      {"hostTables", NULL, host_tables, NULL, NULL, NULL, napi_enumerable, NULL},
      {"isPowerOfTwo", NULL, is_pow2, NULL, NULL, NULL, napi_enumerable, NULL},
      {"deviceCount", NULL, device_count, NULL, NULL, NULL, napi_enumerable, NULL},
      {"featureNames", NULL, feature_names, NULL, NULL, NULL, napi_enumerable, NULL},
      {"featureInfo", NULL, feature_info, NULL, NULL, NULL, napi_enumerable, NULL},
      {"abiVersion", NULL, abi_version, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  if (napi_define_properties(env, exports, sizeof props / sizeof props[0], props) != napi_ok) return NULL;
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
