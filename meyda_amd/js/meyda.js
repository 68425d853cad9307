'use strict';
// Meyda-compatible JavaScript facade over the MI355X engine.
//
// Same surface as the reference class (src/meyda.js:15-263):
//   new Meyda(audioContext, source, bufferSize, callback)      src/meyda.js:17-97
//   get(feature | features[])                                  :244-261
//   start(features) / stop()                                   :233-241
//   setSource(source)                                          :229-231
//   featureInfo, windowingFunction, hanning, hamming, barkScale, signal
// plus, for the batched engine:
//   process(signal)                 push one buffer (what onaudioprocess does, :69-91)
//   getBatch(features, frames)      frames: Float32Array(F * bufferSize) -> SoA typed arrays
//   getBatchAsync(features, frames) same, off the JS thread (napi_async_work)
//   getBatchWav(features, wavBytes[, channel]) / getBatchWavAsync(...)
//                                   every full buffer of a .wav file (RIFF walk in C, raw PCM
//                                   decoded on the device: decodeAudioData's scaling)
//   Meyda.readWav(wavBytes)         the header: {pcmFormat, channels, sampleRate, sampleFrames, ...}
//   flush()                         deliver buffered callbacks now (options.batchFrames > 1)
//   options.devices = [0, 1, ...]   shard batches over several GPUs; the feature records are
//                                   gathered to the first one by RCCL (one plan per device)
//   options.asyncPlans = 2          plans per window that async batch jobs run on; more jobs
//                                   queue on them
//
// Streaming (start/stop, src/meyda.js:69-91,233-241): with options.batchFrames = K > 1
// the buffers pushed by process() are queued and extracted K at a time in one launch;
// the callback still runs once per buffer, in order, with that buffer's features
// (latency of up to K buffers for K-fold fewer launches). stop() flushes the queue.
//
// Every built-in feature is computed by libmeyda_gpu.so through the N-API addon.
// Differences from the snapshot (documented in INTEGRATION.md): the FFT runs per
// buffer (the snapshot never transforms, src/meyda.js:79-84; opt back in with
// {mode: 'literal'}), all 18 extractors are registered (src/extractors/index.js
// enables only loudness), the callback works (src/meyda.js:87 references an
// undefined global), and get() returns fresh arrays rather than internal buffers.
const path = require('path');

// (Loading the module changes nothing outside it, like the reference's constructor: the HIP runtime's
// settings are the application's. For the real-time path, HIP_FORCE_DEV_KERNARG=0 in the environment
// that starts the process keeps kernel arguments in host memory -- a ~1.4 us shorter launch call, ~0.6 us
// per one-frame call end to end; INTEGRATION.md, profiles/r05_inline_frame.txt.)
const addon = require(process.env.MEYDA_AMD_ADDON ||
  path.join(__dirname, '..', 'addon', 'meyda_napi.node'));
const FEATURE_INFO = require('./feature-info');

const GPU_FEATURES = new Set(['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness',
  'spectralSlope', 'spectralRolloff', 'spectralSpread', 'spectralSkewness', 'spectralKurtosis',
  'perceptualSpread', 'perceptualSharpness', 'loudness', 'mfcc', 'amplitudeSpectrum',
  'powerSpectrum', 'complexSpectrum']);

// src/utils.js:13-19
function isPowerOfTwo(num) {
  while (((num % 2) === 0) && num > 1) num /= 2;
  return (num == 1); // eslint-disable-line eqeqeq
}

class Meyda {
  constructor(audioContext, src, bufSize, callback, options) {
    // src/meyda.js:20-26: validated in this order, so `bufSize || 256` is unreachable
    if (!isPowerOfTwo(bufSize)) {
      throw new Error('Buffer size is not a power of two: Meyda will not run.');
    }
    if (!audioContext) {
      throw new Error("AudioContext wasn't specified: Meyda will not run.");
    }
    const bufferSize = bufSize || 256;
    this.audioContext = audioContext;
    this.bufferSize = bufferSize;
    this.sampleRate = audioContext.sampleRate;
    this.options = Object.assign({
      precision: 'faithful', mode: 'per_buffer_fft', numMelBands: 26, numMfccCoeffs: 13, device: 0,
      batchFrames: 1,
    }, options || {});
    this._ring = null;        // queued buffers (batchFrames > 1)
    this._flushing = null;    // the ring whose frames a flush is delivering
    this._layouts = new Map(); // extractViews' output layouts, per (fields, frames)
    this._ringCount = 0;
    this.featureExtractors = {}; // user plugins: fn(bufferSize, m) or {process(signal)}
    this.EXTRACTION_STARTED = false;
    this._featuresToExtract = null;
    this._callback = callback;
    this.windowingFunction = 'hanning';
    const t = addon.hostTables({ bufferSize, sampleRate: this.sampleRate,
      numMelBands: this.options.numMelBands, numMfccCoeffs: this.options.numMfccCoeffs });
    this.barkScale = t.barkScale;
    this.hanning = t.hanning;
    this.hamming = t.hamming;
    this.featureInfo = Object.assign({}, FEATURE_INFO);
    this.signal = null;
    this._plans = {};       // streaming / sync plan per window
    this._asyncPlans = {};  // per window: plans that async batch jobs run on (never the streaming one)
    this._frame = null; // results of the current buffer, filled lazily by get()
    // Web Audio wiring when the context provides it (src/meyda.js:67-94). One node per
    // instance (the reference stored it on a window global).
    if (typeof audioContext.createScriptProcessor === 'function') {
      this.spn = audioContext.createScriptProcessor(bufferSize, 1, 1);
      this.spn.onaudioprocess = (e) => this.process(e.inputBuffer.getChannelData(0));
      if (typeof this.spn.connect === 'function' && audioContext.destination) {
        this.spn.connect(audioContext.destination);
      }
      if (src && typeof src.connect === 'function') src.connect(this.spn, 0, 0);
    }
  }

  // `signal`: the current buffer (src/meyda.js:70). In a batched callback it is a view of the queued
  // frames, made on first read.
  get signal() {
    if (this._sigBatch) {
      const i = this._sigIndex, N = this.bufferSize;
      this._sig = this._sigBatch.subarray(i * N, i * N + N);
      this._sigBatch = null;
    }
    return this._sig;
  }

  set signal(v) {
    this._sig = v;
    this._sigBatch = null;
  }

  _window() {
    const w = this.windowingFunction;
    if (w !== 'hanning' && w !== 'hamming') {
      throw new TypeError('unknown windowingFunction "' + w + '"');
    }
    return w;
  }

  _newPlan(w) {
    return addon.createPlan({
      bufferSize: this.bufferSize, sampleRate: this.sampleRate, windowingFunction: w,
      precision: this.options.precision, mode: this.options.mode,
      numMelBands: this.options.numMelBands, numMfccCoeffs: this.options.numMfccCoeffs,
      device: this.options.device, scalarF64: 1,
      // options.mfccReferenceOrder: mel sums, log and DCT in mfcc.js's own order (bit-identical MFCC)
      mfccReferenceOrder: this.options.mfccReferenceOrder ? 1 : 0,
      // options.resident: one-buffer calls (the per-buffer process()/get() path) served by a workgroup that
      // stays on the device between buffers instead of one launch per buffer (include/meyda_gpu.h
      // MGX_FLAG_RESIDENT); one device, faithful per-buffer plans without mfccReferenceOrder
      resident: this.options.resident && !Array.isArray(this.options.devices) ? 1 : 0,
      // options.devices = [d0, d1, ...]: every batch is sharded over the devices and the
      // per-frame features are gathered to d0 over xGMI (RCCL), include/meyda_gpu.h mgx_group_*
      ...(Array.isArray(this.options.devices) ? { devices: this.options.devices } : {}),
    });
  }

  // One plan per window type, created on first use (windowingFunction may change at
  // runtime as in the reference, src/meyda.js:41,76,164). process()/get()/getBatch() run on it.
  _plan() {
    const w = this._window();
    if (!this._plans[w]) this._plans[w] = this._newPlan(w);
    return this._plans[w];
  }

  // Async batch jobs own their plan for the whole job (the addon marks it busy), so they
  // never run on the streaming plan: per window, a pool of at most options.asyncPlans plans
  // (default 2; with options.devices each one is a whole device group with its RCCL
  // communicators), so onaudioprocess buffers and a second async batch proceed while a job
  // is in flight. Further jobs queue on the pooled plan with the fewest pending jobs.
  _runAsync(job) {
    const w = this._window();
    const pool = this._asyncPlans[w] || (this._asyncPlans[w] = []);
    const cap = Math.max(1, this.options.asyncPlans | 0 || 2);
    let slot = pool.find((sl) => sl.pending === 0);
    if (!slot && pool.length < cap) {
      slot = { plan: this._newPlan(w), pending: 0, tail: Promise.resolve() };
      pool.push(slot);
    }
    if (!slot) slot = pool.reduce((a, b) => (b.pending < a.pending ? b : a));
    slot.pending++;
    const run = () => job(slot.plan);
    const res = slot.tail.then(run, run);
    const done = () => { slot.pending--; };
    slot.tail = res.then(done, done);
    return res;
  }

  // The per-buffer handler (src/meyda.js:69-91): take the buffer, then deliver the
  // started features to the callback.
  process(signal) {
    if (!(signal instanceof Float32Array)) signal = Float32Array.from(signal);
    if (signal.length !== this.bufferSize) {
      throw new RangeError('buffer length ' + signal.length + ' != bufferSize ' + this.bufferSize);
    }
    this.signal = signal;
    this._frame = null;
    if (typeof this._callback !== 'function' || !this.EXTRACTION_STARTED) return;
    const K = this.options.batchFrames | 0;
    if (K <= 1) {
      this._callback(this.get(this._featuresToExtract));
      return;
    }
    if (!this._ring || this._ring === this._flushing || this._ring.length !== K * this.bufferSize) {
      this._ring = new Float32Array(K * this.bufferSize);
    }
    this._ring.set(signal, this._ringCount * this.bufferSize);
    if (++this._ringCount === K) this.flush();
  }

  // Extract every queued buffer in one launch and run the callback for each, in order.
  flush() {
    const count = this._ringCount;
    if (!count) return;
    this._ringCount = 0;
    const list = this._featuresToExtract;
    const names = typeof list === 'string' ? [list] : Array.prototype.slice.call(list || []);
    const plugins = names.some((n) => this.featureExtractors[n]);
    if (!plugins && names.every((n) => GPU_FEATURES.has(n) || n === 'buffer')) {
      this._flushViews(count, list, names);
      return;
    }
    const gpu = names.filter((n) => GPU_FEATURES.has(n) && !this.featureExtractors[n]);
    if (plugins) gpu.push('amplitudeSpectrum', 'complexSpectrum', 'loudness');
    const N = this.bufferSize;
    const frames = this._ring.slice(0, count * N);
    const r = gpu.length ? addon.extract(this._plan(), frames, gpu) : {};
    const keep = this.signal;
    for (let i = 0; i < count; i++) {
      const sig = frames.subarray(i * N, (i + 1) * N);
      this.signal = sig;
      this._frame = {};
      for (const n of new Set(gpu)) this._frame[n] = frameValue(n, r, i, N, this.options.numMfccCoeffs);
      const out = typeof list === 'string' ? this._value(list) : this.get(names);
      this._callback(out);
    }
    this.signal = keep;
    this._frame = null;
  }

  // flush() for built-in features only: one launch, then each callback gets its frame's values as
  // views into the batch's result arrays (numbers, and subarrays where get() returns arrays), built by
  // one compiled object literal per feature list (frameBuilder) instead of per-frame copies and a get()
  // dispatch per buffer. The batch's result arrays are fresh per launch, so a view stays valid after its
  // callback. `signal` is a view of the queued frames, made only if read (the ring is reused by the
  // next batch); 'buffer' is a copy of the frame.
  _flushViews(count, list, names) {
    const N = this.bufferSize, nc = this.options.numMfccCoeffs || 13;
    const frames = this._ring.subarray(0, count * N);
    this._flushing = this._ring;  // (a process() from a callback starts a new ring: these frames stay put)
    const gpu = Array.from(new Set(names.filter((n) => n !== 'buffer')));
    const r = gpu.length ? extractViews(this._layouts, this._plan(), frames, gpu, N, nc) : {};
    const keep = this.signal;
    const cb = this._callback;
    const build = frameBuilder(typeof list === 'string' ? null : names, typeof list === 'string' ? list : null);
    for (let i = 0; i < count; i++) {
      this._sigBatch = frames;
      this._sigIndex = i;
      this._frame = null;
      cb(build(r, frames, i, N, nc));
    }
    this._flushing = null;
    this.signal = keep;
    this._frame = null;
  }

  setSource(_src) {
    _src.connect(this.spn);
  }

  start(features) {
    this._featuresToExtract = features;
    this.EXTRACTION_STARTED = true;
  }

  stop() {
    if (this._ringCount) this.flush();  // queued buffers are still delivered
    this._featuresToExtract = null;
    this.EXTRACTION_STARTED = false;
  }

  // src/meyda.js:244-261
  get(feature) {
    if (typeof feature === 'object') {
      const names = Array.prototype.slice.call(feature); // null throws, as feature.length does
      const gpu = [];
      for (let x = 0; x < names.length; x++) {
        const n = names[x];
        if (GPU_FEATURES.has(n) && !this.featureExtractors[n]) gpu.push(n);
      }
      try {  // one launch for all built-in features; a failure resurfaces per feature below
        this._compute(gpu);
      } catch (e) { /* logged per feature, as the reference does */ }
      const results = {};
      for (let x = 0; x < names.length; x++) {
        try {
          results[names[x]] = this._value(names[x]);
        } catch (e) {
          console.error(e);
        }
      }
      return results;
    } else if (typeof feature === 'string') {
      return this._value(feature);
    }
    throw new Error('Invalid Feature Format');
  }

  _signal() {
    return this.signal || new Float32Array(this.bufferSize);
  }

  // Compute the missing GPU features of the current buffer in one launch.
  _compute(names) {
    const fr = this._frame || (this._frame = {});
    const need = [];
    for (let x = 0; x < names.length; x++) if (!(names[x] in fr)) need.push(names[x]);
    if (!need.length) return;
    // (into the layout's scratch buffer: frameValue copies every value out before anything else runs)
    const r = extractViews(this._layouts, this._plan(), this._signal(), need, this.bufferSize, this.options.numMfccCoeffs,
      true);
    for (const n of need) this._frame[n] = frameValue(n, r, 0, this.bufferSize, this.options.numMfccCoeffs);
  }

  _value(name) {
    const plugin = this.featureExtractors[name];
    if (plugin) return this._runPlugin(plugin);
    const fr = this._frame;
    if (fr && name in fr) return fr[name];  // this buffer's launch computed it
    if (name === 'buffer') return this._signal();
    if (!GPU_FEATURES.has(name)) {
      throw new TypeError("Cannot read property 'process' of undefined (feature '" + name + "')");
    }
    this._compute([name]);
    return this._frame[name];
  }

  // A user extractor sees the same `m` the reference extractors see
  // (SURVEY.md §8(b)): signal, ampSpectrum, complexSpectrum, audioContext, featureExtractors.
  _runPlugin(plugin) {
    if (typeof plugin.process === 'function') return plugin.process(this._signal());
    this._compute(['amplitudeSpectrum', 'complexSpectrum', 'loudness']);
    const m = {
      signal: this._signal(),
      ampSpectrum: this._frame.amplitudeSpectrum,
      complexSpectrum: this._frame.complexSpectrum,
      audioContext: this.audioContext,
      featureExtractors: Object.assign({ loudness: () => this._frame.loudness }, this.featureExtractors),
    };
    return plugin(this.bufferSize, m);
  }

  // Batch API: frames is a Float32Array holding F consecutive buffers.
  getBatch(features, frames) {
    const names = checkBatchNames(features);
    return addon.extract(this._plan(), toF32(frames), names);
  }

  getBatchAsync(features, frames) {
    const names = checkBatchNames(features);
    const x = toF32(frames);
    return this._runAsync((plan) => addon.extractAsync(plan, x, names));
  }

  // Every full buffer of a .wav file (Buffer / Uint8Array / ArrayBuffer), channel `channel`.
  getBatchWav(features, wavBytes, channel) {
    return addon.extractWav(this._plan(), wavBytes, checkBatchNames(features), channel | 0);
  }

  getBatchWavAsync(features, wavBytes, channel) {
    const names = checkBatchNames(features);
    return this._runAsync((plan) => addon.extractWavAsync(plan, wavBytes, names, channel | 0));
  }

  static readWav(wavBytes) {
    return addon.wavParse(wavBytes);
  }

  // Per-frame view of a batch result, in the shapes get() returns.
  static frame(result, name, index, bufferSize, numMfccCoeffs) {
    return frameValue(name, result, index, bufferSize, numMfccCoeffs);
  }

  // Frees the device plans now. A plan an async job still owns is left to that job: the
  // addon keeps it alive until the job settles and the GC then frees it.
  dispose() {
    const all = Object.values(this._plans);
    // (a pooled plan with jobs still queued on it is left to them, like a busy one)
    for (const pool of Object.values(this._asyncPlans)) all.push(...pool.filter((sl) => sl.pending === 0).map((sl) => sl.plan));
    for (const p of all) if (!addon.planBusy(p)) addon.destroyPlan(p);
    this._plans = {};
    this._asyncPlans = {};
  }
}

// The output fields of the C ABI in mgx_outputs order (the addon's extractInto offsets) and the result
// keys each requested feature fills.
const FIELDS = ['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness', 'spectralSlope', 'spectralRolloff',
  'spectralSpread', 'spectralSkewness', 'spectralKurtosis', 'loudness.total', 'perceptualSpread', 'perceptualSharpness',
  'loudness.specific', 'mfcc', 'amplitudeSpectrum', 'powerSpectrum', 'complexSpectrum.real', 'complexSpectrum.imag'];
const KEYS_OF = { loudness: ['loudness.specific', 'loudness.total'],
  complexSpectrum: ['complexSpectrum.real', 'complexSpectrum.imag'] };

// Output-field bits of each feature name (its FIELDS entries).
const FIELD_BITS = {};
FIELDS.forEach((k, i) => { FIELD_BITS[k] = 2 ** i; });
FIELD_BITS.loudness = FIELD_BITS['loudness.specific'] + FIELD_BITS['loudness.total'];
FIELD_BITS.complexSpectrum = FIELD_BITS['complexSpectrum.real'] + FIELD_BITS['complexSpectrum.imag'];

// Extraction of F frames into one ArrayBuffer (addon.extractInto), its layout worked out once per
// (output fields, F) and kept in the instance's `cache`: a result object of typed-array views with
// extract()'s keys and shapes (scalars as Float64Array: the facade's plans use scalarF64). One
// allocation and a few N-API calls per launch instead of an ArrayBuffer, a reference and a typed array
// per output (the real-time paths).
function extractViews(cache, plan, frames, names, N, nc, scratch) {
  const F = frames.length / N;
  let bits = 0;
  for (let j = 0; j < names.length; j++) bits += FIELD_BITS[names[j]] || 0;  // (names are distinct)
  const key = F < 4194304 ? bits * 4194304 + F : bits + ':' + F;
  let lay = cache.get(key);
  if (!lay) {
    const per = (i) => (i < 13 ? 1 : i === 13 ? 24 : i === 14 ? nc : i < 17 ? N / 2 : N);
    const offsets = new Float64Array(19).fill(-1);
    const views = [];
    let at = 0;
    FIELDS.forEach((k, i) => {
      if (!(Math.floor(bits / 2 ** i) % 2)) return;
      const len = F * per(i), bytes = len * (i < 13 ? 8 : 4);
      offsets[i] = at;
      views.push([k, i < 13 ? Float64Array : Float32Array, at, len]);
      at += Math.ceil(bytes / 8) * 8;
    });
    lay = { offsets, views, bytes: Math.max(at, 8) };
    if (cache.size > 256) cache.clear();
    cache.set(key, lay);
  }
  // scratch: the layout's own buffer and views, reused call after call (get(): the values are copied out at
  // once); otherwise a fresh buffer whose views the caller may keep (the batched callbacks)
  if (scratch && lay.scratch) {
    addon.extractInto(plan, frames, lay.offsets, lay.scratch.ab);
    return lay.scratch.r;
  }
  const ab = new ArrayBuffer(lay.bytes);
  addon.extractInto(plan, frames, lay.offsets, ab);
  const r = {};
  const v = lay.views;
  for (let j = 0; j < v.length; j++) r[v[j][0]] = new v[j][1](ab, v[j][2], v[j][3]);
  if (scratch) lay.scratch = { ab, r };
  return r;
}

// A batched callback's value for frame i, compiled once per feature list: an object literal (or, for a
// single name, the bare value) whose entries read the batch's result arrays -- numbers, and subarray
// views where get() returns arrays -- so a callback costs an allocation, not a dispatch per feature.
const BUILDERS = new Map();
function frameBuilder(names, single) {
  const key = single !== null ? '=' + single : names.join('\u0000');
  let f = BUILDERS.get(key);
  if (f) return f;
  const expr = (n) => {
    switch (n) {
      case 'buffer': return 'x.slice(i * N, i * N + N)';
      case 'loudness': return "{ specific: r['loudness.specific'].subarray(i * 24, i * 24 + 24), total: r['loudness.total'][i] }";
      case 'mfcc': return 'r.mfcc.subarray(i * nc, i * nc + nc)';
      case 'amplitudeSpectrum': case 'powerSpectrum': return 'r.' + n + '.subarray(i * (N >> 1), i * (N >> 1) + (N >> 1))';
      case 'complexSpectrum': return "{ real: r['complexSpectrum.real'].subarray(i * N, i * N + N), " +
        "imag: r['complexSpectrum.imag'].subarray(i * N, i * N + N), length: N }";
      default: return 'r[' + JSON.stringify(n) + '][i]';
    }
  };
  const body = single !== null ? expr(single)
    : '{ ' + names.map((n) => JSON.stringify(n) + ': ' + expr(n)).join(', ') + ' }';
  f = new Function('r', 'x', 'i', 'N', 'nc', 'return (' + body + ');');  // eslint-disable-line no-new-func
  BUILDERS.set(key, f);
  return f;
}

function toF32(frames) {
  return frames instanceof Float32Array ? frames : Float32Array.from(frames);
}

function checkBatchNames(features) {
  const names = typeof features === 'string' ? [features] : Array.prototype.slice.call(features);
  for (const n of names) {
    if (!GPU_FEATURES.has(n)) throw new TypeError("unknown batch feature '" + n + "'");
  }
  return names;
}

// Slice frame `i` of a SoA batch result into the reference's return shapes
// (src/feature-info.js): numbers, Float32Array, {specific, total}, {real, imag}.
function frameValue(name, r, i, n, ncoef) {
  ncoef = ncoef || 13;
  const L = n / 2;
  switch (name) {
    case 'loudness':
      return { specific: r['loudness.specific'].slice(i * 24, i * 24 + 24), total: r['loudness.total'][i] };
    case 'mfcc':
      return r.mfcc.slice(i * ncoef, i * ncoef + ncoef);
    case 'amplitudeSpectrum':
      return r.amplitudeSpectrum.slice(i * L, i * L + L);
    case 'powerSpectrum':
      return r.powerSpectrum.slice(i * L, i * L + L);
    case 'complexSpectrum': {
      const real = r['complexSpectrum.real'].slice(i * n, i * n + n);
      const imag = r['complexSpectrum.imag'].slice(i * n, i * n + n);
      return { real, imag, length: n };
    }
    default:
      return r[name][i];
  }
}

module.exports = Meyda;
module.exports.Meyda = Meyda;
module.exports.isPowerOfTwo = isPowerOfTwo;
module.exports.featureInfo = FEATURE_INFO;
module.exports.addon = addon;
