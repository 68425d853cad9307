'use strict';
// Host-side checks of the Meyda facade (no GPU needed): constructor validation in the
// reference's order (src/meyda.js:20-26), isPowerOfTwo (src/utils.js:13-19), the
// tables exposed on the instance vs the reference's own (golden), featureInfo,
// get() dispatch errors (src/meyda.js:244-261), and that feature computation fails
// loudly when no device is present (there is no CPU fallback).
const assert = require('assert');
const path = require('path');
const golden = require('./golden');
const kernargPreset = process.env.HIP_FORCE_DEV_KERNARG;
const envBefore = Object.assign({}, process.env);
const Meyda = require(path.join(__dirname, '..', '..', 'meyda_amd', 'js', 'meyda.js'));

const ctx = { sampleRate: 44100 };
let n = 0;
function check(name, fn) { fn(); n++; console.log('ok ' + name); }

check('isPowerOfTwo', () => {
  for (const v of [1, 2, 256, 512, 1024, 2048, 1 << 20]) assert.strictEqual(Meyda.isPowerOfTwo(v), true);
  for (const v of [0, 3, 6, 1000, 0.5, undefined, NaN]) assert.strictEqual(Meyda.isPowerOfTwo(v), false);
  for (const v of [0, 1, 2, 3, 512, 1000, 1024]) {
    assert.strictEqual(Meyda.addon.isPowerOfTwo(v), Meyda.isPowerOfTwo(v), 'addon vs JS at ' + v);
  }
});

check('constructor errors in reference order', () => {
  assert.throws(() => new Meyda(ctx, null, 1000), /Buffer size is not a power of two: Meyda will not run./);
  assert.throws(() => new Meyda(ctx, null, undefined), /Buffer size is not a power of two/);
  // the size check runs first, even without a context
  assert.throws(() => new Meyda(null, null, 1000), /not a power of two/);
  assert.throws(() => new Meyda(null, null, 512), /AudioContext wasn't specified: Meyda will not run./);
});

check('tables match the reference (golden)', () => {
  for (const N of [512, 1024, 2048]) {
    const g = golden.load(N);
    const m = new Meyda(ctx, null, N);
    assert.deepStrictEqual(Array.from(m.hanning), Array.from(g.hann));
    assert.deepStrictEqual(Array.from(m.hamming), Array.from(g.hamming));
    assert.deepStrictEqual(Array.from(m.barkScale), Array.from(g.bark));
    assert.strictEqual(m.bufferSize, N);
    assert.strictEqual(m.sampleRate, 44100);
    assert.strictEqual(m.windowingFunction, 'hanning');
  }
});

check('featureInfo', () => {
  const m = new Meyda(ctx, null, 512);
  assert.deepStrictEqual(m.featureInfo.rms, { type: 'number' });
  assert.strictEqual(m.featureInfo.loudness.type, 'multipleArrays');
  assert.deepStrictEqual(m.featureInfo.loudness.arrayNames, { 1: 'total', 2: 'specific' });
  assert.strictEqual(m.featureInfo.mfcc.type, 'array');
  const names = Meyda.addon.featureNames();
  for (const k of names) if (k.indexOf('.') < 0) assert.ok(k in m.featureInfo, k);
});

check('get dispatch', () => {
  const m = new Meyda(ctx, null, 512);
  assert.throws(() => m.get(42), /Invalid Feature Format/);
  assert.throws(() => m.get('noSuchFeature'), TypeError);
  const x = new Float32Array(512).map((_, i) => Math.sin(i));
  m.process(x);
  assert.strictEqual(m.get('buffer'), m.signal);
  // a user plugin of the object style runs on the CPU side with the frame's signal
  m.featureExtractors.peak = { process: (s) => s.reduce((a, v) => Math.max(a, Math.abs(v)), 0) };
  assert.strictEqual(m.get('peak'), x.reduce((a, v) => Math.max(a, Math.abs(v)), 0));
});

check('no CPU fallback', () => {
  if (Meyda.addon.deviceCount() > 0) return;  // (a GPU is present: covered by facade_gpu.js)
  const m = new Meyda(ctx, null, 512);
  m.process(new Float32Array(512));
  assert.throws(() => m.get('rms'), /device|HIP|gfx950/);
  assert.throws(() => m.getBatch(['rms'], new Float32Array(1024)), /device|HIP|gfx950/);
  // get(array) logs each failing feature and omits it, as src/meyda.js:246-255 does
  const err = console.error;
  let logged = 0;
  console.error = () => { logged++; };
  try {
    assert.deepStrictEqual(m.get(['rms', 'zcr']), {});
  } finally {
    console.error = err;
  }
  assert.strictEqual(logged, 2);
});

check('readWav (RIFF walk in the library, no device)', () => {
  const { wavS16 } = require('./wav');
  const codes = new Int16Array(2 * 3000).map((_, i) => (i * 37) % 2000 - 1000);
  const info = Meyda.readWav(wavS16(codes, 2, 22050));
  assert.strictEqual(info.pcmFormat, 's16');
  assert.strictEqual(info.channels, 2);
  assert.strictEqual(info.sampleRate, 22050);
  assert.strictEqual(info.sampleFrames, 3000);
  assert.strictEqual(info.dataOffset, 12 + 8 + 16 + 8 + 4 + 8);
  assert.throws(() => Meyda.readWav(Buffer.from('not a wav file at all')), /RIFF/);
});

check('bufferSize 1 and 2 construct (isPowerOfTwo accepts them; tables only)', () => {
  for (const N of [1, 2]) {
    const m = new Meyda(ctx, null, N);
    assert.strictEqual(m.hanning.length, N);
    assert.strictEqual(m.barkScale.length, N);
  }
  const t = Meyda.addon.hostTables({ bufferSize: 1 });
  assert.strictEqual(t.barkLimits[24], -1);  // loudness.js:44: normalisedSpectrum.length - 1
});

check('loading the facade and constructing Meyda leave process.env as it was', () => {
  // (src/meyda.js:17-97: construction has no global side effect beyond its ScriptProcessor; the HIP
  // runtime's settings, HIP_FORCE_DEV_KERNARG among them, are the application's)
  assert.strictEqual(process.env.HIP_FORCE_DEV_KERNARG, kernargPreset);
  const now = Object.assign({}, process.env);
  // (GLOG_*: set by the ROCm runtime's own librocprofiler-register when the HIP runtime loads, not by this code)
  const changed = Object.keys(Object.assign({}, now, envBefore))
    .filter((k) => now[k] !== envBefore[k] && !k.startsWith('GLOG_'));
  assert.deepStrictEqual(changed, [], 'environment keys changed: ' + changed.join(', '));
});

console.log('facade_cpu: ' + n + ' checks passed');
