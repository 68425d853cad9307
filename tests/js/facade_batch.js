'use strict';
// Host-side checks of the facade's batched streaming delivery (meyda.js flush / _flushViews /
// frameBuilder) against a stand-in addon (tests/js/mock_addon.js): which frame each callback's values
// come from, that views outlive their batch, 'buffer' and `signal`, a single-name list, a callback that
// pushes buffers itself, and one launch per batch. The GPU results themselves: tests/js/facade_gpu.js.
process.env.MEYDA_AMD_ADDON = require('path').join(__dirname, 'mock_addon.js');
const assert = require('assert');
const path = require('path');
const mock = require('./mock_addon');
const Meyda = require(path.join(__dirname, '..', '..', 'meyda_amd', 'js', 'meyda.js'));

const ctx = { sampleRate: 44100 };
let n = 0;
function check(name, fn) { fn(); n++; console.log('ok ' + name); }
const N = 256;
const frame = (k) => { const x = new Float32Array(N); x.fill(k / 8); x[0] = k; return x; };

check('every callback gets its own frame, one launch per batch, views valid after later batches', () => {
  const seen = [];
  const list = ['rms', 'zcr', 'loudness', 'mfcc', 'amplitudeSpectrum', 'complexSpectrum', 'buffer'];
  const m = new Meyda(ctx, null, N, (f) => seen.push({ f, sig: m.signal }), { batchFrames: 4 });
  mock.calls.length = 0;
  m.start(list);
  for (let k = 0; k < 10; k++) m.process(frame(k));
  m.stop();
  assert.strictEqual(seen.length, 10);
  assert.deepStrictEqual(mock.calls.map((c) => c.F), [4, 4, 2]);
  seen.forEach(({ f }, k) => {
    assert.strictEqual(f.rms, k + 0);
    assert.strictEqual(f.zcr, k + 2);
    assert.strictEqual(f.loudness.total, k + 99);
    assert.deepStrictEqual(Array.from(f.loudness.specific), Array.from({ length: 24 }, (_, j) => k + 100 + j));
    assert.deepStrictEqual(Array.from(f.mfcc), Array.from({ length: 13 }, (_, j) => k + 200 + j));
    assert.strictEqual(f.amplitudeSpectrum.length, N / 2);
    assert.strictEqual(f.amplitudeSpectrum[5], k + 305);
    assert.strictEqual(f.complexSpectrum.real[7], k + 407);
    assert.strictEqual(f.complexSpectrum.imag[7], k + 507);
    assert.strictEqual(f.complexSpectrum.length, N);
    assert.deepStrictEqual(Array.from(f.buffer), Array.from(frame(k)));  // a copy: the ring is reused
  });
});

check('signal is the delivered buffer during its callback and the last pushed one after', () => {
  const sig = [];
  const m = new Meyda(ctx, null, N, () => sig.push(Array.from(m.signal)), { batchFrames: 3 });
  m.start(['rms']);
  for (let k = 0; k < 6; k++) m.process(frame(k));
  m.stop();
  sig.forEach((s, k) => assert.deepStrictEqual(s, Array.from(frame(k))));
  assert.deepStrictEqual(Array.from(m.signal), Array.from(frame(5)));
});

check('a single feature name delivers the bare value', () => {
  const got = [];
  const m = new Meyda(ctx, null, N, (v) => got.push(v), { batchFrames: 4 });
  m.start('spectralCentroid');
  for (let k = 0; k < 5; k++) m.process(frame(k));
  m.stop();
  assert.deepStrictEqual(got, [3, 4, 5, 6, 7]);
});

check('a callback that pushes buffers itself does not disturb the batch being delivered', () => {
  const got = [];
  let inner = 0;
  const m = new Meyda(ctx, null, N, (f) => {
    got.push([f.rms, m.signal[0]]);
    if (inner < 3) m.process(frame(100 + inner++));  // re-entrant push into a new ring
  }, { batchFrames: 4 });
  m.start(['rms']);
  for (let k = 0; k < 4; k++) m.process(frame(k));
  assert.deepStrictEqual(got.slice(0, 4), [[0, 0], [1, 1], [2, 2], [3, 3]]);
  m.stop();  // flushes the 3 buffers the callbacks pushed
  assert.deepStrictEqual(got.slice(4), [[100, 100], [101, 101], [102, 102]]);
});

console.log('facade_batch: ' + n + ' checks passed');
