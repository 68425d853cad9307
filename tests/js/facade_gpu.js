'use strict';
// GPU checks of the Meyda facade through the N-API addon: per-buffer get() against the
// reference's own outputs (tests/golden), the batch API against get(), start()/stop()
// streaming, the hamming window switch and literal mode. Needs an MI355X.
const assert = require('assert');
const path = require('path');
const golden = require('./golden');
const Meyda = require(path.join(__dirname, '..', '..', 'meyda_amd', 'js', 'meyda.js'));

const ctx = { sampleRate: 44100 };
const SCALARS = ['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness', 'spectralSlope',
  'spectralRolloff', 'spectralSpread', 'spectralSkewness', 'spectralKurtosis'];
const ALL = SCALARS.concat(['loudness', 'perceptualSpread', 'perceptualSharpness', 'mfcc', 'amplitudeSpectrum']);
let n = 0;
const checks = [];
function check(name, fn) { checks.push([name, fn]); }
process.on('unhandledRejection', (e) => { console.error(e); process.exit(1); });
function close(a, b, rtol, atol, what) {
  if (Number.isNaN(b)) { assert.ok(Number.isNaN(a), what + ': expected NaN, got ' + a); return; }
  if (!Number.isFinite(b)) { assert.strictEqual(a, b, what); return; }
  assert.ok(Math.abs(a - b) <= rtol * Math.abs(b) + (atol || 0), what + ': ' + a + ' vs ' + b);
}
function frameOf(g, i) { return g.input.subarray(i * g.N, (i + 1) * g.N); }
function vecClose(a, b, what) {
  let mx = 0;
  for (const v of b) if (Number.isFinite(v)) mx = Math.max(mx, Math.abs(v));
  for (let i = 0; i < b.length; i++) close(a[i], b[i], 1e-5, 1e-5 * mx, what + '[' + i + ']');
}

const g = golden.load(512);
const S = g.scalarNames.length;

check('C1: get([rms, spectralCentroid]) on sound1 frame 0', () => {
  const i = g.labels.indexOf('sound1:0');
  assert.ok(i >= 0);
  const m = new Meyda(ctx, null, 512);
  m.process(frameOf(g, i));
  const r = m.get(['rms', 'spectralCentroid']);
  close(r.rms, g.scalars[i * S + 0], 1e-5, 0, 'rms');
  close(r.spectralCentroid, g.scalars[i * S + 3], 1e-5, 0, 'centroid');
  m.dispose();
});

check('mfccReferenceOrder: the reference MFCC bits on noise frames (bit-exact spectra)', () => {
  const m = new Meyda(ctx, null, 512, null, { mfccReferenceOrder: true });
  let frames = 0;
  for (let i = 0; i < g.F; i++) {
    if (!g.labels[i].startsWith('noise')) continue;
    m.process(frameOf(g, i));
    const r = m.get('mfcc');
    const ref = g.mfcc.subarray(i * 13, i * 13 + 13);
    for (let c = 0; c < 13; c++) assert.ok(Object.is(r[c], ref[c]), g.labels[i] + ' mfcc[' + c + ']: ' + r[c] + ' vs ' + ref[c]);
    frames++;
  }
  assert.ok(frames > 0);
  m.dispose();
});

check('per-buffer get() vs reference on noise and wav frames', () => {
  const m = new Meyda(ctx, null, 512);
  let frames = 0;
  for (let i = 0; i < g.F; i++) {
    const lab = g.labels[i];
    if (!(lab.startsWith('noise') || lab.startsWith('sound'))) continue;
    m.process(frameOf(g, i));
    const r = m.get(ALL);
    assert.strictEqual(r.zcr, g.scalars[i * S + 2], 'zcr exact');
    for (const [k, j] of [['rms', 0], ['energy', 1], ['spectralCentroid', 3], ['spectralFlatness', 4],
      ['spectralRolloff', 6], ['spectralSpread', 7], ['perceptualSpread', 11], ['perceptualSharpness', 12]]) {
      close(r[k], g.scalars[i * S + j], 1e-5, 0, lab + ' ' + k);
    }
    close(r.loudness.total, g.scalars[i * S + 10], 1e-5, 0, lab + ' loudness.total');
    vecClose(r.loudness.specific, g.loudness_specific.subarray(i * 24, i * 24 + 24), lab + ' specific');
    vecClose(r.mfcc, g.mfcc.subarray(i * 13, i * 13 + 13), lab + ' mfcc');
    vecClose(r.amplitudeSpectrum, g.amp.subarray(i * 256, i * 256 + 256), lab + ' amp');
    assert.ok(r.amplitudeSpectrum instanceof Float32Array && r.mfcc instanceof Float32Array);
    frames++;
  }
  assert.ok(frames > 50);
  m.dispose();
});

check('getBatch / getBatchAsync equal per-buffer get()', () => {
  const m = new Meyda(ctx, null, 512);
  const F = 40;
  const x = g.input.subarray(0, F * 512);
  const b = m.getBatch(ALL, x);
  for (let i = 0; i < F; i += 7) {
    m.process(frameOf(g, i));
    const r = m.get(ALL);
    for (const k of SCALARS) assert.strictEqual(Meyda.frame(b, k, i, 512), r[k], k);
    assert.deepStrictEqual(Array.from(Meyda.frame(b, 'mfcc', i, 512)), Array.from(r.mfcc));
    assert.deepStrictEqual(Meyda.frame(b, 'loudness', i, 512).total, r.loudness.total);
  }
  return m.getBatchAsync(ALL, x).then((a) => {
    for (const k of SCALARS) assert.deepStrictEqual(Array.from(a[k]), Array.from(b[k]), 'async ' + k);
    m.dispose();
  });
});

check('start()/stop() streaming callback', () => {
  const seen = [];
  const m = new Meyda(ctx, null, 512, (feat) => seen.push(feat));
  m.process(frameOf(g, 0));             // not started: no callback
  m.start(['rms', 'zcr']);
  for (let i = 0; i < 5; i++) m.process(frameOf(g, i));
  m.stop();
  m.process(frameOf(g, 5));             // stopped: no callback
  assert.strictEqual(seen.length, 5);
  for (let i = 0; i < 5; i++) {
    assert.deepStrictEqual(Object.keys(seen[i]).sort(), ['rms', 'zcr']);
    assert.strictEqual(seen[i].zcr, g.scalars[i * S + 2]);
  }
  m.dispose();
});

check('batched streaming (batchFrames = 4): callbacks per buffer, in order, equal to get()', () => {
  const seen = [];
  const m = new Meyda(ctx, null, 512, (feat) => seen.push(feat), { batchFrames: 4 });
  const list = ['rms', 'zcr', 'spectralCentroid', 'mfcc', 'loudness'];
  m.start(list);
  for (let i = 0; i < 10; i++) m.process(frameOf(g, i));
  assert.strictEqual(seen.length, 8);           // two full batches delivered
  m.stop();                                     // the last 2 queued buffers are flushed
  assert.strictEqual(seen.length, 10);
  const ref = new Meyda(ctx, null, 512);
  for (let i = 0; i < 10; i++) {
    ref.process(frameOf(g, i));
    const r = ref.get(list);
    for (const k of ['rms', 'zcr', 'spectralCentroid']) assert.strictEqual(seen[i][k], r[k], k + ' frame ' + i);
    assert.deepStrictEqual(Array.from(seen[i].mfcc), Array.from(r.mfcc));
    assert.strictEqual(seen[i].loudness.total, r.loudness.total);
  }
  m.dispose();
  ref.dispose();
});

check('batched streaming delivers views that outlive their batch; string, buffer, spectra and plugin lists', () => {
  const N = 512;
  const list = ['buffer', 'rms', 'amplitudeSpectrum', 'complexSpectrum', 'powerSpectrum', 'mfcc', 'loudness'];
  const seen = [];
  const m = new Meyda(ctx, null, N, (feat) => seen.push(feat), { batchFrames: 3 });
  m.start(list);
  for (let i = 0; i < 7; i++) m.process(frameOf(g, i));
  m.stop();
  assert.strictEqual(seen.length, 7);
  const ref = new Meyda(ctx, null, N);
  for (let i = 0; i < 7; i++) {   // every batch's values are still the frame's after later batches
    ref.process(frameOf(g, i));
    const r = ref.get(list.filter((n) => n !== 'buffer'));
    assert.deepStrictEqual(Array.from(seen[i].buffer), Array.from(frameOf(g, i)), 'buffer ' + i);
    assert.strictEqual(seen[i].rms, r.rms);
    for (const k of ['amplitudeSpectrum', 'powerSpectrum', 'mfcc']) {
      assert.ok(seen[i][k] instanceof Float32Array);
      assert.deepStrictEqual(Array.from(seen[i][k]), Array.from(r[k]), k + ' ' + i);
    }
    assert.deepStrictEqual(Array.from(seen[i].complexSpectrum.real), Array.from(r.complexSpectrum.real));
    assert.deepStrictEqual(Array.from(seen[i].complexSpectrum.imag), Array.from(r.complexSpectrum.imag));
    assert.strictEqual(seen[i].complexSpectrum.length, N);
    assert.deepStrictEqual(Array.from(seen[i].loudness.specific), Array.from(r.loudness.specific));
    assert.strictEqual(seen[i].loudness.total, r.loudness.total);
  }
  // a single feature name: the callback gets the bare value, as get('rms') returns it
  const one = [];
  const s1 = new Meyda(ctx, null, N, (v) => one.push(v), { batchFrames: 4 });
  s1.start('rms');
  for (let i = 0; i < 5; i++) s1.process(frameOf(g, i));
  s1.stop();
  assert.deepStrictEqual(one, seen.slice(0, 5).map((x) => x.rms));
  // a user plugin in the list takes the per-frame path (the plugin sees its frame's m)
  const pl = [];
  const s2 = new Meyda(ctx, null, N, (v) => pl.push(v), { batchFrames: 4 });
  s2.featureExtractors.peak = (n, mm) => Math.max(...mm.ampSpectrum);
  s2.start(['rms', 'peak']);
  for (let i = 0; i < 5; i++) s2.process(frameOf(g, i));
  s2.stop();
  for (let i = 0; i < 5; i++) {
    assert.strictEqual(pl[i].rms, seen[i].rms);
    assert.strictEqual(pl[i].peak, Math.max(...seen[i].amplitudeSpectrum));
  }
  [m, ref, s1, s2].forEach((x) => x.dispose());
});

check('getBatchWav: .wav bytes -> device decode -> features', () => {
  const { wavS16 } = require('./wav');
  const idx = [];
  g.labels.forEach((l, i) => { if (l.startsWith('sound1')) idx.push(i); });
  const codes = new Int16Array(idx.length * 512 * 2);   // stereo: channel 1 holds the audio
  idx.forEach((fi, j) => {
    const x = frameOf(g, fi);
    for (let t = 0; t < 512; t++) codes[2 * (j * 512 + t) + 1] = Math.round(x[t] * 32768);
  });
  const m = new Meyda(ctx, null, 512);
  const r = m.getBatchWav(['rms', 'zcr', 'mfcc'], wavS16(codes, 2, 44100), 1);
  assert.strictEqual(r.rms.length, idx.length);
  idx.forEach((fi, j) => {
    close(r.rms[j], g.scalars[fi * S + 0], 1e-5, 0, 'wav rms');
    assert.strictEqual(r.zcr[j], g.scalars[fi * S + 2]);
    vecClose(r.mfcc.subarray(j * 13, j * 13 + 13), g.mfcc.subarray(fi * 13, fi * 13 + 13), 'wav mfcc');
  });
  return m.getBatchWavAsync(['rms'], wavS16(codes, 2, 44100), 1).then((a) => {
    assert.deepStrictEqual(Array.from(a.rms), Array.from(r.rms));
    m.dispose();
  });
});

check('windowingFunction = hamming', () => {
  const m = new Meyda(ctx, null, 512);
  m.windowingFunction = 'hamming';
  g.hammingFrames = golden.manifest.sizes['512'].hammingFrames;
  g.hammingFrames.forEach((fi, j) => {
    m.process(frameOf(g, fi));
    vecClose(m.get('amplitudeSpectrum'), g.hamming_amp.subarray(j * 256, j * 256 + 256), 'hamming amp');
  });
  m.dispose();
});

check('literal (snapshot) mode is bit-exact', () => {
  const m = new Meyda(ctx, null, 512, null, { mode: 'literal' });
  golden.manifest.sizes['512'].literalFrames.forEach((fi, j) => {
    m.process(frameOf(g, fi));
    assert.deepStrictEqual(Array.from(m.get('amplitudeSpectrum')), Array.from(g.literal_amp.subarray(j * 256, j * 256 + 256)));
  });
  m.dispose();
});

check('async batch jobs run on their own plan: streaming continues meanwhile', () => {
  const seen = [];
  const m = new Meyda(ctx, null, 512, (feat) => seen.push(feat));
  m.start(['rms', 'zcr']);
  const F = 64;
  const x = g.input.subarray(0, F * 512);
  const p1 = m.getBatchAsync(['rms', 'mfcc'], x);
  const p2 = m.getBatchAsync(['zcr'], x);       // a second job while the first is pending
  for (let i = 0; i < 6; i++) m.process(frameOf(g, i));   // onaudioprocess during the jobs
  assert.strictEqual(seen.length, 6);
  for (let i = 0; i < 6; i++) assert.strictEqual(seen[i].zcr, g.scalars[i * S + 2]);
  m.dispose();                                  // busy plans are left to their jobs
  return Promise.all([p1, p2]).then(([a, b]) => {
    assert.strictEqual(a.rms.length, F);
    for (let i = 0; i < F; i++) assert.strictEqual(b.zcr[i], g.scalars[i * S + 2]);
  });
});

check('async jobs beyond the pool queue on its plans (at most options.asyncPlans per window)', () => {
  const m = new Meyda(ctx, null, 512, null, { asyncPlans: 2 });
  const F = 48;
  const jobs = [];
  for (let k = 0; k < 6; k++) jobs.push(m.getBatchAsync(['zcr', 'rms'], g.input.subarray(k * 512, (k + F) * 512)));
  assert.ok(m._asyncPlans.hanning.length <= 2, 'pool grew to ' + m._asyncPlans.hanning.length);
  return Promise.all(jobs).then((rs) => {
    rs.forEach((r, k) => {
      for (let i = 0; i < F; i++) assert.strictEqual(r.zcr[i], g.scalars[(k + i) * S + 2]);
    });
    m.dispose();
  });
});

check('plan handle collected while an async job runs (no use-after-free)', () => {
  assert.ok(typeof global.gc === 'function', 'run node with --expose-gc');
  const x = g.input.subarray(0, 90 * 512);
  const jobs = [];
  for (let k = 0; k < 4; k++) {
    // the Meyda instance (and its plans) become unreachable right away
    jobs.push(new Meyda(ctx, null, 512).getBatchAsync(['rms', 'spectralCentroid', 'mfcc'], x));
  }
  global.gc();
  return Promise.all(jobs).then((rs) => {
    global.gc();
    for (const r of rs) {
      assert.strictEqual(r.rms.length, 90);
      for (let i = 0; i < 90; i += 11) close(r.rms[i], g.scalars[i * S + 0], 1e-5, 0, 'rms');
    }
  });
});

check('options.devices: batches through a device group equal the single-device plan', () => {
  const F = 77;
  const x = g.input.subarray(0, F * 512);
  const one = new Meyda(ctx, null, 512);
  const grp = new Meyda(ctx, null, 512, null, { devices: [0] });
  const a = one.getBatch(ALL, x);
  const b = grp.getBatch(ALL, x);
  for (const k of Object.keys(a)) assert.deepStrictEqual(Array.from(b[k]), Array.from(a[k]), k);
  grp.process(frameOf(g, 3));
  assert.strictEqual(grp.get('zcr'), g.scalars[3 * S + 2]);
  return grp.getBatchAsync(['rms'], x).then((r) => {
    assert.deepStrictEqual(Array.from(r.rms), Array.from(a.rms));
    one.dispose();
    grp.dispose();
  });
});

check('addon extractInto: one buffer, caller offsets, equal to extract(); bad offsets rejected', () => {
  const addon = Meyda.addon;
  const plan = addon.createPlan({ bufferSize: 512, sampleRate: 44100, scalarF64: 1 });
  const F = 9;
  const x = g.input.subarray(0, F * 512);
  const want = addon.extract(plan, x, ['rms', 'zcr', 'loudness', 'mfcc', 'amplitudeSpectrum']);
  const off = new Float64Array(19).fill(-1);
  // rms, zcr, loudness.total (f64) then loudness.specific, mfcc, amplitude (f32), packed back to back
  off[0] = 0; off[2] = 8 * F; off[10] = 16 * F; off[13] = 24 * F; off[14] = off[13] + 96 * F; off[15] = off[14] + 52 * F;
  const ab = new ArrayBuffer(off[15] + 4 * 256 * F);
  assert.strictEqual(addon.extractInto(plan, x, off, ab), ab);
  const same = (a, b, k) => assert.deepStrictEqual(Array.from(a), Array.from(b), k);
  same(new Float64Array(ab, off[0], F), want.rms, 'rms');
  same(new Float64Array(ab, off[2], F), want.zcr, 'zcr');
  same(new Float64Array(ab, off[10], F), want['loudness.total'], 'loudness.total');
  same(new Float32Array(ab, off[13], 24 * F), want['loudness.specific'], 'loudness.specific');
  same(new Float32Array(ab, off[14], 13 * F), want.mfcc, 'mfcc');
  same(new Float32Array(ab, off[15], 256 * F), want.amplitudeSpectrum, 'amplitude');
  const bad1 = Float64Array.from(off); bad1[0] = 4;   // an f64 output at a 4-byte offset
  assert.throws(() => addon.extractInto(plan, x, bad1, ab), /misaligned|past the end/);
  const bad2 = Float64Array.from(off); bad2[15] = ab.byteLength - 16;  // runs past the end
  assert.throws(() => addon.extractInto(plan, x, bad2, ab), /past the end/);
  const bad3 = Float64Array.from(off); bad3[17] = 0;  // complex real without imag
  assert.throws(() => addon.extractInto(plan, x, bad3, ab), /go together|past the end/);
  assert.throws(() => addon.extractInto(plan, x, new Float64Array(18), ab), /19 byte offsets/);
  addon.destroyPlan(plan);
});

check('options.resident: per-buffer get() and streaming callbacks equal the launch-per-buffer facade', () => {
  // include/meyda_gpu.h MGX_FLAG_RESIDENT: the same kernel code on the same frames, byte-identical values
  const a = new Meyda(ctx, null, 512, null, { resident: true });
  const b = new Meyda(ctx, null, 512);
  const same = (x, y, what) => {
    if (typeof y === 'number') assert.ok(Object.is(x, y), what + ': ' + x + ' vs ' + y);
    else if (y && y.specific) { same(x.total, y.total, what + '.total'); same(x.specific, y.specific, what + '.specific'); }
    else for (let k = 0; k < y.length; k++) assert.ok(Object.is(x[k], y[k]), what + '[' + k + ']');
  };
  for (let i = 0; i < g.F; i++) {
    a.process(frameOf(g, i));
    b.process(frameOf(g, i));
    for (const list of [['rms', 'spectralCentroid'], ALL]) {
      const ra = a.get(list), rb = b.get(list);
      for (const k of list) same(ra[k], rb[k], g.labels[i] + ' ' + k);
    }
  }
  const got = [];
  const s = new Meyda(ctx, null, 512, (r) => got.push(r), { resident: true });
  s.start(['rms', 'zcr', 'mfcc']);
  for (let i = 0; i < 16; i++) s.process(frameOf(g, i));
  s.stop();
  assert.strictEqual(got.length, 16);
  for (let i = 0; i < 16; i++) {
    b.process(frameOf(g, i));
    const r = b.get(['rms', 'zcr', 'mfcc']);
    for (const k of ['rms', 'zcr', 'mfcc']) same(got[i][k], r[k], 'stream ' + i + ' ' + k);
  }
  a.dispose();
  b.dispose();
  s.dispose();
});

(async () => {
  for (const [name, fn] of checks) {
    await fn();
    n++;
    console.log('ok ' + name);
  }
  console.log('facade_gpu: ' + n + ' checks passed');
})().catch((e) => { console.error(e); process.exit(1); });
