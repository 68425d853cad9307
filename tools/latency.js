'use strict';
// Real-time path latency of the product's JavaScript facade (meyda_amd/js/meyda.js over the
// N-API addon and libmeyda_gpu.so; one GPU launch per extraction, or with options.resident one
// workgroup that stays on the device between buffers), for bench.py's `latency`
// field (SURVEY.md §8(f) row 1, BASELINE.json configs[0]):
//   c1: new Meyda(ctx, null, 512).get(['rms', 'spectralCentroid']) on sound1.wav's frame 0
//       (tests/golden), one process() + get() per call: median / p90 us over >= 1000 calls
//       (src/meyda.js:69-91,244-261);
//   stream: start(features) then process() buffer by buffer with the callback
//       (src/meyda.js:69-91,233-241), options.batchFrames 1 (a launch per buffer, the callback
//       inside process()) and 64 (64 buffers per launch, callbacks in order; stop() flushes):
//       the median us per launch (each launch's K process() calls timed on their own), per buffer and
//       buffers/s, for C1's features at N = 512 and every feature at N = 1024.
// Prints one JSON line. Needs a GPU; reads only the product and tests/golden (data).
const fs = require('fs');
const os = require('os');
const path = require('path');

const Meyda = require(path.join(__dirname, '..', 'meyda_amd', 'js', 'meyda.js'));

const ctx = { sampleRate: 44100 };
const GOLDEN = path.join(__dirname, '..', 'tests', 'golden');
const manifest = JSON.parse(fs.readFileSync(path.join(GOLDEN, 'manifest.json'), 'utf8'));
const ALL = ['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness', 'spectralSlope', 'spectralRolloff',
  'spectralSpread', 'spectralSkewness', 'spectralKurtosis', 'loudness', 'perceptualSpread', 'perceptualSharpness',
  'mfcc'];

function goldenInputs(n) {
  const s = manifest.sizes[String(n)];
  const b = fs.readFileSync(path.join(GOLDEN, s.files.input));
  return { x: new Float32Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength)), labels: s.labels, F: s.frames };
}

function pct(a, p) {
  const s = a.slice().sort((u, v) => u - v);
  return s[Math.min(s.length - 1, Math.floor(s.length * p))];
}

const now = () => process.hrtime.bigint();
const us = (a, b) => Number(b - a) * 1e-3;

function c1(options, gapUs) {
  const g = goldenInputs(512);
  const i = g.labels.indexOf('sound1:0');
  const x = g.x.slice(i * 512, (i + 1) * 512);
  const m = new Meyda(ctx, null, 512, undefined, options);
  let r;
  for (let k = 0; k < 100; k++) {
    m.process(x);
    r = m.get(['rms', 'spectralCentroid']);
  }
  const t = [];
  const t0 = now();
  while (t.length < 1000 || us(t0, now()) < 2e6) {
    if (gapUs) {  // the host idle between buffers, as between a real-time source's callbacks
      const w = now();
      while (us(w, now()) < gapUs) { /* spin */ }
    }
    const a = now();
    m.process(x);  // a new buffer: the next get() launches again
    r = m.get(['rms', 'spectralCentroid']);
    t.push(us(a, now()));
  }
  m.dispose();
  return { us_per_call: pct(t, 0.5), us_p90: pct(t, 0.9), us_min: pct(t, 0), calls: t.length,
    rms: r.rms, spectralCentroid: r.spectralCentroid };
}

function stream(n, feats, K, launches, options) {
  const g = goldenInputs(n);
  const frames = [];
  for (let i = 0; i < g.F; i++) frames.push(g.x.slice(i * n, (i + 1) * n));
  let got = 0;
  const m = new Meyda(ctx, null, n, () => { got++; }, Object.assign({ batchFrames: K }, options));
  m.start(feats);
  for (let i = 0; i < 50 * K; i++) m.process(frames[i % frames.length]);  // plans, JIT, staging
  m.stop();
  m.start(feats);
  got = 0;
  // each launch's K process() calls timed on their own (the K-th launches and delivers the batch): the
  // median per launch, robust to a GC pause or a descheduled host thread, and the mean over all of them
  const t = [];
  let i = 0;
  const t0 = now();
  while (t.length < launches || us(t0, now()) < 1e6) {
    const a = now();
    for (let k = 0; k < K; k++, i++) m.process(frames[i % frames.length]);
    t.push(us(a, now()));
  }
  const el = us(t0, now());
  m.stop();
  m.dispose();
  if (got !== i) throw new Error('callbacks ' + got + ' != buffers ' + i);
  const med = pct(t, 0.5);
  return { bufferSize: n, batchFrames: K, resident: !!(options && options.resident), features: feats, buffers: i,
    launches: t.length, us_per_launch: med,
    us_per_buffer: med / K, buffers_per_s: K / (med * 1e-6), us_per_launch_p90: pct(t, 0.9),
    us_per_launch_mean: el / t.length };
}

// c1: one launch per buffer (the facade's default); c1_resident: options.resident, the buffers handed to a
// workgroup that stays on the device (include/meyda_gpu.h MGX_FLAG_RESIDENT)
// c1_gap / c1_resident_gap: the same with the host idle 1 ms between calls (a real-time source delivers a buffer
// every 11.6 ms at 512 samples and 44.1 kHz; the calls are then never back to back)
const out = { c1: c1(), c1_resident: c1({ resident: true }), c1_gap: c1({}, 1000),
  c1_resident_gap: c1({ resident: true }, 1000), stream: [] };
for (const [n, feats] of [[512, ['rms', 'spectralCentroid']], [1024, ALL]]) {
  for (const K of [1, 64]) out.stream.push(stream(n, feats, K, K === 1 ? 2000 : 300));
  out.stream.push(stream(n, feats, 1, 2000, { resident: true }));
}
out.node = process.version;
out.cpu_model = os.cpus()[0].model;
out.path = 'meyda_amd/js/meyda.js -> meyda_amd/addon/meyda_napi.node -> libmeyda_gpu.so (mgx_extract_host)';
console.log(JSON.stringify(out));
