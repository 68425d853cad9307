#!/usr/bin/env node
// Times the reference's own CPU path (Node + jsfft + the extractor modules) on one core in
// THIS container, for context next to bench.py's cpu_baseline (the C restatement, which is
// what travels to the GPU box). Like tools/gen_golden.js it `require`s the read-only
// reference by path ($MEYDA_REF, default /root/reference/) and copies nothing; the GPU box
// never runs it. Per frame: the intended per-buffer path (window -> ComplexArray -> FFT ->
// amplitude) and every feature of the bench (13 scalars, loudness, 26-band mfcc).
'use strict';
const REF = (process.env.MEYDA_REF || '/root/reference/').replace(/\/?$/, '/');
const N = Number(process.argv[2] || 1024);
const SECONDS = Number(process.argv[3] || 10);
const ctx = { sampleRate: 44100, destination: {}, createScriptProcessor() { return { connect() {} }; } };
global.window = {};
global.audioContext = ctx;
global['µ'] = require(REF + 'src/utils').µ;
const Meyda = require(REF + 'src/meyda.js');
const { ComplexArray } = require(REF + 'lib/jsfft/complex_array');
require(REF + 'lib/jsfft/fft');
const NAMES = ['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness', 'spectralSlope',
  'spectralRolloff', 'spectralSpread', 'spectralSkewness', 'spectralKurtosis', 'perceptualSpread',
  'perceptualSharpness', 'mfcc'];
const EX = {};
for (const n of NAMES) EX[n] = require(REF + 'src/extractors/' + n);
const M = new Meyda(ctx, { connect() {} }, N);
const L = M.featureExtractors.loudness;
const frames = [];
let s = 12345;
for (let f = 0; f < 64; f++) {
  const x = new Float32Array(N);
  for (let i = 0; i < N; i++) { s = (s * 1103515245 + 12345) >>> 0; x[i] = s / 2147483648 - 1; }
  frames.push(x);
}
let done = 0, sink = 0;
const t0 = process.hrtime.bigint();
let el = 0;
while (el < SECONDS) {
  for (const x of frames) {
    const w = M.computeWindow(x, 'hanning');
    const d = new ComplexArray(N);
    d.map(function (v, i) { v.real = w[i]; });
    const spec = d.FFT();
    M.computeAmplitude(spec, M.ampSpectrum, N);
    const m = { signal: x, ampSpectrum: M.ampSpectrum, complexSpectrum: spec, audioContext: ctx,
      featureExtractors: { loudness: () => L.process() } };
    for (const n of NAMES) { const v = EX[n](N, m); sink += typeof v === 'number' ? v : v[0]; }
    sink += L.process().total;
    done++;
  }
  el = Number(process.hrtime.bigint() - t0) / 1e9;
}
console.log(JSON.stringify({ reference: 'Node ' + process.version + ' + jsfft (kirbysayshi/meyda)', n: N,
  frames: done, seconds: el, frames_per_s: done / el, cores: 1, checksum_finite: Number.isFinite(sink) }));
