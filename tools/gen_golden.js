#!/usr/bin/env node
// Golden-vector generator for the meyda hot path.
//
// Runs ONLY in the build container (it requires the read-only reference at
// $MEYDA_REF, default /root/reference/). It never copies reference source: it
// `require`s the reference modules by absolute path, drives them through a
// harness, and writes the resulting numbers (small binary fixtures + a JSON
// manifest) into tests/golden/. The GPU box never runs this script.
//
// Harness (SURVEY.md §8(c)):
//   * globals the extractors expect: `µ` (src/utils.js:1-11) and `audioContext`
//     (src/extractors/mfcc.js:20,37); `window` for src/meyda.js:67.
//   * `new Meyda(ctx, src, N)` with a mock context (no callback: src/meyda.js:87
//     throws a ReferenceError when a callback is set).
//   * Per frame, the INTENDED path: window (src/meyda.js:158-168) -> fresh
//     ComplexArray (lib/jsfft/complex_array.js:22-36) -> map real (:54-70) ->
//     FFT (lib/jsfft/fft.js:123-171) -> computeAmplitude (src/meyda.js:104-114)
//     -> each extractor module (src/extractors/*.js) with a mock `m`.
//   * The LITERAL path (the snapshot's actual onaudioprocess, which never runs
//     an FFT per buffer: src/meyda.js:69-91,184-197) for a few frames.
//   * 40-band MFCC: mfcc.js hard-codes 26 filters (src/extractors/mfcc.js:15).
//     For config C4 we evaluate the reference's mfcc source text in a vm
//     context with that one literal changed to 40 (in memory only). Those
//     vectors are labelled "reference-algorithm, numFilters substituted".
'use strict';
const fs = require('fs');
const path = require('path');
const vm = require('vm');

const REF = (process.env.MEYDA_REF || '/root/reference/').replace(/\/?$/, '/');
const OUT = path.resolve(__dirname, '..', 'tests', 'golden');
const SR = 44100;
const SEED = 0x6D657964n; // "meyd"

// ---------------------------------------------------------------- harness ---
const ctx = {
  sampleRate: SR,
  destination: {},
  createScriptProcessor() { return { connect() {} }; },
};
const source = { connect() {} };
global.window = {};
global.audioContext = ctx;
global['µ'] = require(REF + 'src/utils').µ;
const Meyda = require(REF + 'src/meyda.js');
const { ComplexArray } = require(REF + 'lib/jsfft/complex_array');
require(REF + 'lib/jsfft/fft'); // decorates ComplexArray.prototype.FFT

const EXTRACTORS = {};
for (const name of ['rms', 'energy', 'zcr', 'amplitudeSpectrum', 'powerSpectrum',
  'complexSpectrum', 'spectralCentroid', 'spectralFlatness', 'spectralSlope',
  'spectralRolloff', 'spectralSpread', 'spectralSkewness', 'spectralKurtosis',
  'perceptualSpread', 'perceptualSharpness', 'mfcc']) {
  EXTRACTORS[name] = require(REF + 'src/extractors/' + name);
}

// mfcc with numFilters substituted (in-memory vm evaluation of the reference text).
function mfccWithFilters(numFilters) {
  const src = fs.readFileSync(REF + 'src/extractors/mfcc.js', 'utf8');
  const needle = 'var numFilters = 26;';
  if (src.indexOf(needle) < 0) throw new Error('mfcc.js literal not found');
  const patched = src.replace(needle, 'var numFilters = ' + numFilters + ';');
  const mod = { exports: {} };
  const sandbox = {
    module: mod, exports: mod.exports, Math, Float32Array, Array, Number,
    audioContext: ctx,
    require: (p) => { if (p === './powerSpectrum') return EXTRACTORS.powerSpectrum; throw new Error(p); },
  };
  vm.runInNewContext(patched, sandbox, { filename: 'mfcc.js(numFilters=' + numFilters + ')' });
  return mod.exports;
}
const mfcc40 = mfccWithFilters(40);

// Scalar features in record order (manifest lists them).
const SCALARS = ['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness',
  'spectralSlope', 'spectralRolloff', 'spectralSpread', 'spectralSkewness',
  'spectralKurtosis', 'loudnessTotal', 'perceptualSpread', 'perceptualSharpness'];

function makeMeyda(N) {
  const M = new Meyda(ctx, source, N);
  return M;
}

// Intended per-buffer path for one frame: returns a record of copies.
function runIntended(M, N, x, windowName) {
  const L = M.featureExtractors.loudness;
  const w = M.computeWindow(x, windowName || 'hanning');
  const d = new ComplexArray(N);
  d.map(function (v, i) { v.real = w[i]; });
  const spec = d.FFT();
  M.computeAmplitude(spec, M.ampSpectrum, N);
  const m = {
    signal: x,
    ampSpectrum: M.ampSpectrum,
    complexSpectrum: spec,
    audioContext: ctx,
    featureExtractors: { loudness: () => L.process() },
  };
  const rec = {};
  for (const name of ['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness',
    'spectralSlope', 'spectralRolloff', 'spectralSpread', 'spectralSkewness',
    'spectralKurtosis', 'perceptualSpread', 'perceptualSharpness']) {
    rec[name] = EXTRACTORS[name](N, m);
  }
  const loud = L.process();
  rec.loudnessTotal = loud.total;
  rec.loudnessSpecific = Float32Array.from(loud.specific);
  rec.mfcc = Float32Array.from(EXTRACTORS.mfcc(N, m));
  rec.mfcc40 = Float32Array.from(mfcc40(N, m));
  rec.amp = Float32Array.from(M.ampSpectrum);
  rec.power = Float32Array.from(EXTRACTORS.powerSpectrum(N, m));
  rec.re = Float32Array.from(spec.real);
  rec.im = Float32Array.from(spec.imag);
  return rec;
}

// Literal snapshot path: drive the real onaudioprocess handler (no FFT per buffer).
function runLiteral(M, x) {
  window.spn.onaudioprocess({ inputBuffer: { getChannelData: () => x } });
  const loud = M.get('loudness');
  return {
    amp: Float32Array.from(M.ampSpectrum),
    loudnessTotal: loud.total,
    loudnessSpecific: Float32Array.from(loud.specific),
  };
}

// ------------------------------------------------------------------ inputs ---
const MASK64 = (1n << 64n) - 1n;
// splitmix64 output for state seed advanced (i+1) times; top 24 bits -> [-1, 1).
function synthSample(seed, i) {
  let z = (seed + (BigInt(i) + 1n) * 0x9E3779B97F4A7C15n) & MASK64;
  z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & MASK64;
  z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & MASK64;
  z = z ^ (z >> 31n);
  return Number(z >> 40n) * Math.pow(2, -23) - 1;
}
function noiseFrames(N, F) {
  const out = [];
  for (let f = 0; f < F; f++) {
    const x = new Float32Array(N);
    for (let n = 0; n < N; n++) x[n] = synthSample(SEED, f * N + n);
    out.push(x);
  }
  return out;
}

// Minimal RIFF walk: fmt chunk may be 16 or 18 bytes (sound2.wav), PCM16 mono.
function readWav(file) {
  const b = fs.readFileSync(file);
  if (b.toString('ascii', 0, 4) !== 'RIFF' || b.toString('ascii', 8, 12) !== 'WAVE') throw new Error(file);
  let off = 12, fmt = null;
  while (off + 8 <= b.length) {
    const id = b.toString('ascii', off, off + 4);
    const size = b.readUInt32LE(off + 4);
    if (id === 'fmt ') {
      fmt = { format: b.readUInt16LE(off + 8), channels: b.readUInt16LE(off + 10),
        rate: b.readUInt32LE(off + 12), bits: b.readUInt16LE(off + 22) };
    } else if (id === 'data') {
      if (!fmt || fmt.format !== 1 || fmt.bits !== 16) throw new Error('unsupported ' + file);
      const n = Math.floor(Math.min(size, b.length - off - 8) / 2 / fmt.channels);
      const pcm = new Float32Array(n);
      for (let i = 0; i < n; i++) pcm[i] = b.readInt16LE(off + 8 + i * 2 * fmt.channels) / 32768;
      return { fmt, pcm, dataOffset: off + 8 };
    }
    off += 8 + size + (size & 1);
  }
  throw new Error('no data chunk ' + file);
}
function wavFrames(pcm, N, F) {
  const total = Math.floor(pcm.length / N);
  const out = [], idx = [];
  for (let j = 0; j < F; j++) {
    const fi = Math.floor((j + 0.5) * total / F);
    out.push(pcm.slice(fi * N, fi * N + N));
    idx.push(fi);
  }
  return { frames: out, frameIndex: idx };
}
function edgeFrames(N) {
  const mk = (fn) => { const x = new Float32Array(N); for (let n = 0; n < N; n++) x[n] = fn(n); return x; };
  const e = {};
  e.zeros = mk(() => 0);
  e.dc = mk(() => 0.5);
  e.impulse = mk((n) => (n === N / 2 ? 1 : 0));
  e.nyquist = mk((n) => (n & 1 ? -1 : 1));
  e.square = mk((n) => (n < N / 2 ? 1 : -1));
  e.signedZeros = mk((n) => [-0, 1, 0, -1, 0, -0, 0.25, -0.25][n & 7]);
  e.twoTone = mk((n) => 0.5 * Math.sin(2 * Math.PI * 440 * n / SR) + 0.25 * Math.sin(2 * Math.PI * 3000 * n / SR));
  e.tiny = mk((n) => 1e-30 * synthSample(SEED + 7n, n));
  e.loud = mk((n) => 3e4 * synthSample(SEED + 11n, n));
  return e;
}

// ---------------------------------------------------------- table mirrors ---
// The host tables the build uploads, evaluated here with V8's Math so the C
// table generator can be checked bit-for-bit (SURVEY.md §7 hard part 6).
function melTables(N, numFilters) {
  const freqToMel = (f) => 1125 * Math.log(1 + (f / 700));
  const melToFreq = (m) => 700 * (Math.exp(m / 1125) - 1);
  const melValues = new Float32Array(numFilters + 2);
  const melFreq = new Float32Array(numFilters + 2);
  const lo = freqToMel(0), hi = freqToMel(SR / 2);
  const step = (hi - lo) / (numFilters + 1);
  const bins = new Int32Array(numFilters + 2);
  for (let i = 0; i < melValues.length; i++) {
    melValues[i] = i * step;
    melFreq[i] = melToFreq(melValues[i]);
    bins[i] = Math.floor((N + 1) * melFreq[i] / SR);
  }
  const k = Math.PI / numFilters, w1 = 1.0 / Math.sqrt(numFilters), w2 = Math.sqrt(2.0 / numFilters);
  const dct = new Float32Array(13 * numFilters);
  for (let i = 0; i < 13; i++) for (let j = 0; j < numFilters; j++)
    dct[i + j * 13] = (i === 0 ? w1 : w2) * Math.cos(k * (i + 1) * (j + 0.5));
  return { melValues, melFreq, bins, dct };
}
function twiddleSeeds(N) {
  // del_f per stage as jsfft computes it (lib/jsfft/fft.js:144-145).
  const out = [];
  for (let w = 1; w < N; w <<= 1) out.push(Math.cos(Math.PI / w), Math.sin(Math.PI / w));
  return Float64Array.from(out);
}

// ------------------------------------------------------------------ driver ---
function writeBin(rel, typed) {
  fs.writeFileSync(path.join(OUT, rel), Buffer.from(typed.buffer, typed.byteOffset, typed.byteLength));
  return rel;
}
function concat(Type, arrs) {
  const n = arrs.reduce((a, x) => a + x.length, 0);
  const out = new Type(n);
  let o = 0;
  for (const a of arrs) { out.set(a, o); o += a.length; }
  return out;
}

function main() {
  fs.mkdirSync(OUT, { recursive: true });
  const wavs = {};
  for (const s of ['sound1', 'sound2', 'sound3']) wavs[s] = readWav(REF + 'audio/' + s + '.wav');
  const manifest = {
    generator: 'tools/gen_golden.js',
    reference: 'kirbysayshi/meyda snapshot (src/, lib/jsfft/) evaluated under node ' + process.version,
    sampleRate: SR,
    seed: '0x' + SEED.toString(16),
    synth: 'x[i] = (splitmix64(seed + (i+1)*0x9E3779B97F4A7C15) >> 40) * 2^-23 - 1, i = f*N + n',
    scalars: SCALARS,
    wav: {},
    sizes: {},
  };
  for (const s of Object.keys(wavs)) {
    manifest.wav[s] = { samples: wavs[s].pcm.length, dataOffset: wavs[s].dataOffset, fmt: wavs[s].fmt };
  }
  const plan = { 512: [32, 16], 1024: [32, 16], 2048: [16, 8] };
  for (const N of [512, 1024, 2048]) {
    const [nNoise, nWav] = plan[N];
    const M = makeMeyda(N);
    const frames = [], labels = [];
    noiseFrames(N, nNoise).forEach((x, f) => { frames.push(x); labels.push('noise:' + f); });
    for (const s of Object.keys(wavs)) {
      const { frames: fr, frameIndex } = wavFrames(wavs[s].pcm, N, nWav);
      fr.forEach((x, j) => { frames.push(x); labels.push(s + ':' + frameIndex[j]); });
    }
    const edges = edgeFrames(N);
    for (const k of Object.keys(edges)) { frames.push(edges[k]); labels.push('edge:' + k); }
    // config C1: frame 0 of sound1.wav (the reference's own demo input)
    frames.push(wavs.sound1.pcm.slice(0, N)); labels.push('sound1:0');

    const recs = frames.map((x) => runIntended(M, N, x, 'hanning'));
    const F = frames.length, L = N / 2;
    const scal = new Float64Array(F * SCALARS.length);
    recs.forEach((r, f) => SCALARS.forEach((k, j) => { scal[f * SCALARS.length + j] = r[k]; }));
    const nCx = Math.min(F, 16);

    // hamming window variant on the first 8 noise frames + the edges
    const hamIdx = [0, 1, 2, 3, 4, 5, 6, 7].concat(labels.map((l, i) => (l.startsWith('edge:') ? i : -1)).filter((i) => i >= 0));
    const hamRecs = hamIdx.map((i) => runIntended(M, N, frames[i], 'hamming'));
    const hamScal = new Float64Array(hamIdx.length * SCALARS.length);
    hamRecs.forEach((r, f) => SCALARS.forEach((k, j) => { hamScal[f * SCALARS.length + j] = r[k]; }));

    // literal (snapshot) path on the first 8 frames: no FFT per buffer
    const litIdx = [0, 1, 2, 3, 4, 5, 6, 7];
    const M2 = makeMeyda(N);
    const lit = litIdx.map((i) => runLiteral(M2, frames[i]));

    const t = melTables(N, 26), t40 = melTables(N, 40);
    const dir = 'N' + N + '/';
    fs.mkdirSync(path.join(OUT, dir), { recursive: true });
    manifest.sizes[N] = {
      frames: F,
      labels,
      files: {
        input: writeBin(dir + 'input.f32', concat(Float32Array, frames)),
        amp: writeBin(dir + 'amp.f32', concat(Float32Array, recs.map((r) => r.amp))),
        power: writeBin(dir + 'power.f32', concat(Float32Array, recs.map((r) => r.power))),
        complex_re: writeBin(dir + 'complex_re.f32', concat(Float32Array, recs.slice(0, nCx).map((r) => r.re))),
        complex_im: writeBin(dir + 'complex_im.f32', concat(Float32Array, recs.slice(0, nCx).map((r) => r.im))),
        scalars: writeBin(dir + 'scalars.f64', scal),
        loudness_specific: writeBin(dir + 'loudness_specific.f32', concat(Float32Array, recs.map((r) => r.loudnessSpecific))),
        mfcc: writeBin(dir + 'mfcc.f32', concat(Float32Array, recs.map((r) => r.mfcc))),
        mfcc40: writeBin(dir + 'mfcc40.f32', concat(Float32Array, recs.map((r) => r.mfcc40))),
        hamming_amp: writeBin(dir + 'hamming_amp.f32', concat(Float32Array, hamRecs.map((r) => r.amp))),
        hamming_scalars: writeBin(dir + 'hamming_scalars.f64', hamScal),
        hamming_mfcc: writeBin(dir + 'hamming_mfcc.f32', concat(Float32Array, hamRecs.map((r) => r.mfcc))),
        literal_amp: writeBin(dir + 'literal_amp.f32', concat(Float32Array, lit.map((r) => r.amp))),
        literal_loudness_specific: writeBin(dir + 'literal_loudness_specific.f32', concat(Float32Array, lit.map((r) => r.loudnessSpecific))),
        literal_loudness_total: writeBin(dir + 'literal_loudness_total.f64', Float64Array.from(lit.map((r) => r.loudnessTotal))),
        hann: writeBin(dir + 'hann.f32', M.hanning),
        hamming: writeBin(dir + 'hamming.f32', M.hamming),
        bark: writeBin(dir + 'bark.f32', M.barkScale),
        bblimits: writeBin(dir + 'bblimits.i32', Int32Array.from(M.featureExtractors.loudness.bbLimits)),
        mel_values: writeBin(dir + 'mel_values.f32', t.melValues),
        mel_freq: writeBin(dir + 'mel_freq.f32', t.melFreq),
        mel_bins: writeBin(dir + 'mel_bins.i32', t.bins),
        dct: writeBin(dir + 'dct.f32', t.dct),
        mel40_bins: writeBin(dir + 'mel40_bins.i32', t40.bins),
        dct40: writeBin(dir + 'dct40.f32', t40.dct),
        twiddle_seeds: writeBin(dir + 'twiddle_seeds.f64', twiddleSeeds(N)),
      },
      complexFrames: nCx,
      hammingFrames: hamIdx,
      literalFrames: litIdx,
    };
    console.log('N=' + N + ': ' + F + ' frames');
  }
  fs.writeFileSync(path.join(OUT, 'manifest.json'), JSON.stringify(manifest, null, 1) + '\n');
}
main();
