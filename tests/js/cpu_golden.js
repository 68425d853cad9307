'use strict';
// The JavaScript CPU restatement (oracle/js/meyda_cpu.js) against the reference's own
// outputs (tests/golden, made by running the reference under Node): spectra, specific
// loudness, MFCC and the double scalars bit for bit (NaN where the reference has NaN), in
// both frame layouts, for N = 512, 1024, 2048, the hamming window and 40 mel bands.
const assert = require('assert');
const path = require('path');
const golden = require('./golden');
const cpu = require(path.join(__dirname, '..', '..', 'oracle', 'js', 'meyda_cpu.js'));

function bits(a) { return new Uint32Array(a.buffer, a.byteOffset, a.length); }
function sameBits(a, b, what) {
  assert.strictEqual(a.length, b.length, what + ' length');
  const x = bits(a), y = bits(b);
  let bad = 0;
  for (let i = 0; i < x.length; i++) if (x[i] !== y[i]) bad++;
  assert.strictEqual(bad, 0, what + ': ' + bad + ' of ' + x.length + ' differ');
}
function closeScalars(got, ref, F, what) {
  let worst = 0;
  for (let i = 0; i < F * 13; i++) {
    const g = got[i], r = ref[i];
    if (Number.isNaN(r) || !Number.isFinite(r)) {
      assert.ok(Object.is(g, r) || (Number.isNaN(g) && Number.isNaN(r)), what + ' class at ' + i + ': ' + g + ' vs ' + r);
      continue;
    }
    const d = Math.abs(g - r) / Math.max(Math.abs(r), 1e-300);
    if (r !== g) worst = Math.max(worst, d);
    assert.ok(Object.is(g, r), what + ' scalar ' + (i % 13) + ' of frame ' + Math.floor(i / 13) + ': ' + g + ' vs ' + r);
  }
  return worst;
}

let checks = 0;
for (const N of [512, 1024, 2048]) {
  const g = golden.load(N);
  const s = golden.manifest.sizes[String(N)];
  for (const layout of ['reference', 'batch']) {
    const m = new cpu.CpuMeyda({ bufferSize: N, layout });
    const r = m.batch(g.input, true);
    sameBits(r.amp, g.amp, N + ' ' + layout + ' amplitude');
    sameBits(r.specific, g.loudness_specific, N + ' ' + layout + ' loudness.specific');
    sameBits(r.mfcc, g.mfcc, N + ' ' + layout + ' mfcc');
    const w = closeScalars(r.scalars, g.scalars, g.F, N + ' ' + layout);
    console.log('N=' + N + ' ' + layout + ': spectra/specific/mfcc bit-exact, scalars worst rel ' + w);
    checks++;
  }
  // hamming window subset
  const hm = new cpu.CpuMeyda({ bufferSize: N, window: 'hamming', layout: 'batch' });
  const hx = new Float32Array(s.hammingFrames.length * N);
  s.hammingFrames.forEach((fi, j) => hx.set(g.input.subarray(fi * N, (fi + 1) * N), j * N));
  const hr = hm.batch(hx, true);
  sameBits(hr.amp, g.hamming_amp, N + ' hamming amplitude');
  sameBits(hr.mfcc, g.hamming_mfcc, N + ' hamming mfcc');
  closeScalars(hr.scalars, g.hamming_scalars, s.hammingFrames.length, N + ' hamming');
  // 40 mel bands (restatement-derived golden: the reference hard-codes 26)
  const m40 = new cpu.CpuMeyda({ bufferSize: N, numMelBands: 40, layout: 'batch' });
  sameBits(m40.batch(g.input, false).mfcc, g.mfcc40, N + ' mfcc40');
  // tables
  sameBits(cpu.hanning(N), g.hann, N + ' hann');
  sameBits(cpu.hamming(N), g.hamming, N + ' hamming table');
  sameBits(cpu.barkScale(N, 44100), g.bark, N + ' bark');
  assert.deepStrictEqual(Array.from(cpu.barkLimits(cpu.barkScale(N, 44100), N / 2, 24)), Array.from(g.bblimits));
  assert.deepStrictEqual(Array.from(cpu.melBins(N, 44100, 26)), Array.from(g.mel_bins));
  checks += 2;
}
// the synthetic stream matches the fixtures' noise frames (SURVEY.md §8(d))
{
  const g = golden.load(512);
  const x = cpu.synthFrames(0x6D657964, 0, 2, 512);
  sameBits(x, g.input.subarray(0, 1024), 'synth frames');
  checks++;
}
console.log('cpu_golden: ' + checks + ' checks passed');
