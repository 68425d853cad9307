'use strict';
// meyda_cpu.js — the meyda per-buffer hot path restated in JavaScript for the CPU.
//
// TEST INFRASTRUCTURE AND CPU BASELINE ONLY. Like the C oracle beside it, this file is
// loaded by tests/ (pinned to the reference's golden vectors, tests/test_js_cpu.py) and
// by bench.py's cpu_baseline leg (oracle/js/bench_cpu.js); the product path never loads it.
//
// Written from the semantics tabulated in SURVEY.md §8(a) (rows a1-a29), not from the
// reference's text; the reference itself cannot travel to the GPU box, so this is the
// reference's Node/jsfft CPU path that bench.py times there. Numbers are JavaScript
// doubles, Float32Array stores round to float32, exactly where the reference stores:
//   windows, bark scale      src/meyda.js:116-138, :170-182
//   FFT                      lib/jsfft/fft.js:123-208 (radix-2 DIT, bit reversal,
//                            double butterflies, Float32Array between stages)
//   amplitude                src/meyda.js:104-114
//   extractors               src/extractors/*.js (SURVEY.md §8(a) a11-a29)
//
// Two ways to run a frame:
//   'reference'  the reference's per-buffer structure: every extractor runs on its own,
//                so mu() is recomputed per feature, loudness once more for each perceptual
//                feature, and the MFCC filterbank and DCT matrix are rebuilt per call
//                (SURVEY.md §3(D)). This is the reference path bench.py reports.
//   'batch'      the same arithmetic with the tables built once and shared sums reused.
// Both give identical numbers.

const SQRT1_2 = Math.SQRT1_2;
const NUM_BARK = 24;
const NUM_COEFFS = 13;

// a2, a3: symmetric hann and periodic hamming (the "- 1" kept), stored as float32
function hanning(n) {
  const w = new Float32Array(n);
  for (let i = 0; i < n; i++) w[i] = 0.5 - 0.5 * Math.cos(2 * Math.PI * i / (n - 1));
  return w;
}
function hamming(n) {
  const w = new Float32Array(n);
  for (let i = 0; i < n; i++) w[i] = 0.54 - 0.46 * Math.cos(2 * Math.PI * (i / n - 1));
  return w;
}

// a10: frequency stored to float32 first, then the two arctangents
function barkScale(n, sr) {
  const b = new Float32Array(n);
  const f = new Float32Array(1);
  for (let i = 0; i < n; i++) {
    f[0] = i * sr / n;
    const q = f[0] / 7518;
    b[i] = 13 * Math.atan(f[0] / 1315.8) + 3.5 * Math.atan(q * q);
  }
  return b;
}

// a25: band limits over the first `len` bark values; the last limit is len - 1
function barkLimits(bark, len, nb) {
  const lim = new Int32Array(nb + 1);
  let end = bark[len - 1] / nb;  // NaN for len 0: no limit moves
  let band = 1;
  for (let i = 0; i < len; i++) {
    while (bark[i] > end) {
      if (band <= nb) lim[band] = i;
      band++;
      end = band * bark[len - 1] / nb;
    }
  }
  lim[nb] = len - 1;
  return lim;
}

// a29: mel edges (float32), back to Hz (float32), then FFT bins
function melBins(n, sr, nf) {
  const lo = 1125 * Math.log(1 + 0 / 700);
  const hi = 1125 * Math.log(1 + (sr / 2) / 700);
  const step = (hi - lo) / (nf + 1);
  const mel = new Float32Array(nf + 2), hz = new Float32Array(nf + 2);
  const bins = new Int32Array(nf + 2);
  for (let i = 0; i < nf + 2; i++) {
    mel[i] = i * step;
    hz[i] = 700 * (Math.exp(mel[i] / 1125) - 1);
    bins[i] = Math.floor((n + 1) * hz[i] / sr);
  }
  return bins;
}

// a29: triangular weights (doubles) of every filter over the L bins
function melFilters(bins, nf, L) {
  const fb = [];
  for (let j = 0; j < nf; j++) {
    const w = new Float64Array(L);
    const b0 = bins[j], b1 = bins[j + 1], b2 = bins[j + 2];
    for (let k = b0; k < b1 && k < L; k++) w[k] = (k - b0) / (b1 - b0);
    for (let k = b1; k < b2 && k < L; k++) w[k] = (b2 - k) / (b2 - b1);
    fb.push(w);
  }
  return fb;
}

// a29: DCT-II rows with the (c + 1) index, stored as float32
function dctTable(nf, nc) {
  const d = [];
  const k = Math.PI / nf, w1 = 1 / Math.sqrt(nf), w2 = Math.sqrt(2 / nf);
  for (let c = 0; c < nc; c++) {
    const row = new Float32Array(nf);
    for (let j = 0; j < nf; j++) row[j] = (c === 0 ? w1 : w2) * Math.cos(k * (c + 1) * (j + 0.5));
    d.push(row);
  }
  return d;
}

// a6: bit-reversed index of i over log2(n) bits
function bitReverse(i, n) {
  let r = 0;
  for (let m = n; m > 1; m >>= 1) {
    r = (r << 1) | (i & 1);
    i >>= 1;
  }
  return r;
}

// a5-a7: in place on float32 storage. Per stage of width w: twiddle f advanced by the
// double recurrence from (cos pi/w, +sin pi/w); each butterfly in doubles, both outputs
// scaled by SQRT1_2 and stored to float32.
function fft(re, im, rev) {
  const n = re.length;
  for (let i = 0; i < n; i++) {
    const r = rev[i];
    if (r > i) {
      let t = re[i]; re[i] = re[r]; re[r] = t;
      t = im[i]; im[i] = im[r]; im[r] = t;
    }
  }
  for (let w = 1; w < n; w <<= 1) {
    const dr = Math.cos(Math.PI / w), di = Math.sin(Math.PI / w);
    for (let b = 0; b < n; b += 2 * w) {
      let fr = 1, fi = 0;
      for (let j = 0; j < w; j++) {
        const l = b + j, r = l + w;
        const lr = re[l], li = im[l];
        const rr = fr * re[r] - fi * im[r];
        const ri = fi * re[r] + fr * im[r];
        re[l] = SQRT1_2 * (lr + rr);
        im[l] = SQRT1_2 * (li + ri);
        re[r] = SQRT1_2 * (lr - rr);
        im[r] = SQRT1_2 * (li - ri);
        const t = fr * dr - fi * di;
        fi = fr * di + fi * dr;
        fr = t;
      }
    }
  }
}

// a11: sum_k k^p |a_k| / sum_k a_k
function mu(p, a) {
  let num = 0, den = 0;
  for (let k = 0; k < a.length; k++) {
    num += Math.pow(k, p) * Math.abs(a[k]);
    den += a[k];
  }
  return num / den;
}

class CpuMeyda {
  constructor(opts) {
    const o = Object.assign({ bufferSize: 1024, sampleRate: 44100, window: 'hanning', numMelBands: 26,
      layout: 'reference' }, opts || {});
    this.n = o.bufferSize;
    this.L = this.n / 2;
    this.sr = o.sampleRate;
    this.nf = o.numMelBands;
    this.layout = o.layout;
    this.window = o.window === 'hamming' ? hamming(this.n) : hanning(this.n);
    const bark = barkScale(this.n, this.sr);
    this.lim = barkLimits(bark, this.L, NUM_BARK);
    this.rev = new Int32Array(this.n);
    for (let i = 0; i < this.n; i++) this.rev[i] = bitReverse(i, this.n);
    this.re = new Float32Array(this.n);
    this.im = new Float32Array(this.n);
    this.amp = new Float32Array(this.L);
    this.spec = new Float32Array(NUM_BARK);
    if (this.layout === 'batch') this._mfccTables();
  }

  _mfccTables() {
    this.bins = melBins(this.n, this.sr, this.nf);
    this.fb = melFilters(this.bins, this.nf, this.L);
    this.dct = dctTable(this.nf, NUM_COEFFS);
  }

  // window -> fresh complex array -> FFT -> amplitude (src/meyda.js:69-91,104-114)
  spectrum(x) {
    const { n, L, re, im, amp, window } = this;
    for (let i = 0; i < n; i++) {
      re[i] = x[i] * window[i];
      im[i] = 0;
    }
    fft(re, im, this.rev);
    for (let k = 0; k < L; k++) amp[k] = Math.sqrt(re[k] * re[k] + im[k] * im[k]);
    return amp;
  }

  // a26: specific loudness (float32) and total
  loudness() {
    const { amp, lim, spec } = this;
    for (let b = 0; b < NUM_BARK; b++) {
      let s = 0;
      for (let k = lim[b]; k < lim[b + 1]; k++) s += amp[k];
      spec[b] = Math.pow(s, 0.23);
    }
    let total = 0;
    for (let b = 0; b < NUM_BARK; b++) total += spec[b];
    return { specific: spec, total };
  }

  // a29: power spectrum -> float32 mel sums in ascending bin order -> log -> DCT / 13
  mfcc(out) {
    if (this.layout !== 'batch') this._mfccTables();  // the reference rebuilds them per call
    const { amp, L, nf, fb, dct } = this;
    const p = new Float32Array(L);
    for (let k = 0; k < L; k++) p[k] = amp[k] * amp[k];
    const lm = new Float32Array(nf);
    for (let j = 0; j < nf; j++) {
      const w = fb[j];
      for (let k = 0; k < L; k++) lm[j] += w[k] * p[k];
      lm[j] = Math.log(lm[j]);
    }
    for (let c = 0; c < NUM_COEFFS; c++) {
      let v = 0;
      for (let j = 0; j < nf; j++) v += dct[c][j] * lm[j];
      out[c] = v / NUM_COEFFS;
    }
  }

  // Every feature of one frame x (Float32Array(n)): sc = Float64Array(13) in the record
  // order of include/meyda_gpu.h, spec = Float32Array(24), mf = Float32Array(13) (null: no
  // MFCC); noTime skips rms, energy and zcr (config C3's feature set).
  frame(x, sc, spec, mf, noTime) {
    const { n, L, sr } = this;
    const a = this.spectrum(x);
    if (!noTime) this.timeFeatures(x, sc);
    this.spectralFeatures(a, sc, spec);
    if (mf) this.mfcc(mf);
  }

  // a12-a14 on the unwindowed signal
  timeFeatures(x, sc) {
    const n = this.n;
    let e = 0;
    for (let i = 0; i < n; i++) e += x[i] * x[i];
    let z = 0;
    for (let i = 0; i + 1 < n; i++) {
      if ((x[i] >= 0 && x[i + 1] < 0) || (x[i] < 0 && x[i + 1] >= 0)) z++;
    }
    sc[0] = Math.sqrt(e / n);
    sc[1] = e;
    sc[2] = z;
  }

  // a18-a28 of the amplitude spectrum a (this.amp)
  spectralFeatures(a, sc, spec) {
    const { n, L, sr } = this;
    // a18, a22-a24: mu per feature (the reference calls mu inside each extractor)
    const ref = this.layout !== 'batch';
    const m1 = mu(1, a);
    const m2 = mu(2, a);
    const m3 = mu(3, a);
    const m4 = mu(4, a);
    sc[3] = ref ? mu(1, a) : m1;
    const s1 = ref ? mu(1, a) : m1, s2 = ref ? mu(2, a) : m2;
    sc[7] = Math.sqrt(s2 - s1 * s1);
    const k1 = ref ? mu(1, a) : m1, k2 = ref ? mu(2, a) : m2, k3 = ref ? mu(3, a) : m3;
    sc[8] = (2 * Math.pow(k1, 3) - 3 * k1 * k2 + k3) / Math.pow(Math.sqrt(k2 - k1 * k1), 3);
    sc[9] = (-3 * Math.pow(m1, 4) + 6 * m1 * m2 - 4 * m1 * m3 + m4) / Math.pow(Math.sqrt(m2 - m1 * m1), 4);
    // a19
    let ln = 0, den = 0;
    for (let k = 0; k < L; k++) {
      ln += Math.log(a[k]);
      den += a[k];
    }
    sc[4] = Math.exp(ln / L) * L / den;
    // a20: the denominator without the L factor, as written
    let as = 0, fs = 0, pfs = 0, afs = 0;
    for (let k = 0; k < L; k++) {
      as += a[k];
      const f = k * sr / n;
      pfs += f * f;
      fs += f;
      afs += f * a[k];
    }
    sc[5] = (L * afs - fs * as) / (as * (pfs - fs * fs));
    // a21: descending subtraction from the total
    let ec = 0;
    for (let k = 0; k < L; k++) ec += a[k];
    const thr = 0.99 * ec;
    let k = L - 1;
    while (ec > thr && k >= 0) {
      ec -= a[k];
      --k;
    }
    sc[6] = (k + 1) * (sr / (2 * (L - 1)));
    // a25-a28: the perceptual features call loudness again in the reference
    let loud = this.loudness();
    sc[10] = loud.total;
    if (spec) spec.set(loud.specific);
    if (ref) loud = this.loudness();
    let mx = 0;
    for (let b = 0; b < NUM_BARK; b++) if (loud.specific[b] > mx) mx = loud.specific[b];
    const ps = (loud.total - mx) / loud.total;
    sc[11] = ps * ps;
    if (ref) loud = this.loudness();
    let sh = 0;
    for (let i = 0; i < NUM_BARK; i++) sh += i < 15 ? (i + 1) * loud.specific[i + 1] : 0.066 * Math.exp(0.171 * (i + 1));
    sc[12] = sh * (0.11 / loud.total);
  }

  // F frames (Float32Array(F * n)) -> structure of arrays (scalars F x 13, specific F x 24,
  // mfcc F x 13, amplitude F x n/2)
  batch(frames, wantAmp) {
    const F = frames.length / this.n;
    const out = { scalars: new Float64Array(F * 13), specific: new Float32Array(F * NUM_BARK),
      mfcc: new Float32Array(F * NUM_COEFFS), amp: wantAmp ? new Float32Array(F * this.L) : null };
    const sc = new Float64Array(13), spec = new Float32Array(NUM_BARK), mf = new Float32Array(NUM_COEFFS);
    for (let f = 0; f < F; f++) {
      this.frame(frames.subarray(f * this.n, (f + 1) * this.n), sc, spec, mf);
      out.scalars.set(sc, f * 13);
      out.specific.set(spec, f * NUM_BARK);
      out.mfcc.set(mf, f * NUM_COEFFS);
      if (wantAmp) out.amp.set(this.amp, f * this.L);
    }
    return out;
  }
}

// SURVEY.md §8(d): x[i] = (splitmix64(seed + (i + 1) * 0x9E3779B97F4A7C15) >> 40) * 2^-23 - 1
function synthFrames(seed, firstFrame, count, n) {
  const M = (1n << 64n) - 1n;
  const out = new Float32Array(count * n);
  const s = BigInt(seed);
  for (let t = 0; t < count * n; t++) {
    let z = (s + (BigInt(firstFrame * n + t) + 1n) * 0x9E3779B97F4A7C15n) & M;
    z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & M;
    z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & M;
    z ^= z >> 31n;
    out[t] = Number(z >> 40n) * (1 / 8388608) - 1;
  }
  return out;
}

module.exports = { CpuMeyda, hanning, hamming, barkScale, barkLimits, melBins, dctTable, fft, mu, synthFrames };
