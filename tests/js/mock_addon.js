'use strict';
// A stand-in for meyda_napi.node (host-side tests of the facade's JavaScript logic only; never used by
// the product): extract() returns results of the real shapes whose values encode the frame, so a test
// can tell which frame a delivered value came from (frame value = its first sample).
const SCAL = ['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness', 'spectralSlope', 'spectralRolloff',
  'spectralSpread', 'spectralSkewness', 'spectralKurtosis', 'perceptualSpread', 'perceptualSharpness'];
const calls = [];
module.exports = {
  calls,
  hostTables: ({ bufferSize }) => ({ barkScale: new Float32Array(bufferSize), hanning: new Float32Array(bufferSize),
    hamming: new Float32Array(bufferSize) }),
  createPlan: (o) => ({ o }),
  destroyPlan: () => {},
  planBusy: () => false,
  isPowerOfTwo: (v) => v > 0 && (v & (v - 1)) === 0,
  // extractInto(plan, frames, offsets, out): the same values at the facade's byte offsets (mgx_outputs
  // field order; scalars float64, as the facade's plans ask)
  extractInto: (plan, frames, offsets, out) => {
    const N = plan.o.bufferSize, F = frames.length / N;
    calls.push({ F, into: true, fields: Array.from(offsets).map((o, i) => (o >= 0 ? i : -1)).filter((i) => i >= 0) });
    const base = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 99, 10, 11, 100, 200, 300, 300, 400, 500];
    for (let i = 0; i < 19; i++) {
      if (!(offsets[i] >= 0)) continue;
      const per = i < 13 ? 1 : i === 13 ? 24 : i === 14 ? 13 : i < 17 ? N / 2 : N;
      const a = i < 13 ? new Float64Array(out, offsets[i], F) : new Float32Array(out, offsets[i], F * per);
      for (let f = 0; f < F; f++) for (let k = 0; k < per; k++) a[f * per + k] = frames[f * N] + base[i] + k;
    }
    return out;
  },
  extract: (plan, frames, names) => {
    const N = plan.o.bufferSize, F = frames.length / N, r = {};
    calls.push({ F, names: names.slice() });
    const v = (i) => frames[i * N];
    const fill = (a, per, k0) => { for (let i = 0; i < F; i++) for (let k = 0; k < per; k++) a[i * per + k] = v(i) + k0 + k; return a; };
    for (const n of names) {
      const s = SCAL.indexOf(n);
      if (s >= 0) r[n] = fill(new Float64Array(F), 1, s);
      else if (n === 'loudness') { r['loudness.specific'] = fill(new Float32Array(F * 24), 24, 100); r['loudness.total'] = fill(new Float64Array(F), 1, 99); }
      else if (n === 'mfcc') r.mfcc = fill(new Float32Array(F * 13), 13, 200);
      else if (n === 'amplitudeSpectrum' || n === 'powerSpectrum') r[n] = fill(new Float32Array(F * N / 2), N / 2, 300);
      else if (n === 'complexSpectrum') {
        r['complexSpectrum.real'] = fill(new Float32Array(F * N), N, 400);
        r['complexSpectrum.imag'] = fill(new Float32Array(F * N), N, 500);
      }
    }
    return r;
  },
};
