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
