'use strict';
// A stand-in for meyda_napi.node for tools/facade_overhead.js only: extractInto leaves the output
// buffer as it is (zeros), so only the facade's JavaScript is timed. Never used by the product.
module.exports = {
  hostTables: ({ bufferSize }) => ({ barkScale: new Float32Array(bufferSize), hanning: new Float32Array(bufferSize),
    hamming: new Float32Array(bufferSize) }),
  createPlan: (o) => ({ o }),
  destroyPlan: () => {},
  planBusy: () => false,
  isPowerOfTwo: (v) => v > 0 && (v & (v - 1)) === 0,
  extractInto: (plan, frames, offsets, out) => out,
};
