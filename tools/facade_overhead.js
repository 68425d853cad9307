'use strict';
// The batched streaming path's JavaScript cost alone (no GPU): meyda_amd/js/meyda.js driven through
// process() with batchFrames K against a stand-in addon whose extractInto returns at once, so the time
// per launch is the facade's own (ring copies, result views, one callback object per buffer).
// usage: node tools/facade_overhead.js [K=64] [N=1024]
const path = require('path');
process.env.MEYDA_AMD_ADDON = path.join(__dirname, 'facade_overhead_addon.js');
const Meyda = require(path.join(__dirname, '..', 'meyda_amd', 'js', 'meyda.js'));

const K = +(process.argv[2] || 64), N = +(process.argv[3] || 1024);
const ALL = ['rms', 'energy', 'zcr', 'spectralCentroid', 'spectralFlatness', 'spectralSlope', 'spectralRolloff',
  'spectralSpread', 'spectralSkewness', 'spectralKurtosis', 'loudness', 'perceptualSpread', 'perceptualSharpness', 'mfcc'];
const x = new Float32Array(N).map((_, i) => Math.sin(i));
for (const [label, feats] of [['c1 set', ['rms', 'spectralCentroid']], ['every feature', ALL]]) {
  let sink = 0;
  const m = new Meyda({ sampleRate: 44100 }, null, N, (f) => { sink += f.rms; }, { batchFrames: K });
  m.start(feats);
  const launches = Math.max(2000, Math.floor(200000 / K));
  for (let w = 0; w < 200 * K; w++) m.process(x);  // warm-up (JIT)
  const t0 = process.hrtime.bigint();
  for (let b = 0; b < launches * K; b++) m.process(x);
  const us = Number(process.hrtime.bigint() - t0) / 1e3 / launches;
  console.log(JSON.stringify({ features: label, batchFrames: K, N, us_per_launch: +us.toFixed(2),
    us_per_buffer: +(us / K).toFixed(3), sink: sink > 0 }));
}
