'use strict';
// Times the JavaScript CPU restatement of the reference path (meyda_cpu.js) on the host's
// cores: the cpu_baseline leg of bench.py. CPU BASELINE ONLY (oracle/).
//
// usage: node bench_cpu.js N SECONDS THREADS [layout] [set]
// Each worker_thread synthesises 64 frames of the seeded stream (SURVEY.md §8(d)) at its
// own offset and extracts one feature set of them in a loop for SECONDS; prints one JSON
// line: frames/s over all threads, the per-thread rate, the CPU model and Node version.
// Sets (the GPU configs of BASELINE.json): all (every feature, 26 mel bands; C3+C4 and C5),
// c2 (amplitudeSpectrum + spectralCentroid), c3 (spectral* + loudness + perceptual),
// c4 (40-band mel + 13 MFCC); c1 times get(['rms', 'spectralCentroid']) on sound1.wav's
// frame 0 (tests/golden, N = 512) per call on this thread: median us per call.
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');
const os = require('os');
const path = require('path');

const SEED = 0x6D657964;
const SAMPLE = 64;

// C1 (BASELINE.json configs[0]): one 512-sample frame of sound1.wav, get(['rms',
// 'spectralCentroid']) per call: window, fresh complex array, FFT, amplitude, then rms.js
// and spectralCentroid.js (src/meyda.js:69-91,244-261), timed call by call.
function c1(seconds) {
  const fs = require('fs');
  const { CpuMeyda, mu } = require(path.join(__dirname, 'meyda_cpu.js'));
  const dir = path.join(__dirname, '..', '..', 'tests', 'golden');
  const man = JSON.parse(fs.readFileSync(path.join(dir, 'manifest.json'), 'utf8')).sizes['512'];
  const b = fs.readFileSync(path.join(dir, man.files.input));
  const all = new Float32Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength));
  const i = man.labels.indexOf('sound1:0');
  const x = all.slice(i * 512, (i + 1) * 512);
  const m = new CpuMeyda({ bufferSize: 512 });
  const get = () => {
    const a = m.spectrum(x);
    let e = 0;
    for (let k = 0; k < 512; k++) e += x[k] * x[k];
    return { rms: Math.sqrt(e / 512), spectralCentroid: mu(1, a) };
  };
  for (let k = 0; k < 200; k++) get();  // warm the JIT
  const us = [];
  const t0 = process.hrtime.bigint();
  let r;
  while (Number(process.hrtime.bigint() - t0) * 1e-9 < seconds || us.length < 1000) {
    const a = process.hrtime.bigint();
    r = get();
    us.push(Number(process.hrtime.bigint() - a) * 1e-3);
  }
  us.sort((p, q) => p - q);
  console.log(JSON.stringify({
    set: 'c1', us_per_call: us[us.length >> 1], us_p90: us[Math.floor(us.length * 0.9)], calls: us.length,
    rms: r.rms, spectralCentroid: r.spectralCentroid, cpu_model: os.cpus()[0].model, node: process.version,
  }));
}

if (isMainThread) {
  const N = parseInt(process.argv[2] || '1024', 10);
  const seconds = parseFloat(process.argv[3] || '5');
  const threads = parseInt(process.argv[4] || '1', 10);
  const layout = process.argv[5] || 'reference';
  const set = process.argv[6] || 'all';
  if (set === 'c1') {
    c1(seconds);
    return;
  }
  const t0 = Date.now();
  let done = 0;
  const res = [];
  for (let i = 0; i < threads; i++) {
    const w = new Worker(__filename, { workerData: { N, seconds, layout, set, first: i * SAMPLE } });
    w.on('message', (m) => {
      res.push(m);
      if (++done === threads) {
        const frames = res.reduce((a, r) => a + r.frames, 0);
        const wall = Math.max(...res.map((r) => r.seconds));
        console.log(JSON.stringify({
          value: frames / wall, unit: 'frames/s', threads, layout, set, bufferSize: N, frames,
          seconds: wall, per_thread: res.map((r) => r.frames / r.seconds),
          cpu_model: os.cpus()[0].model, logical_cpus: os.cpus().length, node: process.version,
          wall_s: (Date.now() - t0) / 1000,
        }));
      }
    });
    w.on('error', (e) => { console.error(e); process.exit(1); });
  }
} else {
  const { CpuMeyda, synthFrames, mu } = require(path.join(__dirname, 'meyda_cpu.js'));
  const { N, seconds, layout, set, first } = workerData;
  const m = new CpuMeyda({ bufferSize: N, layout, numMelBands: set === 'c4' ? 40 : 26 });
  const x = synthFrames(SEED, first, SAMPLE, N);
  const sc = new Float64Array(13), spec = new Float32Array(24), mf = new Float32Array(13);
  const sets = {
    all: (f) => m.frame(f, sc, spec, mf),
    c2: (f) => { sc[3] = mu(1, m.spectrum(f)); },  // spectralCentroid.js: mu(1, ampSpectrum)
    c3: (f) => m.frame(f, sc, spec, null, true),
    c4: (f) => { m.spectrum(f); m.mfcc(mf); },
  };
  const run = sets[set];
  if (!run) throw new Error('unknown set ' + set);
  const frame = (i) => run(x.subarray(i * N, (i + 1) * N));
  for (let i = 0; i < 4; i++) frame(i);  // warm the JIT
  let frames = 0;
  const t0 = process.hrtime.bigint();
  let el = 0;
  while (el < seconds) {
    for (let i = 0; i < SAMPLE; i++) frame(i);
    frames += SAMPLE;
    el = Number(process.hrtime.bigint() - t0) * 1e-9;
  }
  parentPort.postMessage({ frames, seconds: el });
}
