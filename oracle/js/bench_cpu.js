'use strict';
// Times the JavaScript CPU restatement of the reference path (meyda_cpu.js) on the host's
// cores: the cpu_baseline leg of bench.py. CPU BASELINE ONLY (oracle/).
//
// usage: node bench_cpu.js N SECONDS THREADS [layout]
// Each worker_thread synthesises 64 frames of the seeded stream (SURVEY.md §8(d)) at its
// own offset and extracts every feature of them in a loop for SECONDS; prints one JSON
// line: frames/s over all threads, the per-thread rate, the CPU model and Node version.
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');
const os = require('os');
const path = require('path');

const SEED = 0x6D657964;
const SAMPLE = 64;

if (isMainThread) {
  const N = parseInt(process.argv[2] || '1024', 10);
  const seconds = parseFloat(process.argv[3] || '5');
  const threads = parseInt(process.argv[4] || '1', 10);
  const layout = process.argv[5] || 'reference';
  const t0 = Date.now();
  let done = 0;
  const res = [];
  for (let i = 0; i < threads; i++) {
    const w = new Worker(__filename, { workerData: { N, seconds, layout, first: i * SAMPLE } });
    w.on('message', (m) => {
      res.push(m);
      if (++done === threads) {
        const frames = res.reduce((a, r) => a + r.frames, 0);
        const wall = Math.max(...res.map((r) => r.seconds));
        console.log(JSON.stringify({
          value: frames / wall, unit: 'frames/s', threads, layout, bufferSize: N, frames,
          seconds: wall, per_thread: res.map((r) => r.frames / r.seconds),
          cpu_model: os.cpus()[0].model, logical_cpus: os.cpus().length, node: process.version,
          wall_s: (Date.now() - t0) / 1000,
        }));
      }
    });
    w.on('error', (e) => { console.error(e); process.exit(1); });
  }
} else {
  const { CpuMeyda, synthFrames } = require(path.join(__dirname, 'meyda_cpu.js'));
  const { N, seconds, layout, first } = workerData;
  const m = new CpuMeyda({ bufferSize: N, layout });
  const x = synthFrames(SEED, first, SAMPLE, N);
  const sc = new Float64Array(13), spec = new Float32Array(24), mf = new Float32Array(13);
  const frame = (i) => m.frame(x.subarray(i * N, (i + 1) * N), sc, spec, mf);
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
