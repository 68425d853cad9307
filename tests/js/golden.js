'use strict';
// Reads the committed golden fixtures (tests/golden/, made by tools/gen_golden.js).
const fs = require('fs');
const path = require('path');

const DIR = path.join(__dirname, '..', 'golden');
const manifest = JSON.parse(fs.readFileSync(path.join(DIR, 'manifest.json'), 'utf8'));

function read(rel) {
  const b = fs.readFileSync(path.join(DIR, rel));
  const ab = b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength);
  if (rel.endsWith('.f32')) return new Float32Array(ab);
  if (rel.endsWith('.f64')) return new Float64Array(ab);
  return new Int32Array(ab);
}

function load(n) {
  const s = manifest.sizes[String(n)];
  const out = { N: n, F: s.frames, labels: s.labels, scalarNames: manifest.scalars };
  for (const k of Object.keys(s.files)) out[k] = read(s.files[k]);
  return out;
}

module.exports = { manifest, load };
