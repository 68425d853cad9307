'use strict';
// Builds a 16-bit PCM .wav file in memory (for the ingest tests).
function wavS16(codes, channels, rate) {
  const frames = codes.length / channels;
  const data = Buffer.alloc(codes.length * 2);
  for (let i = 0; i < codes.length; i++) data.writeInt16LE(codes[i], 2 * i);
  const fmt = Buffer.alloc(16);
  fmt.writeUInt16LE(1, 0); fmt.writeUInt16LE(channels, 2); fmt.writeUInt32LE(rate, 4);
  fmt.writeUInt32LE(rate * channels * 2, 8); fmt.writeUInt16LE(channels * 2, 12); fmt.writeUInt16LE(16, 14);
  const chunk = (id, b) => { const h = Buffer.alloc(8); h.write(id, 0, 'ascii'); h.writeUInt32LE(b.length, 4); return Buffer.concat([h, b]); };
  const body = Buffer.concat([Buffer.from('WAVE'), chunk('fmt ', fmt), chunk('LIST', Buffer.from('info')), chunk('data', data)]);
  const head = Buffer.alloc(8); head.write('RIFF', 0, 'ascii'); head.writeUInt32LE(body.length, 4);
  void frames;
  return Buffer.concat([head, body]);
}
module.exports = { wavS16 };
