"""Writes small RIFF/WAVE files for the ingest tests, and decodes PCM the way the
browser's decodeAudioData does (the reference's decoder: lib/bufferLoader.js:23)."""
import struct

import numpy as np

TAGS = {"u8": (1, 8), "s16": (1, 16), "s24": (1, 24), "s32": (1, 32), "f32": (3, 32)}
DTYPES = {"u8": np.uint8, "s16": "<i2", "s32": "<i4", "f32": "<f4"}


def encode(samples, fmt):
    """samples: (frames, channels) integer codes (or float32 for f32) -> interleaved bytes."""
    a = np.asarray(samples)
    if fmt == "s24":
        v = a.astype(np.int64).reshape(-1) & 0xFFFFFF
        b = np.stack([v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF], axis=1).astype(np.uint8)
        return b.tobytes()
    return a.astype(DTYPES[fmt]).tobytes()


def decode(samples, fmt):
    """The float32 values decodeAudioData yields for integer codes `samples`."""
    a = np.asarray(samples)
    if fmt == "u8":
        return ((a.astype(np.float64) - 128) / 128).astype(np.float32)
    if fmt == "s16":
        return (a.astype(np.float64) / 32768).astype(np.float32)
    if fmt == "s24":
        return (a.astype(np.float64) / 8388608).astype(np.float32)
    if fmt == "s32":
        return (a.astype(np.float64) / 2147483648).astype(np.float32)
    return a.astype(np.float32)


def random_codes(rng, frames, channels, fmt):
    shape = (frames, channels)
    if fmt == "u8":
        return rng.integers(0, 256, shape)
    if fmt == "s16":
        return rng.integers(-32768, 32768, shape)
    if fmt == "s24":
        return rng.integers(-(1 << 23), 1 << 23, shape)
    if fmt == "s32":
        return rng.integers(-(1 << 31), 1 << 31, shape, dtype=np.int64)
    return rng.standard_normal(shape).astype(np.float32)


def wav_bytes(samples, fmt, rate=44100, fmt_size=16, extensible=False, extra_chunks=(), pad_data=b"",
              truncate=0):
    """A WAV file with the given integer codes; fmt chunk of 16/18 bytes or 40
    (WAVE_FORMAT_EXTENSIBLE); extra chunks (id, payload) before the data chunk."""
    a = np.asarray(samples)
    frames, channels = a.shape
    tag, bits = TAGS[fmt]
    align = channels * bits // 8
    if extensible:
        fmt_payload = struct.pack("<HHIIHH", 0xFFFE, channels, rate, rate * align, align, bits)
        fmt_payload += struct.pack("<HHI", 22, bits, 0) + struct.pack("<H", tag) + bytes(14)
    else:
        fmt_payload = struct.pack("<HHIIHH", tag, channels, rate, rate * align, align, bits)
        if fmt_size == 18:
            fmt_payload += struct.pack("<H", 0)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt_payload)) + fmt_payload
    for cid, payload in extra_chunks:
        body += cid + struct.pack("<I", len(payload)) + payload + (b"\0" if len(payload) & 1 else b"")
    data = encode(a, fmt) + pad_data
    body += b"data" + struct.pack("<I", len(data)) + data
    out = b"RIFF" + struct.pack("<I", len(body)) + body
    return out[:len(out) - truncate] if truncate else out
