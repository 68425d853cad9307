"""Loader for the committed golden fixtures (tests/golden/, made by tools/gen_golden.js)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_DTYPES = {".f32": np.float32, ".f64": np.float64, ".i32": np.int32}


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load(n):
    """Return a dict: labels, frames (F x N), and every fixture array, reshaped."""
    m = manifest()
    s = m["sizes"][str(n)]
    F = s["frames"]
    out = {"labels": s["labels"], "F": F, "N": n, "scalar_names": m["scalars"],
           "hamming_frames": s["hammingFrames"], "literal_frames": s["literalFrames"],
           "complex_frames": s["complexFrames"]}
    for key, rel in s["files"].items():
        ext = os.path.splitext(rel)[1]
        out[key] = np.fromfile(os.path.join(GOLDEN, rel), dtype=_DTYPES[ext])
    L = n // 2
    out["input"] = out["input"].reshape(F, n)
    out["amp"] = out["amp"].reshape(F, L)
    out["power"] = out["power"].reshape(F, L)
    out["complex_re"] = out["complex_re"].reshape(-1, n)
    out["complex_im"] = out["complex_im"].reshape(-1, n)
    out["scalars"] = out["scalars"].reshape(F, -1)
    out["loudness_specific"] = out["loudness_specific"].reshape(F, -1)
    out["mfcc"] = out["mfcc"].reshape(F, -1)
    out["mfcc40"] = out["mfcc40"].reshape(F, -1)
    out["hamming_amp"] = out["hamming_amp"].reshape(-1, L)
    out["hamming_scalars"] = out["hamming_scalars"].reshape(-1, out["scalars"].shape[1])
    out["hamming_mfcc"] = out["hamming_mfcc"].reshape(-1, 13)
    out["literal_amp"] = out["literal_amp"].reshape(-1, L)
    out["literal_loudness_specific"] = out["literal_loudness_specific"].reshape(-1, 24)
    return out


def idx(labels, prefix):
    return [i for i, l in enumerate(labels) if l.startswith(prefix)]
