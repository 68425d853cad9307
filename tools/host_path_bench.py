"""PCIe-inclusive rate of the host-buffer entry points (never the bench `value`):
mgx_extract_host (float32 frames in pageable host memory) and mgx_extract_host_pcm
(interleaved s16 PCM, decoded on the device), N=1024, all features, 262,144 frames."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from meyda_amd import capi  # noqa: E402

n, F = 1024, 262144
rng = np.random.default_rng(1)
frames = rng.random((F, n), dtype=np.float32) * 2 - 1
pcm = (frames.reshape(-1) * 32767).astype(np.int16)
plan = capi.Plan(buffer_size=n)
res = {}
for name, fn, nbytes in (
        ("float32_frames", lambda: plan.extract(frames, capi.ALL_FEATURES), frames.nbytes),
        ("s16_pcm", lambda: plan.extract_pcm(pcm, F * n, "s16", 1, 0, capi.ALL_FEATURES), pcm.nbytes)):
    fn()  # warm (staging buffers allocated)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    res[name] = {"frames_per_s": F / t, "ms": t * 1e3, "input_GBs": nbytes / t / 1e9, "input_bytes": nbytes}
    print(name, json.dumps(res[name]), flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "host_path.json"), "w"), indent=1)
