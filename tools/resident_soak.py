#!/usr/bin/env python3
"""A soak of the resident real-time path (MGX_FLAG_RESIDENT): many one-frame calls on one
resident plan, a random frame each time, every 500th compared byte for byte with a plan that launches per
call; every 20,000 calls a 262,144-frame batch on a third plan runs beside the resident launch (its grid one
workgroup smaller), and every 50,000 calls the host idles past the launch's idle timeout, so the next call
starts a new launch. Prints the call-time distribution (median, p99, p99.9, max) and the checks.
usage: resident_soak.py [calls] [N]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from meyda_amd import capi  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    import torch
    feats = ["rms", "spectralCentroid"]
    res = capi.Plan(buffer_size=n, scalar_f64=True, resident=True)
    ref = capi.Plan(buffer_size=n, scalar_f64=True)
    big = capi.Plan(buffer_size=1024)
    xb = torch.empty(262144, 1024, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(xb, 0x6D657964)
    bout, bo = big.alloc_outputs(262144, ["rms", "spectralCentroid", "mfcc", "loudness"])
    rng = np.random.default_rng(11)
    pool = rng.uniform(-1, 1, (4096, n)).astype(np.float32)
    out, o = res._host_outputs(1, feats)
    L = capi.lib()
    t = np.empty(calls)
    checked = mism = batches = idles = 0
    t_start = time.time()
    for k in range(calls):
        x = pool[k % 4096]
        t0 = time.perf_counter_ns()
        rc = L.mgx_extract_host(res._h, x.ctypes.data, 1, ctypes.byref(o))
        t[k] = (time.perf_counter_ns() - t0) / 1e3
        if rc != 0:
            print(json.dumps({"error": L.mgx_last_error().decode(), "call": k}))
            return 1
        if k % 500 == 0:
            r = ref.extract(x[None, :], feats)
            checked += 1
            if any(not np.array_equal(out[f].view(np.uint8), r[f].view(np.uint8)) for f in feats):
                mism += 1
        if k % 20000 == 19999:
            s = torch.cuda.current_stream()
            big.extract_device(xb.data_ptr(), 262144, bo, s.cuda_stream)
            s.synchronize()
            batches += 1
        if k % 50000 == 49999:
            time.sleep(0.05)  # past the 20 ms idle timeout: the launch ends, the next call starts one
            idles += 1
        if k % 50000 == 0:
            print("progress %d calls, %.0f s" % (k, time.time() - t_start), file=sys.stderr, flush=True)
    res.close()
    ref.close()
    big.close()
    q = np.percentile(t, [50, 99, 99.9])
    print(json.dumps({"n": n, "calls": calls, "features": feats, "median_us": round(float(q[0]), 2),
                      "p99_us": round(float(q[1]), 2), "p999_us": round(float(q[2]), 2), "max_us": round(float(t.max()), 1),
                      "calls_over_100us": int((t > 100).sum()), "checked_against_launch_per_call": checked,
                      "mismatches": mism, "batches_beside": batches, "idle_restarts": idles,
                      # the slowest calls, with what preceded them (a batch on the third plan, an idle past the timeout)
                      "slowest": [{"call": int(i), "us": round(float(t[i]), 1),
                                   "after_batch": bool(i % 20000 == 0 and i > 0), "after_idle": bool(i % 50000 == 0 and i > 0)}
                                  for i in np.argsort(t)[::-1][:6]]}))
    return 0 if mism == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
