#!/usr/bin/env python3
"""Where a one-frame host call's time goes (the real-time path): a diagnostic
library (tools/variant.sh wt -DMGX_WAVE_TIMES=1 -> ab/lib_wt.so) stamps the 100 MHz real-time clock
at the phases of the first wave's frame (kernels.hip MGX_STAMP); this runs mgx_extract_host on one
frame many times (the small host path: pinned mapped memory, completion word) and prints, for the
last calls, the median time from the kernel's first instruction to each stamp, and the call's own
duration on the host, and the shader clock the launch ran at (clock64 ticks over real time). With --resident the
plan is MGX_FLAG_RESIDENT: the stamps then count from the request's frame taken from the mailbox (stamp 0), the
last two bracket the completion word's release. usage: small_stamps.py LIB [--resident] [N features ...]"""
import ctypes
import json
import sys
import time
import types

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from meyda_amd import capi  # noqa: E402

NAMES = ["start", "prologue barrier", "tables, first load issued", "frame in, window, stage 0", "FFT", "amplitude",
         "moments, prefix, rolloff", "band sums", "mel, frame end", "phase 2 start", "phase 2 end", "before completion",
         "after completion"]


def main():
    args = [a for a in sys.argv[1:] if a != "--resident"]
    resident = "--resident" in sys.argv
    lib = args[0]
    L = ctypes.CDLL(lib)
    L.mgx_plan_create.argtypes = [ctypes.POINTER(capi.PlanDesc), ctypes.POINTER(ctypes.c_void_p)]
    L.mgx_extract_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(capi.Outputs)]
    cases = [(512, ["rms", "spectralCentroid"]), (1024, capi.ALL_FEATURES)]
    if len(args) > 1:
        cases = [(int(args[1]), args[2:] or capi.ALL_FEATURES)]
    for n, feats in cases:
        d = capi.make_desc(buffer_size=n, scalar_f64=True, resident=resident)
        h = ctypes.c_void_p()
        assert L.mgx_plan_create(ctypes.byref(d), ctypes.byref(h)) == 0
        x = np.random.default_rng(1).uniform(-1, 1, (1, n)).astype(np.float32)
        shim = types.SimpleNamespace(n=n, scalar_dtype=np.float64, desc=d)
        out, o = capi.Plan._host_outputs(shim, 1, feats)
        stamps, calls, sclk = [], [], []
        buf = (ctypes.c_ulonglong * 16)()
        for k in range(3000):
            t0 = time.perf_counter()
            assert L.mgx_extract_host(h, x.ctypes.data, 1, ctypes.byref(o)) == 0
            calls.append(time.perf_counter() - t0)
            if k >= 1000 and k % 10 == 0:
                if resident:  # (the launch's last stamps of this request land just after the call returns)
                    t1 = time.perf_counter()
                    while time.perf_counter() - t1 < 50e-6:
                        pass
                assert L.mgx_debug_stamps(buf) == 0
                s = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
                stamps.append((s[:13] - s[0]) * 10e-3)  # 100 MHz ticks -> us
                sclk.append((s[14] - s[13]) / max(1, s[12] - s[0]) * 100.0)  # shader clocks per us -> MHz
        st = np.median(np.array(stamps), axis=0)
        print(json.dumps({"n": n, "features": len(feats), "host_call_us": float(np.median(calls[1000:]) * 1e6),
                          "kernel_us_by_stamp": {NAMES[i]: round(float(st[i]), 2) for i in range(13)},
                          "shader_clock_mhz": round(float(np.median(sclk)), 1)}))


if __name__ == "__main__":
    main()
