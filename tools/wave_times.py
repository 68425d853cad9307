#!/usr/bin/env python3
"""Wave lifetimes of one extraction launch (diagnostic build abl/libabl_wt.so, -DMGX_WAVE_TIMES=1):
every wave's start, end of prologue and end on the 100 MHz real-time clock plus its CU id, for
the last of a run of back-to-back launches on one stream (the persistent grid, or an
over-subscribed one with MGX_GRID_CAP). Prints the start ramp, the prologue, the finishing
spread (the drain) and the mean end per XCD, relative to the launch.
usage: wave_times.py LIB [--n N] [--frames F] [--features a,b,...]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from meyda_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=262144)
    ap.add_argument("--features", default="all", help="comma-separated feature names (default every per-frame feature)")
    a = ap.parse_args()
    n, F = a.n, a.frames
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0x6D657964)
    plan0 = capi.Plan(buffer_size=n)
    feats = capi.ALL_FEATURES if a.features == "all" else a.features.split(",")
    _, o = plan0.alloc_outputs(F, feats)
    L = ctypes.CDLL(a.lib)
    L.mgx_plan_create.argtypes = [ctypes.POINTER(capi.PlanDesc), ctypes.POINTER(ctypes.c_void_p)]
    L.mgx_extract_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.POINTER(capi.Outputs), ctypes.c_void_p]
    d = capi.make_desc(buffer_size=n)
    h = ctypes.c_void_p()
    assert L.mgx_plan_create(ctypes.byref(d), ctypes.byref(h)) == 0
    s = torch.cuda.current_stream()
    for _ in range(40):
        L.mgx_extract_device(h, ctypes.c_void_p(x.data_ptr()), F, ctypes.byref(o), ctypes.c_void_p(s.cuda_stream))
    torch.cuda.synchronize()
    cnt = 65536 * 4
    buf = (ctypes.c_ulonglong * cnt)()
    assert L.mgx_debug_wave_times(buf, cnt) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4)
    t = t[t[:, 2] > 0]
    t0, t1, t2 = (t[:, i].astype(np.int64) for i in range(3))
    cu = (t[:, 3] & 0xFFFFFFFF).astype(np.int64)
    wg = (t[:, 3] >> 32).astype(np.int64)
    # keep the waves of the last launch: the ones ending within 5 ms of the latest end
    keep = t2 > t2.max() - 500000
    t0, t1, t2, cu, wg = t0[keep], t1[keep], t2[keep], cu[keep], wg[keep]
    base = t0.min()
    us = lambda v: (v - base) / 100.0  # 100 MHz ticks -> us
    span = us(t2.max())
    print("waves %d (workgroups %d), launch span %.1f us" % (len(t0), len(np.unique(wg)), span))
    for name, v in (("start", us(t0)), ("prologue end", us(t1)), ("end", us(t2))):
        q = np.percentile(v, [0, 1, 10, 50, 90, 99, 100])
        print("%-13s pct 0/1/10/50/90/99/100: %s us" % (name, " ".join("%.1f" % z for z in q)))
    print("prologue length median %.2f us" % np.median((t1 - t0) / 100.0))
    xcd = wg % 8
    for k in range(8):
        m = xcd == k
        print("XCD %d (wg %% 8): waves %d  end mean %.1f  min %.1f  max %.1f us" % (k, m.sum(), us(t2[m]).mean(), us(t2[m]).min(), us(t2[m]).max()))
    # which waves finish first: by workgroup rank groups and by the wave's index in its workgroup
    ng = len(np.unique(wg))
    ranks = max(1, ng // 256)  # workgroups per CU of the persistent grid (256 CUs): rank = wg // (grid / ranks)
    for name, key in (("rank wg//(grid/%d)" % ranks, wg // max(1, ng // ranks)), ("wave in wg", np.arange(len(wg)) % 4)):
        print("end by %-15s: %s" % (name, "  ".join("%d:%.0f" % (k, us(t2[key == k]).mean()) for k in np.unique(key)[:8])))
    rk = wg // max(1, ng // ranks)
    for k in np.unique(rk):
        q = np.percentile(us(t2[rk == k]), [0, 10, 50, 90, 100])
        print("rank %d end pct 0/10/50/90/100: %s us" % (k, " ".join("%.0f" % z for z in q)))
    # resident waves over time: what fraction of the 16 slots per CU x 256 CUs is alive
    grid = np.linspace(0, span, 41)
    alive = [((us(t0) <= g) & (us(t2) > g)).sum() for g in grid]
    print("alive waves over the launch (41 samples):", " ".join(str(v) for v in alive))
    area = np.sum((t2 - t0) / 100.0)
    slots = 1024 * ranks
    print("mean resident waves %.1f of %d slots (%.3f)" % (area / span, slots, area / span / slots))


if __name__ == "__main__":
    main()
