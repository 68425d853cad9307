#!/usr/bin/env python3
"""A/B of the batch schedules in one process (kernels.hip extract_kernel: static rank shares against
run-time units of U groups, KernelArgs::dyn): every plan extracts the same device frames with every
feature; outputs compared bit for bit against the static plan; then interleaved rounds of 20 launches
serialised on one stream (the bench's kernel_ms) and 40 launches pipelined over two streams (its period).
usage: python tools/dyn_ab.py [N ...]   (env DYN="1:2 1:4 2:2" -- mode:unit pairs, ROUNDS=7)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from meyda_amd import capi  # noqa: E402


def make_plan(n, dyn, unit, mode=1):
    os.environ["MGX_DYN"] = "1" if dyn else "0"
    os.environ["MGX_DYN_UNIT"] = str(unit)
    os.environ["MGX_DYN_MODE"] = str(mode)
    try:
        return capi.Plan(buffer_size=n)
    finally:
        del os.environ["MGX_DYN"], os.environ["MGX_DYN_UNIT"], os.environ["MGX_DYN_MODE"]


def main():
    ns = [int(a) for a in sys.argv[1:]] or [1024, 2048, 512]
    specs = [tuple(int(t) for t in v.split(":")) for v in os.environ.get("DYN", "1:2 1:4 2:1 2:2").split()]
    rounds = int(os.environ.get("ROUNDS", "7"))
    s0, s1 = torch.cuda.current_stream(), torch.cuda.Stream()
    for n in ns:
        F = int(os.environ.get("FRAMES", "262144"))
        x = torch.empty(F, n, dtype=torch.float32, device="cuda")
        capi.synth_frames_device(x, 0x6D657964)
        variants = [("static", make_plan(n, False, 2))] + [("m%du%d" % (m, u), make_plan(n, True, u, m)) for m, u in specs]
        feats = capi.ALL_FEATURES
        ref = None
        sets = {}
        for name, p in variants:
            sets[name] = [p.alloc_outputs(F, feats) for _ in range(2)]
            p.extract_device(x.data_ptr(), F, sets[name][0][1], s0.cuda_stream)
            torch.cuda.synchronize()
            out = {k: v.clone() for k, v in sets[name][0][0].items()}
            if ref is None:
                ref = out
            else:
                same = all(torch.equal(out[k].view(torch.int32), ref[k].view(torch.int32)) for k in ref)
                print("N=%d %s outputs identical to static: %s" % (n, name, same), flush=True)
        res = {name: {"serial": [], "piped": []} for name, _ in variants}
        # settle the clock
        for _ in range(30):
            for name, p in variants:
                p.extract_device(x.data_ptr(), F, sets[name][0][1], s0.cuda_stream)
        torch.cuda.synchronize()
        for r in range(rounds):
            for name, p in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s0)
                for _ in range(20):
                    p.extract_device(x.data_ptr(), F, sets[name][0][1], s0.cuda_stream)
                e1.record(s0)
                torch.cuda.synchronize()
                res[name]["serial"].append(e0.elapsed_time(e1) / 20)
                ev = torch.cuda.Event()
                ev.record(s0)
                s1.wait_event(ev)
                e0.record(s0)
                for k in range(40):
                    st = s0 if k % 2 == 0 else s1
                    p.extract_device(x.data_ptr(), F, sets[name][k % 2][1], st.cuda_stream)
                ev2 = torch.cuda.Event()
                ev2.record(s1)
                s0.wait_event(ev2)
                e1.record(s0)
                torch.cuda.synchronize()
                res[name]["piped"].append(e0.elapsed_time(e1) / 40)
        base = np.median(res["static"]["serial"]), np.median(res["static"]["piped"])
        for name, _ in variants:
            a, b = np.median(res[name]["serial"]), np.median(res[name]["piped"])
            print("N=%d %-7s serial %.4f ms (%+.1f %%)  pipelined %.4f ms (%+.1f %%)  [min %.4f / %.4f]"
                  % (n, name, a, 100 * (a / base[0] - 1), b, 100 * (b / base[1] - 1),
                     min(res[name]["serial"]), min(res[name]["piped"])), flush=True)
        for _, p in variants:
            p.close()
        del x, sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
