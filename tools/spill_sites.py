#!/usr/bin/env python3
"""Scratch (spill) loads and stores per extraction kernel, by loop depth.

A spill store inside the batch or frame loop runs once per iteration, and on gfx950 those
scratch writes reach HBM (WRITE_SIZE), so a kernel should have none inside its loops.
Usage: tools/isa.sh /tmp/k.s && python3 tools/spill_sites.py /tmp/k.s [kernel-substring]
"""
import re
import sys


def main(path, pat=""):
    txt = open(path).read()
    for part in re.split(r"\n(?=_ZN3mgx\S*:)", txt):
        m = re.match(r"(_ZN3mgx\S*extract_kernelILi(\d+)ELb(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)\S*):", part)
        if not m or pat not in m.group(1):
            continue
        depth = 0
        hist = {}
        for line in part.split("\n"):
            if re.match(r"^\.LBB|^; %bb", line):
                d = re.search(r"Depth=(\d+)", line)
                depth = int(d.group(1)) if d else 0
            op = re.match(r"\s+(scratch_(?:store|load)\S*)", line)
            if op:
                k = ("st" if "store" in op.group(1) else "ld", depth)
                hist[k] = hist.get(k, 0) + 1
        tag = "N=%s faith=%s lit=%s sub=%s light=%s notime=%s chain=%s" % m.group(2, 3, 4, 5, 6, 7, 8)
        print(tag, " ".join("%s@d%d:%d" % (k[0], k[1], v) for k, v in sorted(hist.items())) or "no scratch")


if __name__ == "__main__":
    main(*sys.argv[1:])
