#!/usr/bin/env python3
"""Static instruction histogram of one extract_kernel instance from tools/isa.sh output.
usage: isa_hist.py FILE.s [N] [FAITH LITERAL] [--diff OTHER.s] [--range START_LABEL END_LABEL]"""
import re
import sys
from collections import Counter


def body(path, n=1024, faith=1, lit=0):
    names = ["_ZN3mgx12_GLOBAL__N_114extract_kernelILi%dELb%dELb%dELb0ELb0ELb0ELb0EEEvNS_10KernelArgsE" % (n, faith, lit),
             "_ZN3mgx12_GLOBAL__N_114extract_kernelILi%dELb%dELb%dELb0ELb0ELb0EEEvNS_10KernelArgsE" % (n, faith, lit)]
    lines = open(path).read().split("\n")
    start = [i for i, l in enumerate(lines) if any(l.startswith(nm + ":") for nm in names)][0]
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        out.append(l)
    return out


def hist(lines):
    c = Counter()
    for l in lines:
        l = l.strip()
        if not l or l.startswith(";") or l.startswith(".") or l.endswith(":"):
            continue
        op = l.split()[0]
        c[op] += 1
    return c


def classes(c):
    k = Counter()
    for op, v in c.items():
        if op.startswith("v_cvt"):
            k["cvt"] += v
        elif op.startswith("v_") and "f64" in op:
            k["f64"] += v
        elif op.startswith("v_pk_"):
            k["pk"] += v
        elif op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
            k["lane"] += v
        elif op.startswith("v_"):
            k["valu_other"] += v
        elif op.startswith("ds_"):
            k["ds"] += v
        elif op.startswith("global_") or op.startswith("buffer_"):
            k["vmem"] += v
        elif op.startswith("s_nop"):
            k["s_nop"] += v
        elif op.startswith("s_waitcnt"):
            k["waitcnt"] += v
        elif op.startswith("s_"):
            k["salu"] += v
        else:
            k["other"] += v
    return k


if __name__ == "__main__":
    a = sys.argv[1:]
    n = int(a[1]) if len(a) > 1 and not a[1].startswith("-") else 1024
    ca = hist(body(a[0], n))
    if "--diff" in a:
        cb = hist(body(a[a.index("--diff") + 1], n))
        d = Counter(ca)
        d.subtract(cb)
        print("class diff:", dict(classes(Counter({k: v for k, v in d.items() if v > 0}))))
        for op, v in sorted(d.items(), key=lambda t: -abs(t[1]))[:40]:
            if v:
                print("%6d %s" % (v, op))
    else:
        print("classes:", dict(classes(ca)))
        for op, v in ca.most_common(50):
            print("%6d %s" % (v, op))
