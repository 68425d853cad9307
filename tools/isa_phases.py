#!/usr/bin/env python3
"""Static per-phase instruction counts of one extract_kernel instance, from an assembly
listing built with -DMGX_MARKS (tools/isa.sh OUT.s -DMGX_MARKS): the instructions between
consecutive `;mgxmark` comments, by class (f64 arithmetic, f32<->f64 conversions, other
VALU, LDS, vector memory, scalar).
usage: isa_phases.py FILE.s [N] [SUB[,LIGHT[,NOTIME]]]"""
import re
import sys
from collections import Counter, OrderedDict


def kernel_lines(path, n, sub):
    # extract_kernel<N, FAITH, LITERAL, SUB, LIGHT, NOTIME>; sub = SUB or "sub,light,notime"
    flags = [int(v) for v in str(sub).split(",")] + [0, 0, 0, 0]
    # extract_kernel<N, FAITH, LITERAL, SUB, LIGHT, NOTIME, CHAIN, INL = false>
    name = "_ZN3mgx12_GLOBAL__N_114extract_kernelILi%dELb1ELb0ELb%dELb%dELb%dELb%dELb0EEEv" % (n, *flags[:4])
    lines = open(path).read().split("\n")
    start = [i for i, l in enumerate(lines) if l.startswith(name) and l.split(";")[0].rstrip().endswith(":")][0]
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        out.append(l.strip())
    return out


def cls(op):
    if op.startswith("v_cvt_f32_f64") or op.startswith("v_cvt_f64_f32"):
        return "cvt"
    if op.startswith("v_") and "f64" in op and "mfma" not in op:
        return "f64"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    sub = sys.argv[3] if len(sys.argv) > 3 else "0"
    seg = "prologue"
    counts = OrderedDict()
    order = []
    for l in kernel_lines(path, n, sub):
        m = re.search(r";mgxmark (\w+)", l)
        if m:
            seg = m.group(1)
            continue
        if not l or l.startswith(";") or l.startswith(".") or l.endswith(":"):
            continue
        op = l.split()[0]
        key = "%04d %s" % (len(order), seg)
        if not order or order[-1] != seg:
            order.append(seg)
            key = "%04d %s" % (len(order) - 1, seg)
        counts.setdefault(key, Counter())[cls(op)] += 1
    hdr = ["f64", "cvt", "valu", "lds", "vmem", "salu"]
    print("%-28s" % "segment (after mark)" + "".join("%7s" % h for h in hdr) + "  VALU-total")
    tot = Counter()
    for k, c in counts.items():
        tot.update(c)
        print("%-28s" % k + "".join("%7d" % c[h] for h in hdr) + "  %7d" % (c["f64"] + c["cvt"] + c["valu"]))
    print("%-28s" % "TOTAL(static)" + "".join("%7d" % tot[h] for h in hdr))


if __name__ == "__main__":
    main()
