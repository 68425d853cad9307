#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per kernel name, count / mean / min / max of
the dispatch durations, over all dispatches and over the LAST k (the timed steps of a
bench run, after its clock-settle and warmup launches). With parts > 1 (a step of the
bench is that many launches: mgx_extract_device's parts on two streams), the step spans of
the matching kernel too: first start to last end of each group of `parts` dispatches, over
the last k steps -- the figure the bench's per-step HIP events measure.
With skip > 0 the last `skip` dispatches are left out first (bench.py's single-stream
launches after its timed steps: 20 with an event pair each, then 20 back to back, skip = 40), and for extract kernels the launch period of the k
dispatches before them is printed: (last end - first start) / k -- what bench.py's events
around its pipelined timed region measure (consecutive launches overlap by the drain).
usage: prof_summary.py KERNEL_TRACE.csv [k] [name-substring] [parts] [skip]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    sub = sys.argv[3] if len(sys.argv) > 3 else ""
    parts = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    skip = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    by = defaultdict(list)
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name", "")
        if sub and sub not in name:
            continue
        t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
        by[name].append((t0, t1))
    print("%-70s %6s %10s %10s %10s %10s" % ("kernel", "n", "mean_ms", "min_ms", "max_ms", "lastK_mean"))
    for name, v in sorted(by.items(), key=lambda kv: -sum(b - a for a, b in kv[1])):
        v.sort()
        v_all = list(v)
        if skip and "extract_kernel" in name and len(v) > skip:
            alone = [(b - a) * 1e-6 for a, b in v[-skip:]]
            v = v[:-skip]
            w = v[-k * parts:]
            period = (max(b for _, b in w) - w[0][0]) * 1e-6 / k
            print("  %s: launch period over the %d timed steps %.4f ms; the %d single-stream launches after "
                  "them: mean %.4f ms, median %.4f" % (name[:60], k, period, skip, sum(alone) / skip,
                                                        sorted(alone)[skip // 2]))
            if skip >= 40:
                # bench.py's last 20: back to back on one stream between one event pair (its kernel_ms)
                ser = v_all[-20:]
                print("  the last 20 (back to back, bench.py's launch_serial_ms): mean duration %.4f ms, "
                      "(last end - first start) / 20 = %.4f ms" % (sum((b - a) for a, b in ser) * 1e-6 / 20,
                                                                   (ser[-1][1] - ser[0][0]) * 1e-6 / 20))
        ts = [(b - a) * 1e-6 for a, b in v]  # ns -> ms
        kk = k * parts
        last = ts[-kk:]
        print("%-70s %6d %10.4f %10.4f %10.4f %10.4f" % (name[:70], len(ts), sum(ts) / len(ts), min(ts), max(ts),
                                                          sum(last) / len(last)))
        if parts > 1 and len(v) >= kk and "extract_kernel" in name:
            tail = v[-kk:]
            spans = [(max(b for _, b in tail[i:i + parts]) - tail[i][0]) * 1e-6 for i in range(0, kk, parts)]
            print("  step spans (%d launches per step, last %d steps): mean %.4f ms  min %.4f  max %.4f"
                  % (parts, k, sum(spans) / len(spans), min(spans), max(spans)))


if __name__ == "__main__":
    main()
