#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per kernel name, count / mean / min / max of
the dispatch durations, over all dispatches and over the LAST k (the timed steps of a
bench run, after its clock-settle and warmup launches).
usage: prof_summary.py KERNEL_TRACE.csv [k] [name-substring]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    sub = sys.argv[3] if len(sys.argv) > 3 else ""
    by = defaultdict(list)
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name", "")
        if sub and sub not in name:
            continue
        t = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6  # ns -> ms
        by[name].append((int(row["Start_Timestamp"]), t))
    print("%-70s %6s %10s %10s %10s %10s" % ("kernel", "n", "mean_ms", "min_ms", "max_ms", "lastK_mean"))
    for name, v in sorted(by.items(), key=lambda kv: -sum(t for _, t in kv[1])):
        v.sort()
        ts = [t for _, t in v]
        last = ts[-k:]
        print("%-70s %6d %10.4f %10.4f %10.4f %10.4f" % (name[:70], len(ts), sum(ts) / len(ts), min(ts), max(ts),
                                                          sum(last) / len(last)))


if __name__ == "__main__":
    main()
