#!/usr/bin/env python3
"""Where a gather-inclusive step's time goes in the cross-process rehearsal (MGX_GROUP_TRANSPORT=ipc):
reads the host timestamps group.cpp writes under $MGX_GROUP_TRACE (PREFIX.<rank>, one line per event:
"ns rank tag chunk peer"; a call's first line carries its chunk count and bufferSize) and splits each group call, per rank, into
  * the host's waits inside the hand-over: a peer waiting for its chunk's extraction to complete before
    posting it (post_wait -> posted), a peer waiting for the root to free a transfer slot (slot_wait ->
    slot_free), the root waiting for a peer's post (take_wait -> taken), the root waiting for its copies
    (fin_wait -> consumed);
  * the rest of the call (enqueueing extractions, copies and unpacks).
The last K calls of each rank are the timed steps' (bench.py); the first ones are warm-up.
usage: gather_trace.py PREFIX [--last K]"""
import argparse
import collections
import glob


def load(prefix):
    by_rank = collections.defaultdict(list)
    for path in sorted(glob.glob(prefix + ".*")):
        for line in open(path):
            ns, rank, tag, chunk, peer = line.split()
            by_rank[int(rank)].append((int(ns), tag, int(chunk), int(peer)))
    calls = {}
    for r, evs in by_rank.items():
        cs = []
        for e in evs:
            if e[1] == "call":
                cs.append([])
            if cs:
                cs[-1].append(e)
        calls[r] = cs
    return calls


def waits(call):
    """Sum of each kind of wait in one call (ms), and the call's host span."""
    pairs = {"post_wait": "posted", "slot_wait": "slot_free", "take_wait": "taken", "fin_wait": "consumed"}
    open_at = {}
    tot = collections.Counter()
    for ns, tag, chunk, peer in call:
        if tag in pairs:
            open_at[(pairs[tag], chunk)] = ns
        elif (tag, chunk) in open_at:
            tot[tag] += ns - open_at.pop((tag, chunk))
    span = call[-1][0] - call[0][0]
    return {k: v / 1e6 for k, v in tot.items()}, span / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--last", type=int, default=20, help="calls to average (the timed steps)")
    a = ap.parse_args()
    allcalls = load(a.prefix)
    sizes = sorted({c[0][3] for cs in allcalls.values() for c in cs})
    for n in sizes:
        print("## bufferSize %d" % n)
        report({r: [c for c in cs if c[0][3] == n] for r, cs in allcalls.items()}, a.last)


def report(calls, last):
    for r in sorted(calls):
        cs = calls[r][-last:]
        acc = collections.Counter()
        span = 0.0
        for c in cs:
            w, s = waits(c)
            acc.update(w)
            span += s
        n = max(1, len(cs))
        role = "root" if r == 0 else "peer"
        parts = ", ".join("%s %.3f" % (k, v / n) for k, v in sorted(acc.items()))
        print("rank %d (%s): %d calls, host span %.3f ms per call; waits per call (ms): %s; rest %.3f"
              % (r, role, len(cs), span / n, parts, (span - sum(acc.values())) / n))
    # the hand-over latency: a peer's post to the root's copy of it (same host clock)
    if 0 in calls and 1 in calls:
        lat = []
        for c0, c1 in zip(calls[0][-last:], calls[1][-last:]):
            posted = {ch: ns for ns, tag, ch, p in c1 if tag == "posted"}
            for ns, tag, ch, p in c0:
                if tag == "taken" and p == 1 and ch in posted:
                    lat.append((ns - posted[ch]) / 1e3)
        if lat:
            lat.sort()
            print("post -> root's copy issued: median %.1f us, p90 %.1f us, max %.1f us over %d chunks"
                  % (lat[len(lat) // 2], lat[int(0.9 * (len(lat) - 1))], lat[-1], len(lat)))


if __name__ == "__main__":
    main()
