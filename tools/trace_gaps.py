#!/usr/bin/env python3
"""GPU busy/idle accounting of a timed region from a rocprofv3 kernel trace
(and, if given, its memory-copy trace): how much of the wall time between the
first and last dispatch of the timed steps had no kernel running, and which
kernels ran concurrently. Used on the C5 stream drain, whose wall time exceeds
the sum of its sections' standalone kernel times.

usage: trace_gaps.py kernel_trace.csv [memory_copy_trace.csv] [--skip-before NAME]
  --skip-before NAME: ignore everything before the last dispatch whose kernel
  name contains NAME (e.g. corpus generation kernels before the timed steps)
"""
import csv
import sys


def load(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r.get("Kernel_Name") or r.get("Direction") or kind
        out.append((s, e, name.split("(")[0][-48:], kind))
    return out


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    args = [a for a in sys.argv[1:]]
    skip = None
    if "--skip-before" in args:
        i = args.index("--skip-before")
        skip = args[i + 1]
        del args[i:i + 2]
    ev = load(args[0], "kernel")
    if len(args) > 1:
        ev += load(args[1], "copy")
    ev.sort()
    if skip:
        last = max(i for i, x in enumerate(ev) if skip in x[2])
        ev = ev[last + 1:]
    t0, t1 = min(x[0] for x in ev), max(x[1] for x in ev)
    wall = t1 - t0
    kern = [(s, e) for s, e, n, k in ev if k == "kernel"]
    busy = union(kern)
    per = {}
    for s, e, n, k in ev:
        per.setdefault((k, n), [0, 0])
        per[(k, n)][0] += 1
        per[(k, n)][1] += e - s
    print("window %.2f ms, kernels busy %.2f ms (%.1f%%), no kernel running %.2f ms" %
          (wall / 1e6, busy / 1e6, 100.0 * busy / wall, (wall - busy) / 1e6))
    print("sum of kernel durations %.2f ms (overlap factor %.2f)" % (sum(e - s for s, e in kern) / 1e6,
                                                                    sum(e - s for s, e in kern) / max(busy, 1)))
    for (k, n), (c, d) in sorted(per.items(), key=lambda x: -x[1][1]):
        print("  %-6s %-48s %5d  %10.2f ms" % (k, n, c, d / 1e6))
    # idle gaps between kernels, largest first
    kern.sort()
    gaps, end = [], kern[0][1]
    for s, e in kern[1:]:
        if s > end:
            gaps.append((s - end, end - t0))
        end = max(end, e)
    gaps.sort(reverse=True)
    print("largest idle gaps (ms at offset ms):", ", ".join("%.2f@%.1f" % (g / 1e6, o / 1e6) for g, o in gaps[:12]))


if __name__ == "__main__":
    main()
