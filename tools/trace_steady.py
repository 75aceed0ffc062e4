#!/usr/bin/env python3
"""Steady-state GPU occupancy of a pipelined run from a rocprofv3 kernel trace
(dev tool for c4h / c4h --components with calls in flight): the kernels are cut
into clusters at gaps of over 3 ms with no kernel running (the timed steps are
the cluster with the most ladder launches; corpus generation and the checks
after the timed region are others); over that cluster's window from its ladder
launch at fraction --from to its last ladder's end, the wall time, the time with at least one Ed25519 ladder running, with only
prep / id / other kernels running, and with nothing running; plus the summed
kernel time per class (concurrent kernels stretch each other, so the sums exceed
the union).

usage: trace_steady.py kernel_trace.csv [--from 0.4]"""
import csv
import sys
from collections import defaultdict

CLASSES = (("ladder", ("ed25519_ladder",)), ("prep", ("ed25519_prep",)),
           ("ids", ("kryo_", "sha256_leaves", "merkle_root", "rocprim", "gather_", "store_to_host")))


def cls(name):
    for c, keys in CLASSES:
        if any(k in name for k in keys):
            return c
    return "other"


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if cs is not None else 0)


def main():
    frac = float(sys.argv[sys.argv.index("--from") + 1]) if "--from" in sys.argv else 0.4
    ks = []
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, cls(name)))
    ks.sort()
    clusters, cur, end = [], [], None
    for k in ks:
        if cur and k[0] > end + 3_000_000:
            clusters.append(cur)
            cur = []
        cur.append(k)
        end = k[1] if end is None or not cur[:-1] else max(end, k[1])
    clusters.append(cur)
    best = max(clusters, key=lambda c: sum(1 for k in c if k[3] == "ladder"))
    lad = sorted(k for k in best if k[3] == "ladder")
    t0, t1 = lad[int(len(lad) * frac)][0], max(k[1] for k in lad)
    win = [(max(s, t0), min(e, t1), n, c) for s, e, n, c in ks if e > t0 and s < t1]
    wall = t1 - t0
    by = defaultdict(list)
    for s, e, n, c in win:
        by[c].append((s, e))
    u_all = union([(s, e) for s, e, _, _ in win])
    u_lad = union(by["ladder"])
    u_sig = union(by["ladder"] + by["prep"])
    out = {"window_ms": wall / 1e6, "ladders_in_window": len(by["ladder"]),
           "busy_any_frac": u_all / wall, "ladder_running_frac": u_lad / wall, "ladder_or_prep_frac": u_sig / wall,
           "ids_only_ms": (u_all - u_sig) / 1e6, "idle_ms": (wall - u_all) / 1e6,
           "sum_ms": {c: sum(e - s for s, e in v) / 1e6 for c, v in by.items()},
           "count": {c: len(v) for c, v in by.items()}}
    import json
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
