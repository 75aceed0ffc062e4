#!/usr/bin/env python3
"""Timeline of the last signed-tx call in a rocprofv3 kernel + memory-copy trace
(dev tool for the c4h pipeline): the call is the last cluster of kernels and
copies (more than 1 ms with nothing running between clusters) holding ladder
kernels and at least 20 H2D copies.
Prints the call's wall time, the busy time of each class (signature kernels,
id kernels -- encoder, SHA-256, Merkle --, H2D / D2H copies), how long the GPU
waited before its first ladder, and a 0.5 ms strip: L ladder/prep running,
i id kernels only, c copies only, . nothing.

usage: c4h_timeline.py kernel_trace.csv memory_copy_trace.csv"""
import csv
import sys

SIG = ("ed25519_ladder", "ed25519_prep", "gather_rows32")
IDK = ("kryo_", "sha256_leaves", "merkle_root", "comp_check", "rocprim", "store_to_host")


def load(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        name = (r.get("Kernel_Name") or r.get("Direction") or kind).replace("(anonymous namespace)", "").split("(")[0]
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, kind,
                    int(r.get("Bytes") or r.get("Size") or 0)))
    return out


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    ev = load(sys.argv[1], "K") + load(sys.argv[2], "M")
    ev.sort()
    # clusters separated by > 1 ms with nothing running; the call is the last one
    # with signature kernels and at least 20 H2D copies (the check's device path has none)
    clusters, start, end = [], 0, ev[0][1]
    for i in range(1, len(ev) + 1):
        if i == len(ev) or ev[i][0] > end + 1_000_000:
            clusters.append(ev[start:i])
            start = i
        if i < len(ev):
            end = max(end, ev[i][1])
    call = [c for c in clusters if sum(x[3] == "M" and "HOST_TO_DEVICE" in x[2].upper() for x in c) >= 20
            and any(x[3] == "K" and "ladder" in x[2] for x in c)][-1]
    t0, t1 = call[0][0], max(e[1] for e in call)
    cls = {"sig": [], "id": [], "h2d": [], "d2h": [], "other": []}
    h2d_bytes = 0
    for s, e, n, k, b in call:
        if k == "M":
            key = "d2h" if "DEVICE_TO_HOST" in n.upper() else "h2d"
            if key == "h2d":
                h2d_bytes += b
        elif any(x in n for x in SIG):
            key = "sig"
        elif any(x in n for x in IDK):
            key = "id"
        else:
            key = "other"
        cls[key].append((s, e))
    wall = t1 - t0
    print("call %.2f ms; busy: %s; H2D copies %d" % (
        wall / 1e6, ", ".join("%s %.2f ms" % (k, union(v) / 1e6) for k, v in cls.items() if v), len(cls["h2d"])))
    first_sig = min(s for s, e in cls["sig"]) if cls["sig"] else t1
    print("first signature kernel at %.2f ms; last signature kernel ends %.2f ms before the call ends"
          % ((first_sig - t0) / 1e6, (t1 - max(e for s, e in cls["sig"])) / 1e6 if cls["sig"] else 0))
    strip = []
    step = 500_000
    for x in range(t0, t1, step):
        def on(k):
            return any(s < x + step and e > x for s, e in cls[k])
        strip.append("L" if on("sig") else "i" if on("id") else "c" if on("h2d") or on("d2h") else ".")
    for i in range(0, len(strip), 80):
        print("%6.1f ms %s" % (i * step / 1e6, "".join(strip[i:i + 80])))
    # per-kernel totals inside the call
    per = {}
    for s, e, n, k, b in call:
        if k == "K":
            per.setdefault(n[-40:], [0, 0])
            per[n[-40:]][0] += 1
            per[n[-40:]][1] += e - s
    for n, (c, d) in sorted(per.items(), key=lambda x: -x[1][1])[:14]:
        print("  %-40s %5d %9.2f ms" % (n, c, d / 1e6))


if __name__ == "__main__":
    main()
