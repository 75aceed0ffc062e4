"""Compose profiles/r05_pmc_kryo_traffic.json from two counter passes
(FETCH_SIZE, WRITE_SIZE) over tools/kryo_dev_bench.py (a sizes-only call, then
steady-state calls): the Kryo encoder kernels' L2-to-fabric bytes per
transaction in one steady-state call (each kernel's last dispatch; the scan's
dispatches averaged over the calls). FETCH_SIZE doubled per the gfx950 correction
(/opt/skills/guides/MI355X_MICROARCH.md), WRITE_SIZE as read, both in KB.

usage: pmc_kryo_traffic.py pass1.csv pass2.csv TXS CALLS > out.json (CALLS counts the sizes-only one) (dev tool)
"""
import csv
import json
import re
import sys
from collections import defaultdict


def kind(name):
    n = name.lower()
    m = re.search(r"kryo_\w+?_kernel", n)
    if m:
        return m.group(0)[:-len("_kernel")]
    return "scan" if "scan" in n or "lookback" in n else None


def per_dispatch(path, counter):
    d = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = kind(r["Kernel_Name"])
        if k and r["Counter_Name"] == counter:
            i = int(r["Dispatch_Id"])
            d[k][i] = d[k].get(i, 0.0) + float(r["Counter_Value"])
    return d


def main():
    p1, p2, txs, calls = sys.argv[1], sys.argv[2], float(sys.argv[3]), int(sys.argv[4])
    fetch, write = per_dispatch(p1, "FETCH_SIZE"), per_dispatch(p2, "WRITE_SIZE")
    out = {"command": "profiles/recipes/gpu_r5n.sh: rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, over "
                      "tools/kryo_dev_bench.py --txs %d --calls %d" % (txs, calls - 1),
           "txs": txs, "kernels": {}}
    tot_f = tot_w = 0.0
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, {}), write.get(k, {})
        if k == "scan":  # a few rocprim dispatches per call: their total over the calls
            fb, wb, used = sum(f.values()) / calls, sum(w.values()) / calls, [len(f), len(w)]
        else:  # the last dispatch: a steady-state call (templates cached, leaves written)
            fb, wb, used = f[max(f)] if f else 0.0, w[max(w)] if w else 0.0, [1, 1]
        fb, wb = fb * 1024 * 2 / txs, wb * 1024 / txs
        out["kernels"][k] = {"dispatches_used": used, "fetch_bytes_per_tx": fb, "write_bytes_per_tx": wb}
        # kryo_build runs on the first call only (new shapes): reported, not counted per call
        if k != "kryo_build":
            tot_f += fb
            tot_w += wb
    out["l2_fabric_bytes_per_tx"] = tot_f + tot_w
    out["fetch_bytes_per_tx"], out["write_bytes_per_tx"] = tot_f, tot_w
    out["note"] = ("L2-to-fabric bytes per steady-state encoder call (Infinity-Cache hits included, no MALL split; "
                   "kryo_build, which runs only when a shape is new, left out of the total): the devenc bench line "
                   "adds them to C4's HBM bytes as an upper bound for the encoder's share")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
