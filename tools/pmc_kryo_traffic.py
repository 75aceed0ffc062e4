"""Compose profiles/r04_pmc_kryo_traffic.json from tools/gpu_pmc_kryo2.sh's two
counter passes (FETCH_SIZE, WRITE_SIZE) over `bench.py --workload c4
--device-encode --c4-txs 262144`: the Kryo encoder kernels' L2-to-fabric bytes
per transaction, per dispatch, taken from the dispatches that wrote every leaf
(the bench's sizing call runs the writer with no output buffer; that dispatch is
left out). FETCH_SIZE doubled per the gfx950 correction
(/opt/skills/guides/MI355X_MICROARCH.md), WRITE_SIZE as read, both in KB.

usage: pmc_kryo_traffic.py pass1.csv pass2.csv TXS > out.json (dev tool)
"""
import csv
import json
import sys
from collections import defaultdict

KINDS = {"kryo_size_kernel": "kryo_size", "kryo_write_kernel": "kryo_write", "scan": "scan"}  # hipcub/rocprim scan kernels


def kind(name):
    for k, v in KINDS.items():
        if k in name.lower():
            return v
    return None


def per_dispatch(path, counter):
    d = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = kind(r["Kernel_Name"])
        if k and r["Counter_Name"] == counter:
            d[k][r["Dispatch_Id"]] = d[k].get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return d


def main():
    p1, p2, txs = sys.argv[1], sys.argv[2], float(sys.argv[3])
    fetch, write = per_dispatch(p1, "FETCH_SIZE"), per_dispatch(p2, "WRITE_SIZE")
    out = {"command": "tools/gpu_pmc_kryo2.sh: rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, over bench.py "
                      "--workload c4 --device-encode --c4-txs 262144 --steps 1 --warmup 0",
           "txs": txs, "kernels": {}}
    tot_f = tot_w = 0.0
    for k in sorted(set(fetch) | set(write)):
        w = sorted(write.get(k, {}).values())
        f = sorted(fetch.get(k, {}).values())
        # the writer's sizing-call dispatch writes nothing: keep the full-write dispatches
        if k == "kryo_write":
            w = [x for x in w if x > 0.5 * w[-1]]
            f = f[-len(w):]
        fb = sum(f) / max(1, len(f)) * 1024 * 2 / txs
        wb = sum(w) / max(1, len(w)) * 1024 / txs
        out["kernels"][k] = {"dispatches_used": [len(f), len(w)], "fetch_bytes_per_tx": fb, "write_bytes_per_tx": wb}
        tot_f += fb
        tot_w += wb
    out["l2_fabric_bytes_per_tx"] = tot_f + tot_w
    out["fetch_bytes_per_tx"], out["write_bytes_per_tx"] = tot_f, tot_w
    out["note"] = ("L2-to-fabric bytes of the encoder (Infinity-Cache hits included, no MALL split): the devenc bench "
                   "line adds them to C4's HBM bytes as an upper bound for the encoder's share")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
