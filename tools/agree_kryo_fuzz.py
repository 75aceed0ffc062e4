"""Device encoder against the host encoder on fuzzer mutants (dev tool, one MI355X):
tools/kryo_fuzz.cpp (built here with g++) mutates the seed items of
tests/test_kryo_fuzz.py and dumps every mutant with the host encoder's result;
each dump goes to the GPU in one cordahip_kryo_encode_device call (mixed kinds,
group 1, many fresh shapes per call: the shape table, template builds and the
direct writers under load), and every item must come back invalid exactly when
the host rejected it, otherwise with the host's leaf. One JSON line ->
profiles/r05_agreement_kryo_fuzz.json.

usage: python tools/agree_kryo_fuzz.py [--rounds R] [--calls K]"""
import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def read_dump(path):
    """(blob, items with blob offsets, has mask, host valid mask, host leaves)"""
    from corda_amd import _lib
    raw = open(path, "rb").read()
    pos, rows, parts, valid, leaves = 0, [], [], [], []
    bpos = 0
    while pos < len(raw):
        kind, cls, value, ln, nb, has = struct.unpack_from("<IIqQQB", raw, pos)
        pos += 33
        parts.append(raw[pos:pos + nb])
        rows.append((kind, cls, value, bpos, ln, has))
        bpos += nb
        pos += nb
        v, size = struct.unpack_from("<BQ", raw, pos)
        pos += 9
        valid.append(bool(v))
        leaves.append(raw[pos:pos + size])
        pos += size
    blob = np.frombuffer(b"".join(parts) + b"\0" * 16, np.uint8).copy()
    arr = np.zeros(len(rows), _lib.KRYO_ITEM_DTYPE)
    for i, (kind, cls, value, off, ln, has) in enumerate(rows):
        arr[i]["kind"], arr[i]["class_id"], arr[i]["value"], arr[i]["data"], arr[i]["len"] = kind, cls, value, off, ln
    has = np.array([r[5] for r in rows], bool)
    return blob, arr, has, np.array(valid), leaves


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20000)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_agreement_kryo_fuzz.json"))
    a = ap.parse_args()
    import test_kryo_fuzz as F

    from corda_amd.engine import Engine
    tmp = tempfile.mkdtemp()
    exe = os.path.join(tmp, "kryo_fuzz")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "kryo_fuzz.cpp"),
                           os.path.join(ROOT, "corda_amd", "csrc", "kryo.cpp"),
                           os.path.join(ROOT, "tools", "kryo_tmpl_check.cpp")])
    seeds = os.path.join(tmp, "seeds.bin")
    F._write_seeds(seeds)
    res = {"rounds_per_call": a.rounds, "calls": [], "items": 0, "host_valid": 0, "mismatches": 0}
    t0 = time.time()
    with Engine(1) as eng:
        for c in range(a.calls):
            dump = os.path.join(tmp, "d%d.bin" % c)
            subprocess.check_call([exe, seeds, str(a.rounds), str(1000 + c), "--dump", dump], stdout=subprocess.DEVNULL)
            blob, arr, has, valid, leaves = read_dump(dump)
            out, off, status = eng.kryo_encode_packed_device(blob, arr, has)
            st = status.cpu().numpy()
            o = off.cpu().numpy()
            b = out.cpu().numpy()
            bad = 0
            for i in range(len(arr)):
                if valid[i]:
                    bad += int(st[i] != 0 or b[int(o[i]):int(o[i + 1])].tobytes() != leaves[i])
                else:
                    bad += int(st[i] != 1 or o[i + 1] != o[i])
            res["calls"].append({"items": len(arr), "host_valid": int(valid.sum()), "mismatches": bad,
                                 "leaf_bytes": int(o[-1])})
            res["items"] += len(arr)
            res["host_valid"] += int(valid.sum())
            res["mismatches"] += bad
            os.remove(dump)
            print(json.dumps(res["calls"][-1]), flush=True)
    res["wall_s"] = time.time() - t0
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0 if res["mismatches"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
