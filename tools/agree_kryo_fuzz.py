"""Device encoder against the host encoder on fuzzer mutants (dev tool, one MI355X):
tools/kryo_fuzz.cpp (built here with g++) mutates the seed items of
tests/test_kryo_fuzz.py and dumps every mutant with the host encoder's result;
each dump goes to the GPU in one cordahip_kryo_encode_device call (mixed kinds,
group 1, many fresh shapes per call: the shape table, template builds and the
direct writers under load), and every item must come back invalid exactly when
the host rejected it, otherwise with the host's leaf. One JSON line ->
profiles/r05_agreement_kryo_fuzz.json.

Then (--txcomp-rounds) the component-level call on mutants: consecutive mutants
grouped five to a transaction, each batch through cordahip_signed_txcomp_verify
three times (from the second call on, valid shapes hash straight from their
templates), against the ids the leaf-level path (cordahip_tx_ids) computes over
the host encoder's leaves, and BAD_COMPONENT exactly for the transactions with
an item the host rejects.

usage: python tools/agree_kryo_fuzz.py [--rounds R] [--calls K] [--txcomp-rounds R2]"""
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
    """(blob, items with blob offsets, has mask, host valid mask, host leaves, templated mask,
    shape hashes)"""
    from corda_amd import _lib
    raw = open(path, "rb").read()
    pos, rows, parts, valid, leaves, templ, shapes, fps = 0, [], [], [], [], [], [], []
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
        tb, h, fp = struct.unpack_from("<BQQ", raw, pos)
        pos += 17
        templ.append(bool(tb))
        shapes.append(h)
        fps.append(fp)
    blob = np.frombuffer(b"".join(parts) + b"\0" * 16, np.uint8).copy()
    arr = np.zeros(len(rows), _lib.KRYO_ITEM_DTYPE)
    for i, (kind, cls, value, off, ln, has) in enumerate(rows):
        arr[i]["kind"], arr[i]["class_id"], arr[i]["value"], arr[i]["data"], arr[i]["len"] = kind, cls, value, off, ln
    has = np.array([r[5] for r in rows], bool)
    return (blob, arr, has, np.array(valid), leaves, np.array(templ), np.array(shapes, np.uint64),
            np.array(fps, np.uint64))


def _last_misses(path):
    """the encoder-miss count of the library's last traced component call"""
    n = None
    with open(path) as f:
        for line in f:
            if "encoder misses" in line:
                n = int(line.split("call: ")[1].split()[0])
    return n


def find_misses(eng, blob, titems, n):
    """Bisect the transactions of the templated pass for the items that still go to the
    direct encoder once every shape is built (each probe: one call on a subset; stderr
    is redirected to a file so the library's trace lines can be read back)."""
    path = os.path.join(tempfile.mkdtemp(), "trace.log")
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
    saved = os.dup(2)
    os.dup2(fd, 2)

    def misses(lo, hi):
        its = titems[5 * lo:5 * hi]
        tio = np.arange(0, 5 * (hi - lo) + 1, 5, dtype=np.uint64)
        eng.signed_txcomp_verify_arrays(blob, its, tio, [[(4, bytes(32), bytes(64))]] * (hi - lo), pinned_out=True)
        return _last_misses(path)

    found = []
    try:
        stack = [(0, n)]
        while stack and len(found) < 4:
            lo, hi = stack.pop()
            if not misses(lo, hi):
                continue
            if hi - lo == 1:
                found.append(lo)
                continue
            mid = (lo + hi) // 2
            stack += [(mid, hi), (lo, mid)]
    finally:
        os.dup2(saved, 2)
        os.close(fd)
    res = []
    for t in found:
        for it in titems[5 * t:5 * t + 5]:
            d, ln, k = int(it["data"]), int(it["len"]), int(it["kind"])
            nb = 2 * ln if k in (9, 12) else ln
            res.append({"tx": int(t), "kind": k, "class_id": int(it["class_id"]), "value": int(it["value"]), "len": ln,
                        "payload": bytes(blob[d:d + min(nb, 512)]).hex()})
    return res


def txcomp_phase(eng, exe, seeds, tmp, rounds):
    from corda_amd import _lib
    dump = os.path.join(tmp, "dtx.bin")
    subprocess.check_call([exe, seeds, str(rounds), "4242", "--dump", dump], stdout=subprocess.DEVNULL)
    blob, arr, has, valid, leaves, templ, shapes, fps = read_dump(dump)
    # component payloads are offsets, never null: keep the mutants whose meaning does not
    # depend on a null pointer (a payload, no bytes, or a kind that reads none)
    keep = has | (arr["len"] == 0) | ((arr["kind"] >= 1) & (arr["kind"] <= 8))
    idx = np.nonzero(keep)[0]
    ntx = len(idx) // 5
    idx = idx[:ntx * 5]
    items = arr[idx]
    tvalid = valid[idx].reshape(ntx, 5).all(axis=1)
    good = [[leaves[i] for i in idx[5 * t:5 * t + 5]] for t in range(ntx) if tvalid[t]]
    want_ids, want_st = eng.tx_ids(good)
    out = {"txs": int(ntx), "valid_txs": int(tvalid.sum()), "calls": 3, "mismatches": 0,
           "mismatches_valid_only": 0}
    # (a) every transaction: invalid components make calls miss, so each call is redone
    # on the full chain; (b) the valid ones alone: from the second call on, every leaf
    # hashes from its template
    vitems = items.reshape(ntx, 5)[tvalid].reshape(-1)
    nv = int(tvalid.sum())
    for sel, its, n, key in ((tvalid, items, ntx, "mismatches"), (None, vitems, nv, "mismatches_valid_only")):
        # pass markers for the library's trace lines (CORDAHIP_TRACE=1: a templates-only miss)
        print("[agree] txcomp pass %s" % key, file=sys.stderr, flush=True)
        tio = np.arange(0, 5 * n + 1, 5, dtype=np.uint64)
        sigs = [[(4, bytes(32), bytes(64))]] * n
        for call in range(3):
            r = eng.signed_txcomp_verify_arrays(blob, its, tio, sigs, pinned_out=True)
            ids, st = r[0], r[1]
            if sel is None:
                bad = int((ids != want_ids).any(axis=1).sum()) + int((st == _lib.TX_BAD_COMPONENT).sum())
            else:
                bad = int((ids[sel] != want_ids).any(axis=1).sum())
                bad += int((st[~sel] != _lib.TX_BAD_COMPONENT).sum()) + int((st[sel] == _lib.TX_BAD_COMPONENT).sum())
            out[key] += bad
    # (c) valid transactions whose items all rebuild from templates, taken in order while
    # their distinct shapes fit the arena (512 templates; cleared past 448): from the
    # second call on the templates-only chain, every leaf hashed from its template
    plain = (has | (arr["len"] == 0))[idx].reshape(ntx, 5).all(axis=1)
    tt = templ[idx].reshape(ntx, 5).all(axis=1) & tvalid & plain
    sh = shapes[idx].reshape(ntx, 5)
    fh = fps[idx].reshape(ntx, 5)
    seen, pick = {}, []  # shape hash -> its one exact shape (a second shape under a hash goes direct)
    for t in np.nonzero(tt)[0]:
        pairs = [(int(x), int(f)) for x, f in zip(sh[t], fh[t]) if x]
        if any(seen.get(x, f) != f for x, f in pairs) or len(set(pairs)) != len({x for x, _ in pairs}):
            continue  # a second exact shape under a known hash, or two within this transaction
        new = {x for x, _ in pairs} - seen.keys()
        if len(seen) + len(new) > 400:
            continue
        seen.update(pairs)
        pick.append(t)
    pick = np.array(pick, dtype=np.int64)
    vpos = np.cumsum(tvalid) - 1  # tx t's row in want_ids when valid
    titems = items.reshape(ntx, 5)[pick].reshape(-1)
    n = len(pick)
    tio = np.arange(0, 5 * n + 1, 5, dtype=np.uint64)
    sigs = [[(4, bytes(32), bytes(64))]] * n
    out["templated_txs"], out["templated_shapes"], out["mismatches_templated"] = int(n), len(seen), 0
    print("[agree] txcomp pass mismatches_templated", file=sys.stderr, flush=True)
    for call in range(4):
        r = eng.signed_txcomp_verify_arrays(blob, titems, tio, sigs, pinned_out=True)
        ids, st = r[0], r[1]
        out["mismatches_templated"] += int((ids != want_ids[vpos[pick]]).any(axis=1).sum())
        out["mismatches_templated"] += int((st == _lib.TX_BAD_COMPONENT).sum())
    if os.environ.get("AGREE_FIND_MISS") and os.environ.get("CORDAHIP_TRACE"):
        out["miss_items"] = find_misses(eng, blob, titems, n)
    out["mismatches_total"] = out["mismatches"] + out["mismatches_valid_only"] + out["mismatches_templated"]
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20000)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--txcomp-rounds", type=int, default=20000)
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
            blob, arr, has, valid, leaves, _, _, _ = read_dump(dump)
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
        if a.txcomp_rounds:
            res["txcomp"] = txcomp_phase(eng, exe, seeds, tmp, a.txcomp_rounds)
            res["mismatches"] += res["txcomp"]["mismatches_total"]
    res["wall_s"] = time.time() - t0
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0 if res["mismatches"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
