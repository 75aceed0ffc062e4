"""Subprocess body of tests/test_gpu_multidevice.py (not a test module itself).

Run with CORDAHIP_TEST_DEVICE_REPLICAS=k: every context gets k Device objects
on HIP device 0 (cordahip_init's test knob), so the in-process N-device code
(the cordahip_shard_range split, one host worker per device, shard
tails that are not multiples of 64, per-device statuses and verdict words
reassembled into the caller's arrays) runs on a one-GPU box. Every path's
results are compared with the goldens / the oracle, and with a one-device
context over the same inputs. Prints one JSON line; exit code 1 on a mismatch.
"""
import ctypes
import hashlib
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
ED = 4


def _load(name, key):
    with open(os.path.join(ROOT, "tests", "golden", name)) as f:
        return json.load(f)[key]


def _h(x):
    return bytes.fromhex(x)


def _verdict_words(st):
    n = len(st)
    w = np.zeros((n + 63) // 64, np.uint64)
    for i, s in enumerate(st):
        if s == 0:
            w[i // 64] |= np.uint64(1) << np.uint64(i % 64)
    return w


def main():
    import torch
    from conftest import load_oracle
    from corda_amd.engine import Engine

    k = int(os.environ["CORDAHIP_TEST_DEVICE_REPLICAS"])
    orc = load_oracle()
    out, bad = {"replicas": k}, {}
    eng = Engine(1)
    out["device_count"] = eng.device_count()
    if out["device_count"] != k:
        bad["device_count"] = out["device_count"]
    os.environ["CORDAHIP_TEST_DEVICE_REPLICAS"] = "1"  # read at init: the next context has one device
    one = Engine(1)
    rng = random.Random(1000 + k)

    # 1. generic CSR batch, mixed schemes, lengths that make every shard tail ragged
    ed = _load("ed25519_vectors.json", "vectors")
    ec = _load("ecdsa_vectors.json", "vectors")
    rows = [dict(v, scheme=ED) for v in ed] + ec
    rows = [rows[rng.randrange(len(rows))] for _ in range(3001 + 7 * k)]
    args = ([v["scheme"] for v in rows], [_h(v["pub"]) for v in rows], [_h(v["sig"]) for v in rows],
            [_h(v["msg"]) for v in rows])
    st, vd = eng.verify_batch(*args)
    want = [v["status"] for v in rows]
    miss = [i for i, (s, w) in enumerate(zip(st, want)) if int(s) != w]
    if miss:
        bad["generic"] = miss[:10]
    if not np.array_equal(vd[:(len(rows) + 63) // 64], _verdict_words(want)):
        bad["generic_verdict"] = True
    out["generic_lanes"] = len(rows)

    # 2. dense host Ed25519 rows (oracle-signed, every 7th corrupted)
    n = 1999 + 3 * k
    keys = bytearray()
    sigs = bytearray()
    msgs = bytearray()
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    for i in range(n):
        m = hashlib.sha256(b"md%d" % i).digest()
        orc.oracle_ed25519_sign(hashlib.sha256(b"sd%d" % (i % 97)).digest(), m, 32, pub, sig)
        s = bytearray(sig.raw)
        if i % 7 == 3:
            s[i % 64] ^= 0x10
        keys += pub.raw
        sigs += s
        msgs += m
    K, S, M = (np.frombuffer(bytes(x), np.uint8).copy() for x in (keys, sigs, msgs))
    want = np.zeros(n, np.uint8)
    orc.oracle_ed25519_verify_batch(n, K.ctypes.data, S.ctypes.data, M.ctypes.data, 32, want.ctypes.data, 4)
    st, vd = eng.ed25519_verify_host(K, S, M)
    if not np.array_equal(st, want):
        bad["dense_host"] = np.nonzero(st != want)[0][:10].tolist()
    if not np.array_equal(vd, _verdict_words(want.tolist())):
        bad["dense_host_verdict"] = True
    out["dense_lanes"] = n

    # 3. tx ids: the Merkle goldens, repeated so the tx shards split unevenly
    gold = _load("merkle_vectors.json", "txs")
    txs = [gold[i % len(gold)] for i in range(331)]
    ids, tst = eng.tx_ids([[_h(x) for x in t["leaves"]] for t in txs])
    miss = [i for i, t in enumerate(txs) if (t["id"] is None and tst[i] == 0) or
            (t["id"] is not None and ids[i].tobytes().hex() != t["id"])]
    if miss:
        bad["tx_ids"] = miss[:10]

    # 4. signed transactions: oracle-signed ids, corrupted signatures, empty lists
    ntx = 257
    txl = [[bytes(rng.getrandbits(8) for _ in range(n)) for n in (450, 150, 140, 43, 55)] for _ in range(ntx)]
    tids, _ = one.tx_ids(txl)
    sl = []
    for t in range(ntx):
        per = []
        for j in range(rng.choice([1, 2, 3])):
            orc.oracle_ed25519_sign(hashlib.sha256(b"signer%d" % j).digest(), tids[t].tobytes(), 32, pub, sig)
            s = sig.raw
            if t % 9 == 4 and j == len(per):
                s = s[:20] + bytes([s[20] ^ 1]) + s[21:]
            per.append((ED, pub.raw, s))
        sl.append(per if t % 50 != 7 else [])
    a = eng.signed_tx_verify(txl, sl)
    b = one.signed_tx_verify(txl, sl)
    for name, x, y in zip(("ids", "tx_status", "first_bad", "sig_status"), a, b):
        if not np.array_equal(x, y):
            bad["signed_tx_" + name] = True
    want_st = [7 if t % 50 == 7 else (1 if t % 9 == 4 else 0) for t in range(ntx)]
    if [int(x) for x in a[1]] != want_st:
        bad["signed_tx_expected"] = True

    # 4b. component-level signed transactions (cordahip_txcomp_submit): the cash-issue
    # corpus sharded over the devices, each with its own encoder state; three calls
    # (shapes built, then the templates-only chain) against a one-device context
    from corda_amd import _lib
    from corda_amd.corpus import cash_issue_items
    r2 = np.random.default_rng(77 + k)
    nc = 600 + 13 * k
    blob, items, _ = cash_issue_items(r2.integers(0, 256, (nc, 32), dtype=np.uint8),
                                      r2.integers(0, 256, (nc, 32), dtype=np.uint8), bytes(range(32)),
                                      r2.integers(1, 10**9, nc), r2.integers(-2**63, 2**63 - 1, nc))
    it = items.reshape(-1).copy()
    host_it = it.copy()
    host_it["data"] += np.uint64(blob.ctypes.data)
    hb, ho = _lib.kryo_encode_array(host_it)
    cl = [[hb[int(ho[5 * t + q]):int(ho[5 * t + q + 1])].tobytes() for q in range(5)] for t in range(nc)]
    cids, _ = one.tx_ids(cl)
    csl = []
    for t in range(nc):
        orc.oracle_ed25519_sign(hashlib.sha256(b"comp%d" % (t % 5)).digest(), cids[t].tobytes(), 32, pub, sig)
        s = sig.raw if t % 11 != 3 else sig.raw[:9] + bytes([sig.raw[9] ^ 2]) + sig.raw[10:]
        csl.append([(ED, pub.raw, s)])
    tio = np.arange(0, 5 * nc + 1, 5, dtype=np.uint64)
    cb = one.signed_txcomp_verify_arrays(blob, it, tio, csl)
    for call in range(3):
        ca = eng.signed_txcomp_verify_arrays(blob, it, tio, csl, pinned_out=call == 2)
        for name, x, y in zip(("ids", "tx_status", "first_bad", "sig_status"), ca, cb):
            if not np.array_equal(x, y):
                bad["txcomp_%d_%s" % (call, name)] = True
    if [int(x) for x in cb[1]] != [1 if t % 11 == 3 else 0 for t in range(nc)]:
        bad["txcomp_expected"] = True
    if not np.array_equal(cb[0], cids[:nc]):
        bad["txcomp_ids_vs_leaf_path"] = True

    # 5. filtered transactions: the PartialMerkleTree goldens
    cases = _load("pmt_vectors.json", "cases")
    cs = [cases[i % len(cases)] for i in range(199)]
    fst = eng.filtered_tx_verify([([_h(x) for x in c["leaves"]], [(t, _h(hh) if hh else None) for t, hh in c["tokens"]],
                                   _h(c["root"])) for c in cs])
    miss = [i for i, (s, c) in enumerate(zip(fst, cs)) if int(s) != c["status"]]
    if miss:
        bad["filtered"] = miss[:10]

    # 6. the C5 stream drain (both sections sharded)
    eds = [v for v in ed if len(_h(v["pub"])) == 32 and len(_h(v["sig"])) == 64 and len(_h(v["msg"])) == 32]
    ecs = [v for v in ec if len(_h(v["pub"])) in (33, 65) and len(_h(v["sig"])) <= 72 and len(_h(v["msg"])) == 32]
    E = [eds[rng.randrange(len(eds))] for _ in range(1301)]
    C = [ecs[rng.randrange(len(ecs))] for _ in range(411)]
    ck = np.zeros((len(C), 65), np.uint8)
    cs_ = np.zeros((len(C), 72), np.uint8)
    for i, v in enumerate(C):
        ck[i, :len(_h(v["pub"]))] = np.frombuffer(_h(v["pub"]), np.uint8)
        cs_[i, :len(_h(v["sig"]))] = np.frombuffer(_h(v["sig"]), np.uint8)
    pin = lambda x: torch.from_numpy(np.ascontiguousarray(x)).pin_memory()  # noqa: E731
    edsec = [pin(np.frombuffer(b"".join(_h(v[f]) for v in E), np.uint8).reshape(len(E), -1))
             for f in ("pub", "sig", "msg")] + [torch.zeros(len(E), dtype=torch.uint8).pin_memory()]
    ecsec = [pin(np.array([v["scheme"] for v in C], np.uint8)), pin(ck),
             pin(np.array([len(_h(v["pub"])) for v in C], np.uint8)), pin(cs_),
             pin(np.array([len(_h(v["sig"])) for v in C], np.uint8)),
             pin(np.frombuffer(b"".join(_h(v["msg"]) for v in C), np.uint8).reshape(len(C), 32)),
             torch.zeros(len(C), dtype=torch.uint8).pin_memory()]
    eng.stream_verify(edsec, ecsec)
    if edsec[3].numpy().tolist() != [v["status"] for v in E] or ecsec[6].numpy().tolist() != [v["status"] for v in C]:
        bad["stream"] = True

    one.close()
    eng.close()
    out["bad"] = bad
    print(json.dumps(out))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
