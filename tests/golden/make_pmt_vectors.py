#!/usr/bin/env python3
"""Generate tests/golden/pmt_vectors.json: FilteredTransaction.verify cases.

Each case: the filtered leaves' preimages (their SHA-256 = availableComponentHashes),
the PartialMerkleTree as a post-order token stream, the claimed root, and the
expected outcome of FilteredTransaction.verify (MerkleTransaction.kt:134-140):
0 = true, 1 = false, 6 = MerkleTreeException (no included leaves).

The first block restates the reference's own PartialMerkleTreeTest.kt cases
(lines 142-213) on leaves 'a'..'f' serialised as DERIVED Kryo bytes
("corda\\0\\0\\1" + class id 7 + UTF-16BE char: an assumption about Kryo 4.0.0
framing, not pinned by the reference; the tree rules those tests exercise are).
Expected values come from oracle/partial_merkle.py (restating
PartialMerkleTree.kt:68-158) and match the reference tests' assertions.
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import partial_merkle as pm  # noqa: E402

H = lambda b: hashlib.sha256(b).digest()
kryo_char = lambda c: b"corda\x00\x00\x01" + bytes([7]) + ord(c).to_bytes(2, "big")


def case(name, leaves, tree, root, expect, note=""):
    toks = pm.tokens(tree)
    return {"name": name, "leaves": [x.hex() for x in leaves],
            "tokens": [[t, h.hex() if h else None] for t, h in toks], "root": root.hex(), "status": expect,
            "note": note}


def expected(leaves, tree, root):
    try:
        return 0 if pm.filtered_tx_verify(root, [H(x) for x in leaves], tree) else 1
    except pm.MerkleTreeException:
        return 6


cases = []
pre = [kryo_char(c) for c in "abcdef"]
hashed = [H(x) for x in pre]
mt = pm.merkle_tree(hashed)
# PartialMerkleTreeTest.kt:143-147 only left nodes branch -> true
t = pm.build(mt, [hashed[3], hashed[5]])
cases.append(case("ref_left_branch", [pre[3], pre[5]], t, mt[1], 0))
# :156-159 include all leaves -> true
t = pm.build(mt, hashed)
cases.append(case("ref_all_leaves", pre, t, mt[1], 0))
# :150-153 include zero leaves: PMT.verify(emptyList) is true, FilteredTransaction.verify throws (no leaves)
t = pm.build(mt, [])
cases.append(case("ref_zero_leaves", [], t, mt[1], 6, "MerkleTransaction.kt:137-138"))
# :176-181 too many leaves -> false
t = pm.build(mt, [hashed[3], hashed[5]])
cases.append(case("ref_too_many", [pre[3], pre[5], pre[0]], t, mt[1], 1))
# :184-189 too little leaves -> false
t = pm.build(mt, [hashed[3], hashed[5], hashed[0]])
cases.append(case("ref_too_little", [pre[3], pre[5]], t, mt[1], 1))
# :192-198 duplicate leaves (5-leaf tree) -> false
mt5 = pm.merkle_tree(hashed[:5])
t = pm.build(mt5, [hashed[3], hashed[4]])
cases.append(case("ref_duplicate", [pre[3], pre[4], pre[4]], t, mt5[1], 1))
# :201-205 different leaves -> false
t = pm.build(mt, [hashed[3], hashed[5]])
cases.append(case("ref_different", [pre[2], pre[4]], t, mt[1], 1))
# :208-213 wrong root -> false
cases.append(case("ref_wrong_root", [pre[3], pre[5]], t, pm.hash_concat(hashed[3], hashed[5]), 1))
# one-leaf tree (MerkleTree.kt:51-52: root = leaf)
t1 = pm.build(pm.merkle_tree([hashed[0]]), [hashed[0]])
cases.append(case("one_leaf", [pre[0]], t1, hashed[0], 0))
# same multiset, different order (reference compares groupBy maps) -> true
t = pm.build(mt, [hashed[1], hashed[4]])
cases.append(case("order_insensitive", [pre[4], pre[1]], t, mt[1], 0))

rng = random.Random(0xC0DA0F17)
for i in range(120):
    n = rng.randrange(1, 34)
    pre_i = [bytes([j]) + bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 42, 54, 63, 139]))) for j in range(n)]
    hs = [H(x) for x in pre_i]
    tree = pm.merkle_tree(hs)
    k = rng.randrange(1, n + 1)
    sel = sorted(rng.sample(range(n), k))
    pt = pm.build(tree, [hs[j] for j in sel])
    leaves = [pre_i[j] for j in sel]
    root = tree[1]
    kind = i % 6
    if kind == 1:  # corrupt one filtered leaf byte
        j = rng.randrange(len(leaves))
        b = bytearray(leaves[j])
        b[rng.randrange(len(b))] ^= 1
        leaves[j] = bytes(b)
    elif kind == 2:  # claimed root off by one bit
        r = bytearray(root)
        r[rng.randrange(32)] ^= 1 << rng.randrange(8)
        root = bytes(r)
    elif kind == 3:  # shuffled leaf order: still true
        rng.shuffle(leaves)
    elif kind == 4 and len(leaves) > 1:  # a leaf dropped
        leaves = leaves[:-1]
    cases.append(case("random_%d" % i, leaves, pt, root, expected(leaves, pt, root)))

for c in cases:
    leaves = [bytes.fromhex(x) for x in c["leaves"]]
    toks = [(t, bytes.fromhex(h) if h else None) for t, h in c["tokens"]]
    if not leaves:
        assert c["status"] == 6
        continue
    v = pm.verify_tokens(toks, bytes.fromhex(c["root"]), [H(x) for x in leaves])
    assert (0 if v else 1) == c["status"], c["name"]

with open(os.path.join(HERE, "pmt_vectors.json"), "w") as f:
    json.dump({"generator": "tests/golden/make_pmt_vectors.py", "cases": cases}, f, indent=0)
print(len(cases), "cases")
