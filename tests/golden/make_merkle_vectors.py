#!/usr/bin/env python3
"""Generate tests/golden/merkle_vectors.json: WireTransaction ids from leaf preimages.

Expected roots come from hashlib + a literal restatement of MerkleTree.kt:27-66
(padWithZeros to 2^k with 32 zero bytes, SHA-256(left||right), 1 leaf -> leaf).
Includes the reference's own structural cases (PartialMerkleTreeTest.kt:22-25,
56-81) built on DERIVED leaf preimages: "corda\\0\\0\\1" + Kryo class id 7
(char) + big-endian UTF-16 code unit — the Kryo framing is an assumption
(Kryo 4.0.0 default registration, not pinned by the reference's tests); the
tree-shape rules they exercise are pinned.
"""
import hashlib
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
rng = random.Random(0xC0DA0004)


def merkle(leaf_hashes):
    if not leaf_hashes:
        return None
    n = 1
    while n < len(leaf_hashes):
        n *= 2
    lvl = list(leaf_hashes) + [bytes(32)] * (n - len(leaf_hashes))
    while len(lvl) > 1:
        lvl = [hashlib.sha256(lvl[i] + lvl[i + 1]).digest() for i in range(0, len(lvl), 2)]
    return lvl[0]


def tx_id(leaves):
    r = merkle([hashlib.sha256(x).digest() for x in leaves])
    return r.hex() if r is not None else None


txs = []
kryo_char = lambda c: b"corda\x00\x00\x01" + bytes([7]) + ord(c).to_bytes(2, "big")
for name, leaves in [("ref_abcdef", [kryo_char(c) for c in "abcdef"]), ("ref_one", [kryo_char("a")]),
                     ("ref_three", [kryo_char(c) for c in "abc"]), ("empty", [])]:
    txs.append({"name": name, "leaves": [x.hex() for x in leaves], "id": tx_id(leaves)})
# cash-issue shape: 5 components of [450,150,140,43,55] bytes
for i in range(8):
    leaves = [b"corda\x00\x00\x01" + bytes(rng.getrandbits(8) for _ in range(n - 8)) for n in (450, 150, 140, 43, 55)]
    txs.append({"name": "cash_issue_%d" % i, "leaves": [x.hex() for x in leaves], "id": tx_id(leaves)})
# SHA-256 padding boundaries and tree sizes 1..33
for n in list(range(1, 18)) + [31, 32, 33]:
    lens = [rng.choice([0, 1, 55, 56, 63, 64, 65, 119, 120, 128, 300]) for _ in range(n)]
    leaves = [bytes(rng.getrandbits(8) for _ in range(l)) for l in lens]
    txs.append({"name": "tree_%d" % n, "leaves": [x.hex() for x in leaves], "id": tx_id(leaves)})

with open(os.path.join(HERE, "merkle_vectors.json"), "w") as f:
    json.dump({"generator": "tests/golden/make_merkle_vectors.py", "txs": txs}, f, indent=0)
print(len(txs), "transactions")
