"""Partial Merkle trees on the CPU: the oracle (oracle/partial_merkle.py) against
the reference's PartialMerkleTreeTest.kt assertions and the committed golden
cases; the GPU kernel's stack-machine reading agrees with the recursive one."""
import hashlib
import json
import os
import random

import pytest

import partial_merkle as pm  # noqa: E402 (oracle/ on sys.path via conftest)

HERE = os.path.dirname(os.path.abspath(__file__))
H = lambda b: hashlib.sha256(b).digest()


def test_reference_build_failures():
    h = H(b"x")
    # PartialMerkleTreeTest.kt:84-93 check full tree
    left = ("node", h, ("node", h, ("leaf", h), ("leaf", h)), ("node", h, ("leaf", h), ("leaf", h)))
    right = ("node", h, ("leaf", h), ("leaf", h))
    with pytest.raises(pm.MerkleTreeException):
        pm.build(("node", h, left, right), [h])
    pm.build(right, [h, h])
    pm.build(("leaf", h), [h])
    hashed = [H(c.encode()) for c in "abcdef"]
    mt = pm.merkle_tree(hashed)
    # :162-165 duplicate leaves failure
    with pytest.raises(pm.MerkleTreeException):
        pm.build(mt, [hashed[3], hashed[5], hashed[3], hashed[5]])
    # :168-173 only duplicate leaves, less included
    aaa = [H(b"a")] * 3
    with pytest.raises(pm.MerkleTreeException):
        pm.build(pm.merkle_tree(aaa), aaa[:1])
    with pytest.raises(ValueError):
        pm.build(mt, [pm.ZERO])
    with pytest.raises(pm.MerkleTreeException):
        pm.merkle_tree([])


def test_golden_cases_consistent():
    cases = json.load(open(os.path.join(HERE, "golden", "pmt_vectors.json")))["cases"]
    names = {c["name"] for c in cases}
    for n in ("ref_left_branch", "ref_all_leaves", "ref_zero_leaves", "ref_too_many", "ref_too_little",
              "ref_duplicate", "ref_different", "ref_wrong_root"):
        assert n in names
    for c in cases:
        leaves = [bytes.fromhex(x) for x in c["leaves"]]
        toks = [(t, bytes.fromhex(h) if h else None) for t, h in c["tokens"]]
        if not leaves:
            assert c["status"] == 6
            continue
        v = pm.verify_tokens(toks, bytes.fromhex(c["root"]), [H(x) for x in leaves])
        assert (0 if v else 1) == c["status"], c["name"]


def test_stack_machine_matches_recursive_verify():
    rng = random.Random(5)
    for _ in range(200):
        n = rng.randrange(1, 20)
        hs = [H(bytes([i, rng.getrandbits(8)])) for i in range(n)]
        tree = pm.merkle_tree(hs)
        inc = [hs[j] for j in sorted(rng.sample(range(n), rng.randrange(0, n + 1)))]
        pt = pm.build(tree, inc)
        check = list(inc)
        if check and rng.random() < 0.3:
            check.pop()
        assert pm.verify_tokens(pm.tokens(pt), tree[1], check) == pm.verify(pt, tree[1], check)
    # malformed streams are not trees
    h = H(b"q")
    assert pm.verify_tokens([(pm.TOK_NODE, None)], h, []) is None
    assert pm.verify_tokens([(pm.TOK_LEAF, h), (pm.TOK_LEAF, h)], h, []) is None
