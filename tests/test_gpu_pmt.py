"""K6 on the GPU: cordahip_filtered_tx_verify (FilteredTransaction.verify ->
PartialMerkleTree.verify) against the golden cases made by the oracle
(tests/golden/make_pmt_vectors.py), in one batch, plus malformed token streams."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    cases = json.load(open(os.path.join(HERE, "golden", "pmt_vectors.json")))["cases"]
    out = []
    for c in cases:
        leaves = [bytes.fromhex(x) for x in c["leaves"]]
        toks = [(t, bytes.fromhex(h) if h else None) for t, h in c["tokens"]]
        out.append(((leaves, toks, bytes.fromhex(c["root"])), c["status"], c["name"]))
    return out


def test_golden_filtered_txs(engine):
    cs = _cases()
    st = engine.filtered_tx_verify([c[0] for c in cs])
    bad = [(c[2], int(s), c[1]) for c, s in zip(cs, st) if s != c[1]]
    assert not bad, bad[:10]


def test_malformed_token_streams(engine):
    cs = _cases()
    (leaves, toks, root), _, _ = cs[0]
    h = bytes(32)
    batch = [(leaves, [(2, None)] + toks, root),        # Node on an empty stack
             (leaves, toks + [(1, h)], root),            # two roots left on the stack
             (leaves, [(7, h)], root),                   # unknown token
             (leaves, toks, root)]                       # control: the golden case itself
    st = engine.filtered_tx_verify(batch)
    assert [int(x) for x in st] == [8, 8, 8, cs[0][1]]
