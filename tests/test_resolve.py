"""Batched ResolveTransactionsFlow / SignedTransaction.verifySignatures (SURVEY.md
§8f rank 1, corda_amd/resolve.py).

CPU tests drive the host logic (topological order, exception precedence,
missing-signer / CompositeKey rules, stop-at-first-failure recording) through
OracleEngine, a test double whose signed_tx_verify is restated from the
oracle per signature; the GPU test runs the same scenarios through the real
C-ABI engine and requires identical outcomes.

Reference behaviour followed:
  ResolveTransactionsFlow.call / topologicalSort   ResolveTransactionsFlow.kt:40-66, :97-114
  SignedTransaction ctor / verifySignatures        SignedTransaction.kt:37-39, :70-85, :95-108
  CompositeKey.isFulfilledBy                       CompositeKey.kt:186-209
  topologicalSort test shape                       ResolveTransactionsFlowTest.kt (chain of
                                                   dependent issuances, resolved deepest-first)
"""
import ctypes
import hashlib

import numpy as np
import pytest

from corda_amd import resolve as R

ED, K1, R1 = 4, 2, 3


class OracleEngine:
    """signed_tx_verify with the C-ABI's contract (include/cordahip.h), computed by
    the oracle. Test infrastructure only."""

    def __init__(self, oracle):
        self.o = oracle

    def _sig_status(self, scheme, key, sig, msg):
        if scheme in (K1, R1):
            if len(key) not in (33, 65):
                return R.BAD_KEY
            return self.o.oracle_ecdsa_verify(scheme, key, len(key), sig, len(sig), msg, len(msg))
        if scheme != ED:
            return R.UNSUPPORTED
        if len(key) != 32:
            return R.BAD_KEY
        return self.o.oracle_ed25519_verify(key, 32, sig, len(sig), msg, len(msg))

    def signed_tx_verify(self, txs, sigs):
        n = len(txs)
        ids = np.zeros((n, 32), np.uint8)
        tx_st = np.zeros(n, np.uint8)
        first_bad = np.full(n, -1, np.int64)
        sig_st = []
        out = ctypes.create_string_buffer(32)
        for t, (tx, per) in enumerate(zip(txs, sigs)):
            blob = np.frombuffer(b"".join(tx) or b"\0", np.uint8).copy()
            off = np.zeros(len(tx) + 1, np.uint64)
            off[1:] = np.cumsum([len(x) for x in tx])
            rc = self.o.oracle_tx_id(blob.ctypes.data, off.ctypes.data, len(tx), out) if tx else -1
            if rc == 0:
                ids[t] = np.frombuffer(out.raw, np.uint8)
            sts = [self._sig_status(s, k, g, out.raw) if rc == 0 else R.OK for s, k, g in per]
            sig_st += sts
            if not per:
                tx_st[t] = R.TX_NO_SIGNATURES
            elif rc != 0:
                tx_st[t] = R.TX_NO_LEAVES
            else:
                bad = [i for i, s in enumerate(sts) if s != R.OK]
                if bad:
                    first_bad[t], tx_st[t] = bad[0], sts[bad[0]]
        return ids, tx_st, first_bad, np.asarray(sig_st, np.uint8)


def _ed_sign(oracle, seed, msg):
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_sign(seed, msg, len(msg), pub, sig)
    return pub.raw, sig.raw


def _ed_pub(oracle, seed):
    pub = ctypes.create_string_buffer(32)
    oracle.oracle_ed25519_keypair(seed, pub)
    return pub.raw


SEEDS = [hashlib.sha256(b"party%d" % i).digest() for i in range(4)]


def _txid(oracle, comps):
    return OracleEngine(oracle).signed_tx_verify([comps], [[(ED, b"k", b"s")]])[0][0].tobytes()


def _issue(oracle, tag, inputs=(), signers=(0,), must=None):
    """A synthetic transaction: components carry the tag and the input hashes
    (so the id commits to them, as WireTransaction's inputs group does), every
    signer signs the id."""
    comps = [b"output:" + tag, b"command:" + tag, b"notary"] + [b"input:" + h for h in inputs]
    tid = _txid(oracle, comps)
    sigs = []
    for s in signers:
        pub, sg = _ed_sign(oracle, SEEDS[s], tid)
        sigs.append((ED, pub, sg))
    must_sign = [_ed_pub(oracle, SEEDS[s]) for s in signers] if must is None else must
    return R.SignedTx(comps, sigs, must_sign, list(inputs)), tid


def _chain(oracle, n):
    """n transactions, each spending the previous one's output."""
    out, prev = [], ()
    for i in range(n):
        stx, tid = _issue(oracle, b"c%d" % i, inputs=prev)
        out.append(stx)
        prev = (tid,)
    return out


def test_topological_sort_chain_and_diamond(oracle):
    chain = _chain(oracle, 6)
    eng = OracleEngine(oracle)
    shuffled = [chain[i] for i in (3, 0, 5, 1, 4, 2)]
    res = R.resolve_transactions(eng, shuffled)
    assert res.error is None
    order = [shuffled[i] for i in res.order]
    assert order == chain  # dependencies before dependers
    assert res.recorded == res.order
    # diamond: a -> (b, c) -> d ; deterministic in input order like the LinkedHashSet walk
    a, ta = _issue(oracle, b"a")
    b, tb = _issue(oracle, b"b", inputs=(ta,))
    c, tc = _issue(oracle, b"c", inputs=(ta,))
    d, _ = _issue(oracle, b"d", inputs=(tb, tc))
    res = R.resolve_transactions(eng, [d, c, b, a])
    ordered = [[d, c, b, a][i] for i in res.order]
    assert ordered.index(a) < ordered.index(b) < ordered.index(d)
    assert ordered.index(a) < ordered.index(c) < ordered.index(d)
    assert R.resolve_transactions(eng, [d, c, b, a]).order == res.order


def test_long_chain_no_recursion_limit(oracle):
    chain = _chain(oracle, 1500)
    ids = [_txid(oracle, s.components) for s in chain]
    order = R.topological_sort(chain[::-1], ids[::-1])
    assert [chain[::-1][i] for i in order] == chain


def test_duplicate_transaction_fails_require(oracle):
    a, _ = _issue(oracle, b"a")
    res = R.resolve_transactions(OracleEngine(oracle), [a, a])
    assert isinstance(res.error, R.TransactionGraphException) and res.recorded == []


def test_first_failure_stops_recording(oracle):
    chain = _chain(oracle, 5)
    bad = bytearray(chain[2].sigs[0][2])
    bad[5] ^= 0x40
    chain[2].sigs[0] = (ED, chain[2].sigs[0][1], bytes(bad))
    res = R.resolve_transactions(OracleEngine(oracle), chain[::-1])
    rec = [chain[::-1][i] for i in res.recorded]
    assert rec == chain[:2]
    assert chain[::-1][res.failed] is chain[2]
    assert isinstance(res.error, R.SignatureException) and "Verification failed" in str(res.error)
    # the later transactions' signatures were verified in the same batch regardless
    assert res.outcomes[0].error is None


def test_exception_precedence(oracle):
    eng = OracleEngine(oracle)
    ok, tid = _issue(oracle, b"ok", signers=(0, 1))
    # bad signature beats missing signer
    s1, _ = _issue(oracle, b"s1", signers=(0,), must=[_ed_pub(oracle, SEEDS[0]), _ed_pub(oracle, SEEDS[2])])
    g = bytearray(s1.sigs[0][2]); g[40] ^= 1
    s1.sigs[0] = (ED, s1.sigs[0][1], bytes(g))
    # missing signer, partially allowed
    s2, t2 = _issue(oracle, b"s2", signers=(0,), must=[_ed_pub(oracle, SEEDS[i]) for i in (0, 1, 2)])
    # unsupported scheme at index 1 after a good one; malformed length; empty sig
    s3, _ = _issue(oracle, b"s3", signers=(0,))
    s3.sigs.append((9, s3.sigs[0][1], s3.sigs[0][2]))
    s4, _ = _issue(oracle, b"s4", signers=(0, 1))
    s4.sigs[1] = (ED, s4.sigs[1][1], s4.sigs[1][2][:63])
    s5, _ = _issue(oracle, b"s5", signers=(0,))
    s5.sigs[0] = (ED, s5.sigs[0][1], b"")
    s6, _ = _issue(oracle, b"s6", signers=(0,))
    s6.sigs[0] = (ED, s6.sigs[0][1][:31], s6.sigs[0][2])
    nosig = R.SignedTx([b"x"], [], [])
    noleaf = R.SignedTx([], [(ED, b"\0" * 32, b"\0" * 64)], [])
    outs = R.verify_signatures_batch(eng, [ok, s1, s2, s3, s4, s5, s6, nosig, noleaf],
                                     allowed_to_be_missing=[_ed_pub(oracle, SEEDS[2])])
    assert outs[0].error is None and outs[0].id == tid
    assert isinstance(outs[1].error, R.SignatureException) and outs[1].first_bad_sig == 0
    e2 = outs[2].error
    assert isinstance(e2, R.SignaturesMissingException) and e2.missing == [_ed_pub(oracle, SEEDS[1])]
    assert e2.id == t2
    assert isinstance(outs[3].error, R.IllegalArgumentException) and outs[3].first_bad_sig == 1
    assert isinstance(outs[4].error, R.SignatureException) and outs[4].first_bad_sig == 1
    assert isinstance(outs[5].error, R.IllegalArgumentException) and "empty" in str(outs[5].error)
    assert isinstance(outs[6].error, R.IllegalArgumentException) and "key" in str(outs[6].error)
    assert isinstance(outs[7].error, R.IllegalArgumentException) and outs[7].id is None
    assert isinstance(outs[8].error, R.MerkleTreeException) and outs[8].id is None
    # nothing missing once every key is allowed
    outs = R.verify_signatures_batch(eng, [s2], allowed_to_be_missing=[_ed_pub(oracle, SEEDS[i]) for i in (1, 2)])
    assert outs[0].error is None


def test_idless_transaction_fails_before_recording(oracle):
    chain = _chain(oracle, 3)
    noleaf = R.SignedTx([], [(ED, b"\0" * 32, b"\0" * 64)], [])
    res = R.resolve_transactions(OracleEngine(oracle), chain + [noleaf])
    assert res.recorded == [] and res.failed == 3 and isinstance(res.error, R.MerkleTreeException)


def test_missing_signers_are_a_set_with_descriptions(oracle):
    """getMissingSignatures is mustSign.filter{..}.toSet() (SignedTransaction.kt:106)
    and needed = missing - allowed (:79): duplicate mustSign keys appear once, in
    first-occurrence order; descriptions come from getMissingKeyDescriptions
    (:114-124): commands with a missing signer, then "notary"."""
    k = [_ed_pub(oracle, s) for s in SEEDS]
    eng = OracleEngine(oracle)
    stx, tid = _issue(oracle, b"dup", signers=(0,), must=[k[2], k[1], k[2], k[0], k[1], k[3]])
    stx.commands = [("Issue(owner=1)", [k[1]]), ("Move(owner=0)", [k[0]]), ("Exit(owner=2,3)", [k[2], k[3]])]
    stx.notary = k[3]
    e = R.verify_signatures_batch(eng, [stx])[0].error
    assert isinstance(e, R.SignaturesMissingException)
    assert e.missing == [k[2], k[1], k[3]]  # set semantics, first-occurrence order
    assert e.descriptions == ["Issue(owner=1)", "Exit(owner=2,3)", "notary"]
    assert e.id == tid
    e = R.verify_signatures_batch(eng, [stx], allowed_to_be_missing=[k[2], k[2]])[0].error
    assert e.missing == [k[1], k[3]] and e.descriptions == ["Issue(owner=1)", "Exit(owner=2,3)", "notary"]
    e = R.verify_signatures_batch(eng, [stx], allowed_to_be_missing=[k[2], k[3]])[0].error
    assert e.missing == [k[1]] and e.descriptions == ["Issue(owner=1)"]


def test_composite_key_fulfilment(oracle):
    k = [_ed_pub(oracle, s) for s in SEEDS]
    two_of_three = R.CompositeKey(2, ((k[0], 1), (k[1], 1), (k[2], 1)))
    weighted = R.CompositeKey(3, ((k[0], 2), (R.CompositeKey(1, ((k[1], 1), (k[2], 1))), 1)))
    assert two_of_three.is_fulfilled_by({k[0], k[2]})
    assert not two_of_three.is_fulfilled_by({k[1]})
    assert weighted.is_fulfilled_by({k[0], k[2]}) and not weighted.is_fulfilled_by({k[1], k[2]})
    eng = OracleEngine(oracle)
    stx, _ = _issue(oracle, b"ck", signers=(0, 2), must=[two_of_three])
    assert R.verify_signatures_batch(eng, [stx])[0].error is None
    stx, _ = _issue(oracle, b"ck2", signers=(1,), must=[two_of_three])
    e = R.verify_signatures_batch(eng, [stx])[0].error
    assert isinstance(e, R.SignaturesMissingException) and e.missing == [two_of_three]


def test_mixed_scheme_scenarios_on_oracle(oracle):
    _, extra = _scenarios(oracle)
    outs = R.verify_signatures_batch(OracleEngine(oracle), extra[-4:])
    assert [o.error is None for o in outs] == [True, True, False, True]
    assert outs[2].first_bad_sig == 1


def test_contract_hook_failure(oracle):
    chain = _chain(oracle, 4)

    def verify_contracts(i, stx):
        if stx is chain[1]:
            raise RuntimeError("TransactionVerificationException")

    res = R.resolve_transactions(OracleEngine(oracle), chain, verify_contracts)
    assert [chain[i] for i in res.recorded] == chain[:1] and isinstance(res.error, RuntimeError)


def _scenarios(oracle):
    rng = np.random.default_rng(7)
    chain = _chain(oracle, 40)
    for i in rng.choice(40, 6, replace=False):
        g = bytearray(chain[i].sigs[0][2]); g[int(rng.integers(64))] ^= 1 << int(rng.integers(8))
        chain[i].sigs[0] = (ED, chain[i].sigs[0][1], bytes(g))
    extra = []
    for j in range(30):
        stx, _ = _issue(oracle, b"m%d" % j, signers=tuple(range(1 + j % 3)),
                        must=[_ed_pub(oracle, SEEDS[i]) for i in range(1 + (j + 1) % 4)])
        extra.append(stx)
    import bc_ecdsa
    for j, scheme in enumerate((K1, R1, K1, R1)):
        # mixed-scheme signer sets: an Ed25519 signer plus an ECDSA one (compressed key for j odd)
        stx, tid = _issue(oracle, b"ec%d" % j, signers=(0,))
        d = 0x1234567 + 977 * j
        pub = bc_ecdsa.keypair(scheme, d)
        if j % 2:
            pub = bc_ecdsa.compress(pub)
        r, sv = bc_ecdsa.sign(scheme, d, tid, 0xabcdef + j)
        der = bc_ecdsa.der_encode(r, sv)
        if j == 2:
            der = der[:-1] + bytes([der[-1] ^ 1])  # BAD_SIG on the second signature
        stx.sigs.append((scheme, pub, der))
        stx.must_sign.append(pub)
        extra.append(stx)
    return chain, extra


@pytest.mark.gpu
def test_gpu_matches_oracle_engine(engine, oracle):
    chain, extra = _scenarios(oracle)
    ref = OracleEngine(oracle)
    for batch in (chain, extra, chain[::-1] + extra):
        a = R.verify_signatures_batch(engine, batch)
        b = R.verify_signatures_batch(ref, batch)
        assert [(o.id, type(o.error), str(o.error), o.first_bad_sig) for o in a] == \
               [(o.id, type(o.error), str(o.error), o.first_bad_sig) for o in b]
        ra, rb = R.resolve_transactions(engine, batch), R.resolve_transactions(ref, batch)
        assert (ra.order, ra.recorded, ra.failed, type(ra.error)) == (rb.order, rb.recorded, rb.failed, type(rb.error))
