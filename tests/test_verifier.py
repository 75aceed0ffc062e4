"""Verifier-module signature batches (corda_amd/verifier.py).

CPU tests drive the wire format, the node-side service (nonce handles, the
unknown-nonce error, success/failure counters, isValid/doVerify views) and the
verifier worker (many queued requests -> one engine submission, max_lanes
splitting, malformed requests, engine failures) through OracleBatchEngine, a
test double whose verify_batch computes each lane with the oracle. Expected
statuses are the committed golden vectors' (tests/golden/*_vectors.json). The
GPU test runs the same drain through the real C-ABI engine.

Reference behaviour followed:
  VerifierApi request/response, id + result-exception fields   VerifierApi.kt:11-58
  consumer loop: parse, verify, reply to JMSReplyTo, ack        Verifier.kt:58-75
  nonce handles, VerificationResultForUnknownTransaction        OutOfProcessTransactionVerifierService.kt:25-71
  VerifierType                                                  NodeConfiguration.kt:91-94
  per-item isValid / doVerify semantics                         Crypto.kt:472-483, 534-541
"""
import queue
import random

import numpy as np
import pytest

from corda_amd import verifier as V
from corda_amd.resolve import IllegalArgumentException, SignatureException

ED, K1, R1 = 4, 2, 3


class _Ticket:
    def __init__(self, status):
        self.status = status

    def wait(self):
        return self.status, None


class OracleBatchEngine:
    """Engine.verify_batch's contract (include/cordahip.h lane statuses), computed
    per lane by the oracle. Test infrastructure only."""

    def __init__(self, oracle, fail=False):
        self.o, self.fail, self.calls = oracle, fail, []

    def _status(self, scheme, key, sig, msg):
        if scheme in (K1, R1):
            if len(key) not in (33, 65):
                return 3
            return self.o.oracle_ecdsa_verify(scheme, key, len(key), sig, len(sig), msg, len(msg))
        if scheme != ED:
            return 4
        if len(key) != 32:
            return 3
        return self.o.oracle_ed25519_verify(key, 32, sig, len(sig), msg, len(msg))

    def verify_batch(self, schemes, keys, sigs, msgs, async_=False):
        self.calls.append(len(keys))
        if self.fail:
            raise RuntimeError("cordahip_sig_submit failed: -3")
        st = np.array([self._status(*x) for x in zip(schemes, keys, sigs, msgs)], np.uint8)
        return _Ticket(st) if async_ else (st, None)


def _golden_items(ed_vectors, ec_vectors, n, seed):
    rng = random.Random(seed)
    pool = [((ED, v["pub"], v["sig"], v["msg"]), v["status"]) for v in ed_vectors]
    pool += [((v["scheme"], v["pub"], v["sig"], v["msg"]), v["status"]) for v in ec_vectors]
    pool.append(((1, b"\x01" * 32, b"\x02" * 64, b"\x03" * 32), 4))  # RSA: UNSUPPORTED, stays on the JVM
    return [rng.choice(pool) for _ in range(n)]


class Wire:
    """In-process transport: node -> requests queue -> worker -> response handler."""

    def __init__(self):
        self.requests = queue.Queue()
        self.responses = {}

    def reply(self, address, msg):
        self.responses.setdefault(address, []).append(msg)


def _service(wire, addr="verifier.responses.node1"):
    return V.GpuSignatureVerifierService(wire.requests.put, addr)


def test_wire_round_trip():
    items = [(ED, b"k" * 32, b"s" * 64, b"m" * 32), (K1, b"\x04" + b"x" * 64, b"\x30" * 71, b""), (R1, b"", b"", b"z")]
    m = V.Message()
    V.SignatureVerificationRequest(12345, items, "verifier.responses.a").write_to_message(m)
    r = V.SignatureVerificationRequest.from_message(m)
    assert (r.verification_id, r.items, r.response_address) == (12345, items, "verifier.responses.a")
    m2 = V.Message()
    V.SignatureVerificationResponse(7, bytes([0, 1, 2]), None).write_to_message(m2)
    assert V.RESULT_EXCEPTION_FIELD_NAME not in m2.properties  # absent when ok (VerifierApi.kt:52-56)
    assert V.SignatureVerificationResponse.from_message(m2) == V.SignatureVerificationResponse(7, bytes([0, 1, 2]))
    m3 = V.Message()
    V.SignatureVerificationResponse(8, b"", "boom").write_to_message(m3)
    assert V.SignatureVerificationResponse.from_message(m3).exception == "boom"


@pytest.mark.parametrize("body", [b"", b"\x02\x00\x00\x00\x00", b"\x01\x01\x00\x00\x00\x04\x20\x00",
                                  b"\x01\x00\x00\x00\x00\xff"])
def test_malformed_bodies_raise(body):
    with pytest.raises(V.MalformedRequestException):
        V.SignatureVerificationRequest.from_message(V.Message({V.VERIFICATION_ID_FIELD_NAME: 1}, body, "a"))


def test_verifier_type_values():
    assert [t.value for t in V.VerifierType] == ["InMemory", "OutOfProcess", "Gpu"]


def test_drain_batches_requests_and_matches_goldens(oracle, ed_vectors, ec_vectors):
    wire = Wire()
    svc = _service(wire)
    eng = OracleBatchEngine(oracle)
    rng = random.Random(5)
    futs, want = [], []
    for r in range(40):
        g = _golden_items(ed_vectors, ec_vectors, rng.randint(0, 25), seed=r)
        futs.append(svc.verify_signatures([x for x, _ in g]))
        want.append(bytes(s for _, s in g))
    assert svc.in_flight() == 40
    worker = V.SignatureVerifier(eng, wire.requests, wire.reply, max_lanes=1 << 20)
    assert worker.drain() == 40
    assert eng.calls == [sum(len(w) for w in want)]  # every queued request in ONE engine submission
    for m in wire.responses["verifier.responses.node1"]:
        svc.on_response(m)
    assert svc.in_flight() == 0 and svc.success == 40 and svc.failure == 0
    for f, w in zip(futs, want):
        res = f.result(timeout=0)
        assert res.statuses == w
        for i, st in enumerate(w):
            if st == 0:
                assert res.is_valid(i) and res.do_verify(i)
            elif st == 1:  # BAD_SIG: isValid false, doVerify throws (Crypto.kt:481)
                assert res.is_valid(i) is False
                with pytest.raises(SignatureException, match="Signature Verification failed!"):
                    res.do_verify(i)
            else:
                exc = SignatureException if st == 2 else IllegalArgumentException
                with pytest.raises(exc):
                    res.is_valid(i)
                with pytest.raises(exc):
                    res.do_verify(i)


def test_max_lanes_splits_batches(oracle, ed_vectors, ec_vectors):
    wire = Wire()
    svc = _service(wire)
    eng = OracleBatchEngine(oracle)
    futs = [svc.verify_signatures([x for x, _ in _golden_items(ed_vectors, ec_vectors, 10, seed=s)])
            for s in range(9)]
    worker = V.SignatureVerifier(eng, wire.requests, wire.reply, max_lanes=25)
    assert worker.drain() == 9
    assert eng.calls == [30, 30, 30]  # requests are never split; a batch closes once >= max_lanes
    for m in wire.responses["verifier.responses.node1"]:
        svc.on_response(m)
    assert all(len(f.result(timeout=0).statuses) == 10 for f in futs)


def test_engine_failure_fails_each_request(oracle, ed_vectors, ec_vectors):
    wire = Wire()
    svc = _service(wire)
    futs = [svc.verify_signatures([x for x, _ in _golden_items(ed_vectors, ec_vectors, 3, seed=s)])
            for s in range(3)]
    V.SignatureVerifier(OracleBatchEngine(oracle, fail=True), wire.requests, wire.reply).drain()
    for m in wire.responses["verifier.responses.node1"]:
        svc.on_response(m)
    assert svc.failure == 3
    for f in futs:
        with pytest.raises(V.VerificationException, match="cordahip_sig_submit failed"):
            f.result(timeout=0)


def test_malformed_request_answered_and_batch_continues(oracle, ed_vectors, ec_vectors):
    wire = Wire()
    svc = _service(wire)
    good = svc.verify_signatures([x for x, _ in _golden_items(ed_vectors, ec_vectors, 4, seed=1)])
    bad_nonce = 99
    svc._handles[bad_nonce] = bad = V.Future()
    wire.requests.put(V.Message({V.VERIFICATION_ID_FIELD_NAME: bad_nonce}, b"\x01\xff", "verifier.responses.node1"))
    wire.requests.put(V.Message({}, b"junk", None))  # no id, no reply address: dropped
    V.SignatureVerifier(OracleBatchEngine(oracle), wire.requests, wire.reply).drain()
    for m in wire.responses["verifier.responses.node1"]:
        svc.on_response(m)
    assert len(good.result(timeout=0).statuses) == 4
    with pytest.raises(V.VerificationException, match="MalformedRequestException"):
        bad.result(timeout=0)


def test_unknown_nonce_raises():
    svc = _service(Wire())
    m = V.Message()
    V.SignatureVerificationResponse(424242, b"\x00").write_to_message(m)
    with pytest.raises(V.VerificationResultForUnknownTransaction, match="424242"):
        svc.on_response(m)


def test_empty_request_and_multiple_response_addresses(oracle, ed_vectors, ec_vectors):
    wire = Wire()
    a, b = _service(wire, "verifier.responses.a"), _service(wire, "verifier.responses.b")
    fa = a.verify_signatures([])
    fb = b.verify_signatures([x for x, _ in _golden_items(ed_vectors, ec_vectors, 5, seed=3)])
    V.SignatureVerifier(OracleBatchEngine(oracle), wire.requests, wire.reply).drain()
    for m in wire.responses["verifier.responses.a"]:
        a.on_response(m)
    for m in wire.responses["verifier.responses.b"]:
        b.on_response(m)
    assert fa.result(timeout=0).statuses == b"" and fa.result(timeout=0).all_valid()
    assert len(fb.result(timeout=0).statuses) == 5


def test_threaded_worker(oracle, ed_vectors, ec_vectors):
    wire = Wire()
    svc = _service(wire)
    worker = V.SignatureVerifier(OracleBatchEngine(oracle), wire.requests,
                                 lambda addr, m: svc.on_response(m))
    worker.start()
    try:
        g = [_golden_items(ed_vectors, ec_vectors, 6, seed=s) for s in range(20)]
        futs = [svc.verify_signatures([x for x, _ in gi]) for gi in g]
        for f, gi in zip(futs, g):
            assert f.result(timeout=30).statuses == bytes(s for _, s in gi)
    finally:
        worker.stop()


@pytest.mark.gpu
def test_gpu_drain_matches_goldens(engine, ed_vectors, ec_vectors):
    """The same drain through the real engine (cordahip_sig_submit / _wait)."""
    wire = Wire()
    svc = _service(wire)
    rng = random.Random(11)
    futs, want = [], []
    for r in range(64):
        g = _golden_items(ed_vectors, ec_vectors, rng.randint(0, 300), seed=100 + r)
        futs.append(svc.verify_signatures([x for x, _ in g]))
        want.append(bytes(s for _, s in g))
    worker = V.SignatureVerifier(engine, wire.requests, wire.reply, max_lanes=4096)
    assert worker.drain() == 64
    assert worker.batches >= 2  # several submissions in flight back to back
    for m in wire.responses["verifier.responses.node1"]:
        svc.on_response(m)
    for f, w in zip(futs, want):
        assert f.result(timeout=0).statuses == w
