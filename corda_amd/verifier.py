"""Verifier-module signature batches.

Reference today: the out-of-process verifier (`verifier/.../Verifier.kt:58-75`)
consumes `VerifierApi.VerificationRequest`s (`node-api/.../VerifierApi.kt:17-58`)
one message at a time and runs `LedgerTransaction.verify()` -- contract logic
only, it never checks a signature. The node picks the backend with
`VerifierType` (`NodeConfiguration.kt:91-94`, `NodeMessagingClient.kt:117-120`)
and tracks in-flight requests by a random 63-bit nonce
(`OutOfProcessTransactionVerifierService.kt:25-71`).

This module adds the request type the north star asks for: a batch of
(scheme, encoded key, signature, clear data) tuples whose per-item results are
`Crypto.isValid` / `Crypto.doVerify` (`Crypto.kt:472-483,534-541`), a
`VerifierType.Gpu` value, the node-side service (futures keyed by nonce, the
unknown-nonce error, success/failure counters) and the verifier-side worker.
The worker is where the GPU pays: it drains every request waiting on the queue
into ONE engine submission (`cordahip_sig_submit`), assembles the next drain
while the GPU works on the current one, then splits the status bytes back per
request. Artemis is out of scope (SURVEY §8 / DESIGN §8): `Message` stands for
`ClientMessage` (long/bytes properties + body) and queues are `queue.Queue`s.
"""
from __future__ import annotations

import enum
import queue
import secrets
import struct
import threading
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .resolve import OK, _lane_exception

# VerifierApi.kt:11-15 (+ one queue for the new request type)
VERIFIER_USERNAME = "SystemUsers/Verifier"
VERIFICATION_REQUESTS_QUEUE_NAME = "verifier.requests"
SIGNATURE_REQUESTS_QUEUE_NAME = "verifier.signature-requests"
VERIFICATION_RESPONSES_QUEUE_NAME_PREFIX = "verifier.responses"
VERIFICATION_ID_FIELD_NAME = "id"
RESULT_EXCEPTION_FIELD_NAME = "result-exception"

_WIRE_VERSION = 1


class VerifierType(enum.Enum):
    """NodeConfiguration.kt:91-94 plus the GPU batch backend."""
    InMemory = "InMemory"
    OutOfProcess = "OutOfProcess"
    Gpu = "Gpu"


@dataclass
class Message:
    """Stand-in for Artemis `ClientMessage`: typed properties + body bytes."""
    properties: Dict[str, object] = field(default_factory=dict)
    body: bytes = b""
    reply_to: Optional[str] = None   # MessageUtil.setJMSReplyTo / getJMSReplyTo


Item = Tuple[int, bytes, bytes, bytes]  # (Corda schemeNumberID, key, signature, clear data)


class MalformedRequestException(Exception):
    """The request body does not parse (truncated / trailing bytes / wrong version)."""


def _pack_items(items: Sequence[Item]) -> bytes:
    out = [struct.pack("<BI", _WIRE_VERSION, len(items))]
    for scheme, key, sig, clear in items:
        out.append(struct.pack("<BHHI", scheme, len(key), len(sig), len(clear)))
        out += (key, sig, clear)
    return b"".join(out)


def _unpack_items(body: bytes) -> List[Item]:
    try:
        ver, n = struct.unpack_from("<BI", body, 0)
        if ver != _WIRE_VERSION:
            raise MalformedRequestException("wire version %d" % ver)
        pos, items = 5, []
        for _ in range(n):
            scheme, kl, sl, cl = struct.unpack_from("<BHHI", body, pos)
            pos += 9
            end = pos + kl + sl + cl
            if end > len(body):
                raise MalformedRequestException("truncated item")
            items.append((scheme, body[pos:pos + kl], body[pos + kl:pos + kl + sl], body[pos + kl + sl:end]))
            pos = end
    except struct.error as e:
        raise MalformedRequestException(str(e)) from None
    if pos != len(body):
        raise MalformedRequestException("trailing bytes")
    return items


@dataclass
class SignatureVerificationRequest:
    """The new VerifierApi request type: a batch of signature checks."""
    verification_id: int
    items: List[Item]
    response_address: str

    def write_to_message(self, message: Message) -> None:  # cf. VerificationRequest.writeToClientMessage
        message.properties[VERIFICATION_ID_FIELD_NAME] = self.verification_id
        message.body = _pack_items(self.items)
        message.reply_to = self.response_address

    @staticmethod
    def from_message(message: Message) -> "SignatureVerificationRequest":
        return SignatureVerificationRequest(int(message.properties[VERIFICATION_ID_FIELD_NAME]),
                                            _unpack_items(message.body), message.reply_to)


@dataclass
class SignatureVerificationResponse:
    """Per-item status bytes (include/cordahip.h lane statuses), or a request-level
    exception (malformed request / engine failure), as VerificationResponse carries
    `exception: Throwable?` (VerifierApi.kt:40-58)."""
    verification_id: int
    statuses: bytes
    exception: Optional[str] = None

    def write_to_message(self, message: Message) -> None:
        message.properties[VERIFICATION_ID_FIELD_NAME] = self.verification_id
        message.body = bytes(self.statuses)
        if self.exception is not None:
            message.properties[RESULT_EXCEPTION_FIELD_NAME] = self.exception.encode()

    @staticmethod
    def from_message(message: Message) -> "SignatureVerificationResponse":
        exc = message.properties.get(RESULT_EXCEPTION_FIELD_NAME)
        return SignatureVerificationResponse(int(message.properties[VERIFICATION_ID_FIELD_NAME]), bytes(message.body),
                                             exc.decode() if exc is not None else None)


class VerificationException(Exception):
    """A request-level failure reported by the verifier."""


@dataclass
class SignatureResults:
    """What the node's future resolves to: per-item isValid / doVerify views."""
    statuses: bytes

    def is_valid(self, i: int) -> bool:
        """Crypto.isValid: True/False for a decodable input, throws like the JCA engine otherwise
        (MALFORMED_SIG, BAD_KEY, UNSUPPORTED, EMPTY)."""
        st = self.statuses[i]
        if st in (OK, 1):
            return st == OK
        raise _lane_exception(st)

    def do_verify(self, i: int) -> bool:
        """Crypto.doVerify: True or throws (Crypto.kt:472-483)."""
        st = self.statuses[i]
        if st != OK:
            raise _lane_exception(st)
        return True

    def all_valid(self) -> bool:
        return all(s == OK for s in self.statuses)


class VerificationResultForUnknownTransaction(Exception):
    """OutOfProcessTransactionVerifierService.kt:40-41"""

    def __init__(self, nonce: int):
        super().__init__("Verification result arrived for unknown transaction nonce %d" % nonce)


def random63_bit_value() -> int:
    return secrets.randbits(63)


class GpuSignatureVerifierService:
    """Node side: OutOfProcessTransactionVerifierService (:18-72) for signature batches.

    `send_request(message)` is the transport (the Artemis producer in the node);
    `on_response(message)` is the response consumer's handler (`start`, :43-60)."""

    def __init__(self, send_request: Callable[[Message], None], response_address: str):
        self._send, self._addr = send_request, response_address
        self._handles: Dict[int, Future] = {}
        self._lock = threading.Lock()
        self.success = 0
        self.failure = 0

    def in_flight(self) -> int:  # the "VerificationsInFlight" gauge (:45)
        with self._lock:
            return len(self._handles)

    def verify_signatures(self, items: Sequence[Item]) -> Future:
        fut: Future = Future()
        with self._lock:
            nonce = random63_bit_value()
            while nonce in self._handles:
                nonce = random63_bit_value()
            self._handles[nonce] = fut
        msg = Message()
        SignatureVerificationRequest(nonce, list(items), self._addr).write_to_message(msg)
        self._send(msg)
        return fut

    def on_response(self, message: Message) -> None:
        resp = SignatureVerificationResponse.from_message(message)
        with self._lock:
            fut = self._handles.pop(resp.verification_id, None)
        if fut is None:
            raise VerificationResultForUnknownTransaction(resp.verification_id)
        if resp.exception is None:
            self.success += 1
            fut.set_result(SignatureResults(resp.statuses))
        else:
            self.failure += 1
            fut.set_exception(VerificationException(resp.exception))


class SignatureVerifier:
    """Verifier side (Verifier.kt:58-75) with batching: every request waiting on
    `requests` is folded into one engine submission of up to `max_lanes` items.

    `engine` needs `verify_batch(schemes, keys, sigs, msgs, async_=True)` returning
    a ticket with `wait() -> (status, verdict)` (corda_amd.engine.Engine).
    `reply(address, message)` is the reply producer (`replyProducer.send`)."""

    def __init__(self, engine, requests: "queue.Queue[Message]", reply: Callable[[str, Message], None],
                 max_lanes: int = 1 << 22):
        self.engine, self.requests, self.reply, self.max_lanes = engine, requests, reply, max_lanes
        self.batches = 0            # engine submissions made
        self.requests_served = 0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def _collect(self, block: bool, timeout: float):
        """Take queued request messages until max_lanes items are gathered."""
        reqs, bad, lanes = [], [], 0
        while lanes < self.max_lanes:
            try:
                msg = self.requests.get(block=block and not reqs and not bad, timeout=timeout)
            except queue.Empty:
                break
            try:
                req = SignatureVerificationRequest.from_message(msg)
            except (MalformedRequestException, KeyError, ValueError) as e:
                bad.append((msg, "MalformedRequestException: %s" % e))
                continue
            reqs.append(req)
            lanes += len(req.items)
        return reqs, bad

    def _submit(self, reqs):
        items = [it for r in reqs for it in r.items]
        if not items:
            return None
        return self.engine.verify_batch([it[0] for it in items], [it[1] for it in items],
                                        [it[2] for it in items], [it[3] for it in items], async_=True)

    def _answer(self, reqs, ticket, error: Optional[str] = None):
        status = None
        if ticket is not None and error is None:
            try:
                status, _ = ticket.wait()
            except Exception as e:  # noqa: BLE001 - a failed batch fails each of its requests
                error = "%s: %s" % (type(e).__name__, e)
        pos = 0
        for r in reqs:
            n = len(r.items)
            msg = Message()
            if error is None:
                sts = bytes(status[pos:pos + n]) if n else b""
                SignatureVerificationResponse(r.verification_id, sts).write_to_message(msg)
            else:
                SignatureVerificationResponse(r.verification_id, b"", error).write_to_message(msg)
            pos += n
            self.reply(r.response_address, msg)
            self.requests_served += 1

    def _reply_malformed(self, bad):
        for msg, err in bad:
            vid = msg.properties.get(VERIFICATION_ID_FIELD_NAME)
            if vid is None or msg.reply_to is None:
                continue  # nowhere to answer; Artemis would dead-letter it
            out = Message()
            SignatureVerificationResponse(int(vid), b"", err).write_to_message(out)
            self.reply(msg.reply_to, out)
            self.requests_served += 1

    def drain(self, block: bool = False, timeout: float = 0.05) -> int:
        """Serve everything queued now (double-buffered: drain k+1 is parsed and
        packed while drain k is on the GPU). Returns the number of requests served."""
        served0 = self.requests_served
        pending = None  # (reqs, ticket, error)
        while True:
            reqs, bad = self._collect(block and pending is None and self.requests_served == served0, timeout)
            self._reply_malformed(bad)
            nxt = None
            if reqs:
                try:
                    nxt = (reqs, self._submit(reqs), None)
                except Exception as e:  # noqa: BLE001
                    nxt = (reqs, None, "%s: %s" % (type(e).__name__, e))
                self.batches += 1
            if pending is not None:
                self._answer(*pending)
            pending = nxt
            if pending is None and not bad:
                return self.requests_served - served0

    # ---- thread lifecycle (Verifier.main's consumer loop) ----------------------
    def start(self) -> None:
        def loop():
            while not self._stop.is_set():
                self.drain(block=True, timeout=0.05)
        self._thread = threading.Thread(target=loop, name="signature-verifier", daemon=True)
        self._thread.start()

    def stop(self, timeout: float = 10.0) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout)
            self._thread = None
