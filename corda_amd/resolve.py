"""Batched transaction resolution: the signature and transaction-id half of
ResolveTransactionsFlow / FinalityFlow / SignedTransaction.verifySignatures
 over ONE submission to the engine.

Reference call chain today (serial on the Node thread, one JCA call per
signature, every signature checked twice):

  ResolveTransactionsFlow.call                core/.../flows/ResolveTransactionsFlow.kt:97-131
    topologicalSort(downloaded)               :40-66
    for stx in newTxns:                       :106-114
      stx.toLedgerTransaction(serviceHub)     core/.../transactions/SignedTransaction.kt:155-159
        checkSignaturesAreValid()             :95-100   first invalid signature throws
        verifySignatures()                    :70-85    checkSignaturesAreValid() AGAIN, then
                                                        getMissingSignatures() :102-108 ->
                                                        SignaturesMissingException :54-55, :81
      transactionVerifierService.verify(ltx)  contract logic: out of scope (a hook here)
      recordTransactions(stx)

Here every transaction's id (K3/K4) and every signature (K1/K2) go to the GPU
in one cordahip_signed_tx_verify call (Engine.signed_tx_verify), each
signature is verified once, and the host then walks the topological order
raising exactly the exception the Kotlin loop would raise first. The JVM side
of this (the Kotlin a maintainer adds) is sketched in INTEGRATION.md §3.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple, Union

# per-lane statuses of include/cordahip.h
OK, BAD_SIG, MALFORMED_SIG, BAD_KEY, UNSUPPORTED, EMPTY = 0, 1, 2, 3, 4, 5
TX_NO_LEAVES, TX_NO_SIGNATURES = 6, 7


class SignatureException(Exception):
    """java.security.SignatureException"""


class SignaturesMissingException(SignatureException):
    """SignedTransaction.SignaturesMissingException (SignedTransaction.kt:54-55)."""

    def __init__(self, missing, descriptions, tx_id: bytes):
        super().__init__("Missing signatures for %s on transaction %s" % (descriptions, tx_id.hex()[:6].upper()))
        self.missing, self.descriptions, self.id = missing, descriptions, tx_id


class IllegalArgumentException(Exception):
    """java.lang.IllegalArgumentException (require failures, unsupported schemes, bad keys)."""


class MerkleTreeException(Exception):
    """MerkleTreeException: a transaction with no components (MerkleTree.kt:49-50)."""


class TransactionGraphException(IllegalArgumentException):
    """topologicalSort's require(result.size == transactions.size) (ResolveTransactionsFlow.kt:64)."""


@dataclass(frozen=True)
class CompositeKey:
    """CompositeKey (core/.../crypto/composite/CompositeKey.kt:35): a threshold tree whose
    leaves are encoded public keys (bytes) and whose inner nodes are CompositeKeys."""
    threshold: int
    children: Tuple[Tuple[Union[bytes, "CompositeKey"], int], ...]  # (node, weight)

    def is_fulfilled_by(self, keys) -> bool:
        # checkFulfilledBy, CompositeKey.kt:186-196
        total = sum(w for node, w in self.children if is_fulfilled_by(node, keys))
        return total >= self.threshold


def is_fulfilled_by(key, keys) -> bool:
    """PublicKey.isFulfilledBy(otherKeys), CryptoUtils.kt:79-82."""
    return key.is_fulfilled_by(keys) if isinstance(key, CompositeKey) else key in keys


@dataclass
class SignedTx:
    """What SignedTransaction holds for the path: the serialised available components
    (the Merkle leaves, MerkleTransaction.kt:51-62), the signatures in list order as
    DigitalSignature.WithKey (scheme, encoded key, signature bytes), tx.mustSign, and
    tx.inputs' transaction hashes (for topologicalSort)."""
    components: List[bytes]
    sigs: List[Tuple[int, bytes, bytes]]
    must_sign: List[Union[bytes, CompositeKey]] = field(default_factory=list)
    inputs: List[bytes] = field(default_factory=list)
    # for getMissingKeyDescriptions (SignedTransaction.kt:114-124): tx.commands as
    # (command.toString(), signers) and tx.notary?.owningKey
    commands: List[Tuple[str, List[Union[bytes, CompositeKey]]]] = field(default_factory=list)
    notary: Optional[Union[bytes, CompositeKey]] = None


def _lane_exception(status: int) -> Exception:
    """Per-lane status -> the exception Crypto.doVerify / the key decoder throws
    (INTEGRATION.md §1 table)."""
    if status == BAD_SIG:
        return SignatureException("Signature Verification failed!")  # Crypto.kt:481
    if status == MALFORMED_SIG:
        return SignatureException("error decoding signature bytes.")  # engine-level (JCA)
    if status == BAD_KEY:
        return IllegalArgumentException("invalid public key")  # key decode (Kryo.kt:389-392, Crypto.kt:353)
    if status == UNSUPPORTED:
        return IllegalArgumentException("Unsupported key/algorithm")  # Crypto.kt:474
    if status == EMPTY:
        return IllegalArgumentException("Signature data is empty!")  # Crypto.kt:475-476
    raise ValueError("status %d is not an exception" % status)


@dataclass
class Outcome:
    id: Optional[bytes]                 # WireTransaction.id (None when it cannot be computed)
    error: Optional[Exception]          # what verifySignatures() throws first, or None
    first_bad_sig: int = -1             # index in stx.sigs of the signature that threw


def missing_key_descriptions(stx: SignedTx, missing) -> List[str]:
    """getMissingKeyDescriptions (SignedTransaction.kt:114-124): every command with a
    missing signer (command.toString(), in command order), then "notary" if the
    notary's key is missing."""
    miss = set(missing)
    out = [desc for desc, signers in stx.commands if any(k in miss for k in signers)]
    if stx.notary is not None and stx.notary in miss:
        out.append("notary")
    return out


def verify_signatures_batch(engine, stxs: Sequence[SignedTx], allowed_to_be_missing=()) -> List[Outcome]:
    """SignedTransaction.verifySignatures(*allowed_to_be_missing) for every stx, one engine call.

    Exception precedence per transaction follows the Kotlin code: the
    constructor's require(sigs.isNotEmpty()) (:37-39), then tx.id (MerkleTree),
    then the signatures in list order (:95-100), then the missing signers
    (:76-82, minus allowed_to_be_missing)."""
    if not stxs:
        return []
    ids, tx_st, first_bad, _ = engine.signed_tx_verify([s.components for s in stxs], [s.sigs for s in stxs])
    allowed = set(allowed_to_be_missing)
    out = []
    for t, stx in enumerate(stxs):
        st = int(tx_st[t])
        if st == TX_NO_SIGNATURES:
            out.append(Outcome(None, IllegalArgumentException("Failed requirement.")))
            continue
        if st == TX_NO_LEAVES:
            out.append(Outcome(None, MerkleTreeException("Cannot calculate Merkle root on empty hash list.")))
            continue
        tid = bytes(ids[t])
        if st != OK:
            out.append(Outcome(tid, _lane_exception(st), int(first_bad[t])))
            continue
        sig_keys = {k for _, k, _ in stx.sigs}
        # getMissingSignatures (:102-108): mustSign.filter { !isFulfilledBy }.toSet() -- a
        # LinkedHashSet, so duplicates collapse and list order is kept; `missing - allowed`
        # (:79) keeps that order too
        missing = dict.fromkeys(k for k in stx.must_sign if not is_fulfilled_by(k, sig_keys))
        needed = [k for k in missing if k not in allowed]
        if needed:
            out.append(Outcome(tid, SignaturesMissingException(needed, missing_key_descriptions(stx, needed), tid)))
            continue
        out.append(Outcome(tid, None))
    return out


def topological_sort(stxs: Sequence[SignedTx], ids: Sequence[bytes]) -> List[int]:
    """ResolveTransactionsFlow.topologicalSort (:40-66) over indices: dependencies
    before dependers, deterministic in input order. Iterative DFS (the Kotlin
    recursion, unrolled) so long chains do not hit Python's recursion limit."""
    forward = {}  # txhash -> dependent tx indices, insertion-ordered (LinkedHashSet)
    for t, stx in enumerate(stxs):
        for h in stx.inputs:
            forward.setdefault(h, {})[t] = None
    visited, result = set(), []
    for root in range(len(stxs)):
        if ids[root] in visited:
            continue
        visited.add(ids[root])
        stack = [(root, iter(forward.get(ids[root], ())))]
        while stack:
            t, it = stack[-1]
            nxt = next(it, None)
            if nxt is None:
                stack.pop()
                result.append(t)
            elif ids[nxt] not in visited:
                visited.add(ids[nxt])
                stack.append((nxt, iter(forward.get(ids[nxt], ()))))
    result.reverse()
    if len(result) != len(stxs):
        raise TransactionGraphException("Failed requirement.")
    return result


@dataclass
class Resolution:
    order: List[int]                    # topological order (indices into the input)
    recorded: List[int]                 # transactions that passed, in the order they were recorded
    failed: Optional[int] = None        # index of the transaction whose check threw
    error: Optional[Exception] = None   # what ResolveTransactionsFlow.call would throw
    outcomes: List[Outcome] = field(default_factory=list)


def resolve_transactions(engine, stxs: Sequence[SignedTx],
                         verify_contracts: Optional[Callable[[int, SignedTx], None]] = None) -> Resolution:
    """The verification loop of ResolveTransactionsFlow.call (:98-114) over already
    downloaded transactions: ids and signatures of all of them in one engine call,
    then, in topological order, the first exception stops the loop (earlier
    transactions stay recorded, as in the flow). verify_contracts(i, stx) stands
    in for transactionVerifierService.verify (contract logic is out of scope)."""
    outcomes = verify_signatures_batch(engine, stxs)
    res = Resolution(order=[], recorded=[], outcomes=outcomes)
    # A transaction without an id cannot even be sorted: the SignedTransaction
    # constructor (:37-39) or stx.id inside topologicalSort's visit() (:53-54)
    # throws before anything is recorded -- the first such one in input order.
    for t, o in enumerate(outcomes):
        if o.id is None:
            res.failed, res.error = t, o.error
            return res
    ids = [o.id for o in outcomes]
    try:
        res.order = topological_sort(stxs, ids)
    except TransactionGraphException as e:
        res.error = e
        return res
    for t in res.order:
        err = outcomes[t].error
        if err is None and verify_contracts is not None:
            try:
                verify_contracts(t, stxs[t])
            except Exception as e:  # noqa: BLE001 - the flow propagates whatever the verifier throws
                err = e
        if err is not None:
            res.failed, res.error = t, err
            return res
        res.recorded.append(t)
    return res
