"""ctypes binding of libcordahip.so (include/cordahip.h).

The product path has no CPU fallback: if the in-tree HIP library is missing
or fails to load, every entry point raises `EngineUnavailable` loudly.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libcordahip.so")

# lane statuses (CORDAHIP_STATUS_*)
OK, BAD_SIG, MALFORMED_SIG, BAD_KEY, UNSUPPORTED, EMPTY = 0, 1, 2, 3, 4, 5
STATUS_NAMES = {OK: "OK", BAD_SIG: "BAD_SIG", MALFORMED_SIG: "MALFORMED_SIG", BAD_KEY: "BAD_KEY",
                UNSUPPORTED: "UNSUPPORTED", EMPTY: "EMPTY"}

# schemes = Corda SignatureScheme.schemeNumberID (Crypto.kt:77-167)
RSA_SHA256, ECDSA_SECP256K1_SHA256, ECDSA_SECP256R1_SHA256, EDDSA_ED25519_SHA512, SPHINCS256_SHA256 = 1, 2, 3, 4, 5

SUCCESS = 0
ERR_TIMEOUT = -5
ERR_NOT_IMPLEMENTED = -7

# every symbol include/cordahip.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "cordahip_abi_version", "cordahip_strerror", "cordahip_init", "cordahip_shutdown",
    "cordahip_device_count", "cordahip_alloc_pinned", "cordahip_free_pinned", "cordahip_sig_submit",
    "cordahip_wait", "cordahip_poll", "cordahip_sig_verify", "cordahip_ed25519_verify_device",
    "cordahip_ed25519_verify_host", "cordahip_ed25519_sign_device", "cordahip_ecdsa_sign_device", "cordahip_last_kernel_ms",
    "cordahip_tx_ids", "cordahip_signed_tx_verify", "cordahip_signed_tx_verify_ed25519_device",
    "cordahip_ecdsa_verify_device", "cordahip_stream_verify", "cordahip_filtered_tx_verify",
    "cordahip_tx_submit", "cordahip_txid_submit", "cordahip_filtered_tx_submit", "cordahip_shard_range",
    "cordahip_kryo_encode", "cordahip_kryo_encode_device", "cordahip_signed_txcomp_verify", "cordahip_txcomp_submit",
    "cordahip_signed_txcomp_verify_ed25519_device", "cordahip_device_mem", "cordahip_trim",
]
ERR_BUFFER_TOO_SMALL = -8
# cordahip_kryo_item kinds (CORDAHIP_KRYO_*)
KRYO_KINDS = {"raw": 0, "char": 1, "short": 2, "int": 3, "long": 4, "byte": 5, "boolean": 6, "float": 7,
              "double": 8, "String": 9, "ed25519_key": 10, "public_key": 11, "kotlin_object": 12, "party": 13,
              "issue_command": 14, "cash_state": 15}
ABI_VERSION = 4
FLAG_IS_VALID = 1  # CORDAHIP_FLAG_IS_VALID: Crypto.isValid semantics (no emptiness checks)
TX_NO_LEAVES, TX_NO_SIGNATURES, TX_BAD_TREE, TX_BAD_COMPONENT = 6, 7, 8, 9


class EngineUnavailable(RuntimeError):
    pass


class EngineError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__("%s failed: %s (%d)" % (what, strerror(code), code))
        self.code = code


class SigBatch(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("scheme", ctypes.c_void_p),
        ("key", ctypes.c_void_p), ("key_off", ctypes.c_void_p),
        ("sig", ctypes.c_void_p), ("sig_off", ctypes.c_void_p),
        ("msg", ctypes.c_void_p), ("msg_off", ctypes.c_void_p),
        ("status", ctypes.c_void_p),
        ("verdict", ctypes.c_void_p),
        ("flags", ctypes.c_uint32),
        ("key_bytes", ctypes.c_uint64), ("sig_bytes", ctypes.c_uint64), ("msg_bytes", ctypes.c_uint64),  # ABI 4
    ]


class KryoItem(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_uint32), ("class_id", ctypes.c_uint32), ("value", ctypes.c_int64),
        ("data", ctypes.c_void_p), ("len", ctypes.c_uint64),
    ]


class TxidBatch(ctypes.Structure):
    _fields_ = [
        ("ntx", ctypes.c_uint64),
        ("leaf_bytes", ctypes.c_void_p), ("leaf_off", ctypes.c_void_p), ("tx_leaf_off", ctypes.c_void_p),
        ("txid", ctypes.c_void_p), ("tx_status", ctypes.c_void_p),
        ("nleaves", ctypes.c_uint64), ("leaf_bytes_len", ctypes.c_uint64),  # ABI 4
    ]


class SignedTxBatch(ctypes.Structure):
    _fields_ = [
        ("tx", TxidBatch),
        ("tx_sig_off", ctypes.c_void_p),
        ("scheme", ctypes.c_void_p),
        ("key", ctypes.c_void_p), ("key_off", ctypes.c_void_p),
        ("sig", ctypes.c_void_p), ("sig_off", ctypes.c_void_p),
        ("sig_status", ctypes.c_void_p), ("first_bad_sig", ctypes.c_void_p),
        ("nsig", ctypes.c_uint64), ("key_bytes", ctypes.c_uint64), ("sig_bytes", ctypes.c_uint64),  # ABI 4
    ]


class TxcompBatch(ctypes.Structure):
    _fields_ = [
        ("ntx", ctypes.c_uint64),
        ("items", ctypes.c_void_p), ("tx_item_off", ctypes.c_void_p),
        ("payload", ctypes.c_void_p), ("payload_len", ctypes.c_uint64),
        ("txid", ctypes.c_void_p), ("tx_status", ctypes.c_void_p),
        ("n_items", ctypes.c_uint64),  # ABI 4
    ]


class SignedTxcompBatch(ctypes.Structure):
    _fields_ = [
        ("tx", TxcompBatch),
        ("tx_sig_off", ctypes.c_void_p),
        ("scheme", ctypes.c_void_p),
        ("key", ctypes.c_void_p), ("key_off", ctypes.c_void_p),
        ("sig", ctypes.c_void_p), ("sig_off", ctypes.c_void_p),
        ("sig_status", ctypes.c_void_p), ("first_bad_sig", ctypes.c_void_p),
        ("nsig", ctypes.c_uint64), ("key_bytes", ctypes.c_uint64), ("sig_bytes", ctypes.c_uint64),  # ABI 4
    ]


class FilteredTxBatch(ctypes.Structure):
    _fields_ = [
        ("ntx", ctypes.c_uint64),
        ("leaf_bytes", ctypes.c_void_p), ("leaf_off", ctypes.c_void_p), ("tx_leaf_off", ctypes.c_void_p),
        ("tok", ctypes.c_void_p), ("tok_hash", ctypes.c_void_p), ("tx_tok_off", ctypes.c_void_p),
        ("root", ctypes.c_void_p), ("tx_status", ctypes.c_void_p),
        ("nleaves", ctypes.c_uint64), ("leaf_bytes_len", ctypes.c_uint64), ("ntok", ctypes.c_uint64),  # ABI 4
    ]


class StreamBatch(ctypes.Structure):
    _fields_ = [
        ("n_ed", ctypes.c_uint64),
        ("ed_keys", ctypes.c_void_p), ("ed_sigs", ctypes.c_void_p), ("ed_msgs", ctypes.c_void_p),
        ("ed_msg_len", ctypes.c_uint32), ("ed_status", ctypes.c_void_p),
        ("n_ec", ctypes.c_uint64),
        ("ec_scheme", ctypes.c_void_p), ("ec_keys", ctypes.c_void_p), ("ec_key_len", ctypes.c_void_p),
        ("ec_sigs", ctypes.c_void_p), ("ec_sig_len", ctypes.c_void_p), ("ec_msgs", ctypes.c_void_p),
        ("ec_msg_len", ctypes.c_uint32), ("ec_status", ctypes.c_void_p),
    ]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable("%s not built (run __graft_entry__.build())" % LIB_PATH)
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7
    # (same SONAME as /opt/rocm's). Loading torch first makes the dynamic linker
    # bind libcordahip.so to that already-loaded runtime, so torch tensors,
    # streams and RCCL share one HIP/HSA instance with our kernels.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    try:
        l = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise EngineUnavailable("cannot load %s: %s" % (LIB_PATH, e))
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    sig = {
        "cordahip_abi_version": (u32, []),
        "cordahip_strerror": (ctypes.c_char_p, [i32]),
        "cordahip_init": (i32, [u32, ctypes.POINTER(vp)]),
        "cordahip_shutdown": (None, [vp]),
        "cordahip_device_count": (i32, [vp]),
        "cordahip_alloc_pinned": (i32, [vp, ctypes.c_size_t, ctypes.POINTER(vp)]),
        "cordahip_free_pinned": (i32, [vp, vp]),
        "cordahip_sig_submit": (i32, [vp, ctypes.POINTER(SigBatch), ctypes.POINTER(u64)]),
        "cordahip_wait": (i32, [vp, u64, ctypes.c_int64]),
        "cordahip_poll": (i32, [vp, u64]),
        "cordahip_sig_verify": (i32, [vp, ctypes.POINTER(SigBatch)]),
        "cordahip_ed25519_verify_device": (i32, [vp, i32, vp, vp, vp, u32, u64, vp, vp, vp]),
        "cordahip_ed25519_verify_host": (i32, [vp, vp, vp, vp, u32, u64, vp, vp]),
        "cordahip_ed25519_sign_device": (i32, [vp, i32, vp, vp, u32, u64, vp, vp, vp]),
        "cordahip_last_kernel_ms": (ctypes.c_double, [vp, i32]),
        "cordahip_tx_ids": (i32, [vp, ctypes.POINTER(TxidBatch)]),
        "cordahip_signed_tx_verify": (i32, [vp, ctypes.POINTER(SignedTxBatch)]),
        "cordahip_signed_tx_verify_ed25519_device": (i32, [vp, i32, vp, vp, u64, vp, u64, vp, vp, vp, u64, vp, vp,
                                                           vp, vp, vp]),
        "cordahip_ecdsa_verify_device": (i32, [vp, i32, vp, vp, vp, vp, vp, vp, u32, u64, vp, vp, vp]),
        "cordahip_ecdsa_sign_device": (i32, [vp, i32, vp, vp, vp, u32, u64, vp, vp, vp, vp, vp]),
        "cordahip_stream_verify": (i32, [vp, ctypes.POINTER(StreamBatch)]),
        "cordahip_filtered_tx_verify": (i32, [vp, ctypes.POINTER(FilteredTxBatch)]),
        "cordahip_tx_submit": (i32, [vp, ctypes.POINTER(SignedTxBatch), ctypes.POINTER(u64)]),
        "cordahip_txid_submit": (i32, [vp, ctypes.POINTER(TxidBatch), ctypes.POINTER(u64)]),
        "cordahip_filtered_tx_submit": (i32, [vp, ctypes.POINTER(FilteredTxBatch), ctypes.POINTER(u64)]),
        "cordahip_shard_range": (None, [u64, u32, u32, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "cordahip_kryo_encode": (i32, [ctypes.POINTER(KryoItem), u64, vp, u64, vp]),
        "cordahip_kryo_encode_device": (i32, [vp, i32, vp, u64, u32, vp, u64, vp, vp, vp]),
        "cordahip_signed_txcomp_verify": (i32, [vp, ctypes.POINTER(SignedTxcompBatch)]),
        "cordahip_txcomp_submit": (i32, [vp, ctypes.POINTER(SignedTxcompBatch), ctypes.POINTER(u64)]),
        "cordahip_signed_txcomp_verify_ed25519_device": (i32, [vp, i32, vp, u64, u32, vp, u64, vp, u64, vp, vp, vp, u64,
                                                               vp, vp, vp, vp, vp]),
        "cordahip_device_mem": (i32, [vp, i32, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "cordahip_trim": (i32, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(l, name)
        f.restype = res
        f.argtypes = args
    _lib = l
    return l


def shard_range(n: int, nshards: int, shard: int, align: int = 64):
    """The library's in-process partition rule (cordahip_shard_range): [lo, hi)."""
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    lib().cordahip_shard_range(n, nshards, shard, align, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


# numpy image of cordahip_kryo_item (natural alignment: 32 bytes)
KRYO_ITEM_DTYPE = np.dtype([("kind", "<u4"), ("class_id", "<u4"), ("value", "<i8"), ("data", "<u8"), ("len", "<u8")])


def kryo_encode_array(items):
    """cordahip_kryo_encode over a contiguous KRYO_ITEM_DTYPE array whose data pointers
    the caller keeps alive; returns (leaf bytes uint8, off uint64[n + 1])."""
    n = len(items)
    items = np.ascontiguousarray(items)
    assert items.dtype == KRYO_ITEM_DTYPE and KRYO_ITEM_DTYPE.itemsize == ctypes.sizeof(KryoItem)
    off = np.zeros(n + 1, np.uint64)
    cap = int(items["len"].sum()) * 3 + 256 * n + 64
    out = np.empty(cap, np.uint8)
    rc = lib().cordahip_kryo_encode(ctypes.cast(items.ctypes.data, ctypes.POINTER(KryoItem)), n, out.ctypes.data, cap,
                                    off.ctypes.data)
    if rc == ERR_BUFFER_TOO_SMALL:
        cap = int(off[n])
        out = np.empty(cap, np.uint8)
        rc = lib().cordahip_kryo_encode(ctypes.cast(items.ctypes.data, ctypes.POINTER(KryoItem)), n, out.ctypes.data, cap,
                                    off.ctypes.data)
    check(rc, "cordahip_kryo_encode")
    return out[:int(off[n])], off


def _pack_party(p):
    """(X.500 name DER or b"" for an AnonymousParty, key bytes, key registration id)"""
    name, key, key_class = p
    return (int(key_class).to_bytes(2, "little") + len(key).to_bytes(2, "little") + bytes(key)
            + len(name).to_bytes(2, "little") + bytes(name))


def pack_cash_state(d):
    """The CORDAHIP_KRYO_CASH_STATE payload (include/cordahip.h) of a dict with keys
    issuer / owner / notary (parties as _pack_party takes them), reference (bytes),
    currency (ISO code), digits (its fraction digits), legal_ref (32 bytes),
    encumbrance (None or an int); the quantity goes in the item's value."""
    enc = d.get("encumbrance")
    code = d["currency"].encode("ascii")
    return (_pack_party(d["issuer"]) + bytes([len(d["reference"])]) + bytes(d["reference"]) + _pack_party(d["owner"])
            + _pack_party(d["notary"]) + bytes([len(code)]) + code + int(d["digits"]).to_bytes(1, "little", signed=True)
            + bytes(d["legal_ref"]) + bytes([0 if enc is None else 1])
            + (0 if enc is None else int(enc)).to_bytes(4, "little", signed=True))


def kryo_pack(items):
    """(kind, value, class_id) tuples -> (payload blob uint8, KRYO_ITEM_DTYPE[n] whose `data` are
    OFFSETS into the blob, bool[n]: the item has a payload). kind: a KRYO_KINDS key; value: bytes
    for raw / keys, str for String / kotlin_object (and char), int otherwise (float / double: their
    IEEE bits). Rebase `data` onto the blob's host or device address before encoding."""
    n = len(items)
    arr = np.zeros(n, KRYO_ITEM_DTYPE)
    has = np.zeros(n, bool)
    parts = []
    pos = 0
    for i, (kind, value, class_id) in enumerate(items):
        arr[i]["kind"], arr[i]["class_id"] = KRYO_KINDS[kind], class_id
        b = None
        if kind in ("String", "kotlin_object"):
            b = value.encode("utf-16-le")
            arr[i]["len"] = len(b) // 2
        elif kind in ("raw", "ed25519_key", "public_key"):
            b = bytes(value)
            arr[i]["len"] = len(b)
        elif kind == "party":  # value = (X.500 name DER, key bytes, key class id); class_id = X500Name's id
            name_der, key, key_class = value
            b = bytes(name_der) + bytes(key)
            arr[i]["len"] = len(b)
            arr[i]["value"] = key_class
        elif kind == "issue_command":  # value = (class name, nonce, [(key class id, key bytes)]); class_id = Arrays$ArrayList's
            cls, nonce, keys = value
            nm = cls.encode("ascii")
            b = bytes([len(nm)]) + nm + bytes([len(keys)]) + b"".join(
                int(kc).to_bytes(2, "little") + len(k).to_bytes(2, "little") + bytes(k) for kc, k in keys)
            arr[i]["len"] = len(b)
            arr[i]["value"] = nonce
        elif kind == "cash_state":  # value = a dict (pack_cash_state); class_id = X500Name's id
            b = pack_cash_state(value)
            arr[i]["len"] = len(b)
            arr[i]["value"] = int(value["quantity"])
        else:
            arr[i]["value"] = ord(value) if (kind == "char" and isinstance(value, str)) else int(value)
        if b is not None:
            has[i] = True
            arr[i]["data"] = pos
            parts.append(b)
            pos += len(b)
    blob = np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy()
    return blob, arr, has


def kryo_encode(items):
    """Leaf preimages of transaction components (cordahip_kryo_encode; host only, no
    device). items as kryo_pack takes them. Returns the list of leaves (bytes)."""
    n = len(items)
    blob, arr, has = kryo_pack(items)
    arr["data"] = np.where(has, arr["data"] + np.uint64(blob.ctypes.data), 0)
    if n == 0:
        return []
    out, off = kryo_encode_array(arr)
    del blob
    return [out[int(off[i]):int(off[i + 1])].tobytes() for i in range(n)]


def strerror(code: int) -> str:
    try:
        return lib().cordahip_strerror(code).decode()
    except EngineUnavailable:
        return "engine unavailable"


def check(code: int, what: str) -> None:
    if code != SUCCESS:
        raise EngineError(code, what)
