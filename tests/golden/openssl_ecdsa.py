"""ctypes bridge to OpenSSL 3 libcrypto ECDSA (EC_KEY / ECDSA_verify), an
INDEPENDENT implementation used to pin oracle/bc_ecdsa.py. ECDSA_verify
returns 1 (valid), 0 (bad signature), -1 (error, e.g. DER decode failure)."""
import ctypes
import ctypes.util
import hashlib

NID = {2: 714, 3: 415}  # secp256k1, prime256v1
_l = None


def lib():
    global _l
    if _l is None:
        l = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
        l.EC_KEY_new_by_curve_name.restype = ctypes.c_void_p
        l.EC_KEY_new_by_curve_name.argtypes = [ctypes.c_int]
        l.EC_KEY_oct2key.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        l.EC_KEY_free.argtypes = [ctypes.c_void_p]
        l.ECDSA_verify.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                   ctypes.c_void_p]
        l.ERR_clear_error.argtypes = []
        _l = l
    return _l


def verify(scheme: int, pub: bytes, sig: bytes, msg: bytes):
    """Returns 1 / 0 / -1 as ECDSA_verify, or None if OpenSSL rejects the key."""
    l = lib()
    k = l.EC_KEY_new_by_curve_name(NID[scheme])
    try:
        if l.EC_KEY_oct2key(k, pub, len(pub), None) != 1:
            l.ERR_clear_error()
            return None
        d = hashlib.sha256(msg).digest()
        r = l.ECDSA_verify(0, d, 32, sig, len(sig), k)
        l.ERR_clear_error()
        return r
    finally:
        l.EC_KEY_free(k)
