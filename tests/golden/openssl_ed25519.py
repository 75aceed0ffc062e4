"""ctypes bridge to OpenSSL 3 libcrypto Ed25519 (an INDEPENDENT implementation).

Test infrastructure: used to pin `oracle/` on the valid path (SURVEY.md §8c:
OpenSSL 3.0.2 is present in the image, here and on the GPU box). OpenSSL
implements RFC 8032, which rejects S >= L; i2p 0.2.0 (the reference's engine)
does not, so OpenSSL is not an oracle for the malleability cases.
"""
import ctypes
import ctypes.util

_EVP_PKEY_ED25519 = 1087

_lib = None


def lib():
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        l = ctypes.CDLL(name)
        l.EVP_PKEY_new_raw_public_key.restype = ctypes.c_void_p
        l.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        l.EVP_PKEY_new_raw_private_key.restype = ctypes.c_void_p
        l.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        l.EVP_PKEY_get_raw_public_key.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)]
        l.EVP_PKEY_free.argtypes = [ctypes.c_void_p]
        l.EVP_MD_CTX_new.restype = ctypes.c_void_p
        l.EVP_MD_CTX_free.argtypes = [ctypes.c_void_p]
        l.EVP_DigestVerifyInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        l.EVP_DigestVerify.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        l.EVP_DigestSignInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        l.EVP_DigestSign.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_size_t]
        _lib = l
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except OSError:
        return False


def keypair(seed: bytes):
    l = lib()
    k = l.EVP_PKEY_new_raw_private_key(_EVP_PKEY_ED25519, None, seed, 32)
    assert k
    out = ctypes.create_string_buffer(32)
    n = ctypes.c_size_t(32)
    assert l.EVP_PKEY_get_raw_public_key(k, out, ctypes.byref(n)) == 1
    l.EVP_PKEY_free(k)
    return out.raw


def sign(seed: bytes, msg: bytes) -> bytes:
    l = lib()
    k = l.EVP_PKEY_new_raw_private_key(_EVP_PKEY_ED25519, None, seed, 32)
    ctx = l.EVP_MD_CTX_new()
    assert l.EVP_DigestSignInit(ctx, None, None, None, k) == 1
    out = ctypes.create_string_buffer(64)
    n = ctypes.c_size_t(64)
    assert l.EVP_DigestSign(ctx, out, ctypes.byref(n), msg, len(msg)) == 1
    l.EVP_MD_CTX_free(ctx)
    l.EVP_PKEY_free(k)
    return out.raw


def verify(pub: bytes, sig: bytes, msg: bytes) -> bool:
    l = lib()
    k = l.EVP_PKEY_new_raw_public_key(_EVP_PKEY_ED25519, None, pub, len(pub))
    if not k:
        return False
    ctx = l.EVP_MD_CTX_new()
    ok = l.EVP_DigestVerifyInit(ctx, None, None, None, k) == 1 and \
        l.EVP_DigestVerify(ctx, sig, len(sig), msg, len(msg)) == 1
    l.EVP_MD_CTX_free(ctx)
    l.EVP_PKEY_free(k)
    return ok
