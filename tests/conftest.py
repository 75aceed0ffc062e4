"""Shared fixtures. `-m "not gpu"` runs here (no GPU); `-m gpu` on an MI355X box.

Oracle access (oracle/) is test infrastructure: tests may load it as the
checker; the product under test is corda_amd/libcordahip.so.
"""
import ctypes
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

ORACLE_SO = os.path.join(ROOT, "oracle", "c", "liboracle.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def load_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle", "c")])
    lib = ctypes.CDLL(ORACLE_SO)
    cp, sz = ctypes.c_char_p, ctypes.c_size_t
    lib.oracle_ed25519_verify.argtypes = [cp, sz, cp, sz, cp, sz]
    lib.oracle_ed25519_verify_batch.argtypes = [sz, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, sz,
                                                ctypes.c_void_p, ctypes.c_int]
    lib.oracle_ed25519_sign.argtypes = [cp, cp, sz, ctypes.c_char_p, ctypes.c_char_p]
    lib.oracle_ed25519_keypair.argtypes = [cp, ctypes.c_char_p]
    lib.oracle_sha256.argtypes = [cp, sz, ctypes.c_char_p]
    lib.oracle_sha512.argtypes = [cp, sz, ctypes.c_char_p]
    lib.oracle_merkle_root.argtypes = [cp, sz, ctypes.c_char_p]
    lib.oracle_slide.argtypes = [cp, ctypes.c_char_p]
    lib.oracle_ecdsa_verify.argtypes = [ctypes.c_int, cp, sz, cp, sz, cp, sz]
    lib.oracle_ecdsa_is_valid.argtypes = [ctypes.c_int, cp, sz, cp, sz, cp, sz]
    lib.oracle_ed25519_is_valid.argtypes = [cp, sz, cp, sz, cp, sz]
    lib.oracle_ecdsa_verify_batch.argtypes = [sz] + [ctypes.c_void_p] * 8 + [ctypes.c_int]
    lib.oracle_tx_id.argtypes = [ctypes.c_void_p, ctypes.c_void_p, sz, ctypes.c_char_p]
    lib.oracle_tx_id_batch.argtypes = [sz] + [ctypes.c_void_p] * 5 + [ctypes.c_int]
    return lib


@pytest.fixture(scope="session")
def oracle():
    return load_oracle()


@pytest.fixture(scope="session")
def ed_vectors():
    with open(os.path.join(ROOT, "tests", "golden", "ed25519_vectors.json")) as f:
        vs = json.load(f)["vectors"]
    return [dict(v, pub=bytes.fromhex(v["pub"]), sig=bytes.fromhex(v["sig"]), msg=bytes.fromhex(v["msg"]))
            for v in vs]


@pytest.fixture(scope="session")
def ec_vectors():
    with open(os.path.join(ROOT, "tests", "golden", "ecdsa_vectors.json")) as f:
        vs = json.load(f)["vectors"]
    return [dict(v, pub=bytes.fromhex(v["pub"]), sig=bytes.fromhex(v["sig"]), msg=bytes.fromhex(v["msg"]))
            for v in vs]


@pytest.fixture(scope="session")
def cert_vectors():
    """ECDSA signatures made by the reference's own BouncyCastle path: the dev
    certificates it ships (tests/golden/make_cert_vectors.py), plus derived flips."""
    with open(os.path.join(ROOT, "tests", "golden", "cert_vectors.json")) as f:
        vs = json.load(f)["vectors"]
    return [dict(v, pub=bytes.fromhex(v["pub"]), sig=bytes.fromhex(v["sig"]), msg=bytes.fromhex(v["msg"]))
            for v in vs]


@pytest.fixture(scope="session")
def engine():
    from corda_amd.engine import Engine
    e = Engine(1)  # device 0
    yield e
    e.close()
