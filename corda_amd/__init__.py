"""corda_amd — MI355X-native batch verification engine for Corda's signature
and transaction-id hot path (include/cordahip.h).

The compute lives in libcordahip.so (hand-written gfx950 HIP kernels behind a
C-ABI). This package is the Python handle used by tests and bench.py.
"""
from ._lib import (BAD_KEY, BAD_SIG, EDDSA_ED25519_SHA512, ECDSA_SECP256K1_SHA256, ECDSA_SECP256R1_SHA256, EMPTY,
                   MALFORMED_SIG, OK, UNSUPPORTED, EngineError, EngineUnavailable)

__all__ = ["OK", "BAD_SIG", "MALFORMED_SIG", "BAD_KEY", "UNSUPPORTED", "EMPTY", "EDDSA_ED25519_SHA512",
           "ECDSA_SECP256K1_SHA256", "ECDSA_SECP256R1_SHA256", "EngineError", "EngineUnavailable"]
