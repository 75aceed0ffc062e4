"""The drop-in boundary: libcordahip.so loads and exports exactly the C-ABI
include/cordahip.h declares (CPU-only checks; no compute without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cordahip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cordahip_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from corda_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.check_call(["make", "-s", "-j4", "-C", os.path.join(ROOT, "corda_amd", "csrc")])
    return _lib.lib()


def test_header_declares_the_binding_list():
    from corda_amd import _lib
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_every_declared_symbol_is_exported(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(ROOT, "corda_amd", "libcordahip.so")],
                                  text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    for f in declared_functions():
        assert getattr(lib, f) is not None


def test_abi_version_and_errors(lib):
    assert lib.cordahip_abi_version() == 1
    assert lib.cordahip_strerror(0) == b"success"
    assert lib.cordahip_strerror(-7) == b"not implemented on the GPU path"
    assert lib.cordahip_strerror(12345) == b"unknown error"


def test_init_rejects_bad_args_without_device(lib):
    assert lib.cordahip_init(0, None) == -1
    # no context: every entry point fails with INVALID_ARG instead of crashing
    assert lib.cordahip_sig_verify(None, None) == -1
    assert lib.cordahip_wait(None, 1, 0) == -1
    assert lib.cordahip_device_count(None) == 0


def test_status_codes_match_header():
    from corda_amd import _lib
    src = open(HEADER).read()
    vals = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"#define CORDAHIP_STATUS_(\w+) (\d+)", src))
    assert vals == {"OK": _lib.OK, "BAD_SIG": _lib.BAD_SIG, "MALFORMED_SIG": _lib.MALFORMED_SIG,
                    "BAD_KEY": _lib.BAD_KEY, "UNSUPPORTED": _lib.UNSUPPORTED, "EMPTY": _lib.EMPTY}
    import i2p_ed25519 as ed
    assert (ed.OK, ed.BAD_SIG, ed.MALFORMED_SIG, ed.BAD_KEY, ed.UNSUPPORTED, ed.EMPTY) == (0, 1, 2, 3, 4, 5)
