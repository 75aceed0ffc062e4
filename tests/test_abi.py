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
    from corda_amd import _lib
    assert lib.cordahip_abi_version() == _lib.ABI_VERSION == 4
    assert "#define CORDAHIP_ABI_VERSION 4u" in open(HEADER).read()
    assert lib.cordahip_strerror(0) == b"success"
    assert lib.cordahip_strerror(-7) == b"not implemented on the GPU path"
    assert lib.cordahip_strerror(12345) == b"unknown error"


def test_init_rejects_bad_args_without_device(lib):
    assert lib.cordahip_init(0, None) == -1
    # no context: every entry point fails with INVALID_ARG instead of crashing
    assert lib.cordahip_sig_verify(None, None) == -1
    assert lib.cordahip_wait(None, 1, 0) == -1
    assert lib.cordahip_poll(None, 1) == -1
    assert lib.cordahip_device_count(None) == 0
    for f in ("cordahip_sig_submit", "cordahip_tx_submit", "cordahip_txid_submit", "cordahip_filtered_tx_submit"):
        assert getattr(lib, f)(None, None, None) == -1, f


def test_status_codes_match_header():
    from corda_amd import _lib
    src = open(HEADER).read()
    vals = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"#define CORDAHIP_STATUS_(\w+) (\d+)", src))
    assert vals == {"OK": _lib.OK, "BAD_SIG": _lib.BAD_SIG, "MALFORMED_SIG": _lib.MALFORMED_SIG,
                    "BAD_KEY": _lib.BAD_KEY, "UNSUPPORTED": _lib.UNSUPPORTED, "EMPTY": _lib.EMPTY}
    import i2p_ed25519 as ed
    assert (ed.OK, ed.BAD_SIG, ed.MALFORMED_SIG, ed.BAD_KEY, ed.UNSUPPORTED, ed.EMPTY) == (0, 1, 2, 3, 4, 5)


def test_sig_batch_layout_matches_header():
    """cordahip_sig_batch as ctypes sees it == the C struct (flags appended in ABI 2)."""
    import ctypes
    from corda_amd import _lib
    assert [f[0] for f in _lib.SigBatch._fields_] == ["n", "scheme", "key", "key_off", "sig", "sig_off", "msg",
                                                      "msg_off", "status", "verdict", "flags", "key_bytes",
                                                      "sig_bytes", "msg_bytes"]
    # 10 8-byte fields + u32 flags padded to 8 + the three ABI-4 buffer lengths
    assert ctypes.sizeof(_lib.SigBatch) == 14 * 8
    src = open(HEADER).read()
    assert "#define CORDAHIP_FLAG_IS_VALID 1u" in src and _lib.FLAG_IS_VALID == 1


def test_shard_range_rule(lib):
    """The in-process partition (cordahip_shard_range, used by every multi-device
    host path: Ed25519, ECDSA, stream sections, tx batches): contiguous, covering,
    disjoint, 64-aligned starts so each device owns whole verdict words."""
    from corda_amd import _lib
    for n in (0, 1, 63, 64, 65, 1000, 4096, 100003, 1 << 24):
        for nd in (1, 2, 3, 7, 8):
            for align in (1, 64):
                prev = 0
                for i in range(nd):
                    lo, hi = _lib.shard_range(n, nd, i, align)
                    assert lo == prev and lo <= hi <= n, (n, nd, align, i, lo, hi)
                    if lo < n:
                        assert lo % align == 0
                    prev = hi
                assert prev == n
                # equal shares up to alignment: no device gets more than ceil(n/nd) rounded up to align
                per = -(-(-(-n // nd)) // align) * align
                assert all(_lib.shard_range(n, nd, i, align)[1] - _lib.shard_range(n, nd, i, align)[0] <= per
                           for i in range(nd))
    assert _lib.shard_range(100, 4, 9, 64) == (100, 100)  # out-of-range shard: empty
    assert _lib.shard_range(100, 0, 0, 64) == (100, 100)


def test_struct_layouts_match_header(tmp_path):
    """Every batch struct as ctypes lays it out == the C compiler's layout of
    include/cordahip.h (sizeof and every field's offsetof), so a binding built
    from the header and the Python mirror agree byte for byte."""
    import shutil
    if shutil.which("gcc") is None:
        pytest.skip("gcc absent")
    from corda_amd import _lib
    structs = {"cordahip_sig_batch": _lib.SigBatch, "cordahip_txid_batch": _lib.TxidBatch,
               "cordahip_signed_tx_batch": _lib.SignedTxBatch, "cordahip_txcomp_batch": _lib.TxcompBatch,
               "cordahip_signed_txcomp_batch": _lib.SignedTxcompBatch,
               "cordahip_filtered_tx_batch": _lib.FilteredTxBatch, "cordahip_stream_batch": _lib.StreamBatch,
               "cordahip_kryo_item": _lib.KryoItem}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "cordahip.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in cls._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f[0], cname, f[0]))
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = str(tmp_path / "layout")
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", exe, str(src)])
    got = dict(l.split() for l in subprocess.check_output([exe], text=True).splitlines())
    for cname, cls in structs.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f in cls._fields_:
            assert int(got["%s.%s" % (cname, f[0])]) == getattr(cls, f[0]).offset, (cname, f[0])
