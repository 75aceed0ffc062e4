"""Mutation fuzzing of the C-ABI's CSR validation under AddressSanitizer + UBSan
(host only): tools/csr_fuzz.cpp builds generic signature batches and transaction
batches (txid + signature levels, components, filtered transactions) with every
array in a heap block of exactly its declared entries, mutates offsets and
declared lengths, and checks that the library's checks (csr_check.hpp, and
pack_rows.hpp's per-lane classify in the pipeline's chunk order) fail exactly
the batches the contract rejects -- and that a batch they accept is walked
without a read outside any caller buffer."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ absent")
def test_csr_validation_fuzz_asan_ubsan(tmp_path):
    exe = str(tmp_path / "csr_fuzz")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-o", exe,
                           os.path.join(ROOT, "tools", "csr_fuzz.cpp")])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe, "20000", "20261018"], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    st = json.loads(p.stdout.strip().splitlines()[-1])
    # both verdicts occur in every family, and valid generic batches were packed lane by lane
    for k in ("sig", "tx", "comp", "ftx"):
        assert 0 < st["%s_invalid" % k] < st["%s_batches" % k], st
    assert st["sig_lanes_packed"] > 100000, st
