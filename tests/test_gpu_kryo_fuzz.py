"""The device encoder against the host encoder on fuzzer mutants (the small form of
tools/agree_kryo_fuzz.py): tools/kryo_fuzz.cpp, built here with g++, mutates the
seed items of test_kryo_fuzz.py and dumps each mutant with the host encoder's
result; one cordahip_kryo_encode_device call over the dump (statuses and leaves
item by item), then the component-level call over the mutants grouped into
transactions -- every transaction, the valid ones alone, and the valid ones
whose shapes fit the template arena, three or four calls each (the last ones on the
templates-only chain) -- against the leaf-level path's ids over the host
encoder's leaves. Parity beyond the key bytes stays UNPINNED (no Kryo here), as
for the encoder itself."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.gpu


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ absent")
def test_fuzz_mutants_device_vs_host(engine, tmp_path):
    import agree_kryo_fuzz as A
    import test_kryo_fuzz as F
    exe = str(tmp_path / "kryo_fuzz")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "kryo_fuzz.cpp"),
                           os.path.join(ROOT, "corda_amd", "csrc", "kryo.cpp"),
                           os.path.join(ROOT, "tools", "kryo_tmpl_check.cpp")])
    seeds = str(tmp_path / "seeds.bin")
    F._write_seeds(seeds)
    dump = str(tmp_path / "d.bin")
    subprocess.check_call([exe, seeds, "1500", "77", "--dump", dump], stdout=subprocess.DEVNULL)
    blob, arr, has, valid, leaves, _, _, _ = A.read_dump(dump)
    out, off, status = engine.kryo_encode_packed_device(blob, arr, has)
    st, o, b = status.cpu().numpy(), off.cpu().numpy(), out.cpu().numpy()
    for i in range(len(arr)):
        if valid[i]:
            assert st[i] == 0 and b[int(o[i]):int(o[i + 1])].tobytes() == leaves[i], i
        else:
            assert st[i] == 1 and o[i + 1] == o[i], i
    assert 0 < valid.sum() < len(arr)
    res = A.txcomp_phase(engine, exe, seeds, str(tmp_path), 6000)
    assert res["mismatches_total"] == 0 and res["templated_txs"] > 1000, res
