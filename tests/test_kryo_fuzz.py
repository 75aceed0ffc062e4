"""Mutation fuzzing of the Kryo encoder core under AddressSanitizer + UBSan (host
only; the same core runs on the GPU, and its items come from the JVM):
tools/kryo_fuzz.cpp mutates valid seed items (payload bytes, lengths, kinds,
class ids, values, missing payloads) and checks, per item, the host entry point's
size pass, exact write and one-byte-short write, the batch status, and that every
templated item equals the direct encoder's leaf (kryo_template_check). Each
payload sits in its own heap block of exactly the bytes the item may read, so a
read past it is a sanitizer report. Seeds: the item families of test_kryo /
test_kryo_template plus the bench's cash-issue components."""
import os
import random
import shutil
import subprocess
import struct

import numpy as np
import pytest

from corda_amd import _lib
from test_kryo import C, L, O, _cash_state, _key_vectors, _random_items, x500_der
from test_kryo_template import _fixups, _rnd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _seed_items():
    rng = random.Random(21)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    items = _fixups(_random_items(rng))
    items += [("cash_state", _cash_state(rng, ref_keys, big=i % 4 == 0), 52) for i in range(24)]
    for i in range(12):
        name = x500_der([(O, "Party %d" % i), (L, "London"), (C, "GB")] + ([(O, "y" * 200)] if i % 5 == 0 else []))
        key, kc = (rng.choice(ref_keys), 45) if i % 2 else (_rnd(rng, 91), 77)
        items.append(("party", (name, key, kc), 60))
        keys = [(45, rng.choice(ref_keys)), (88, _rnd(rng, 88))][: 1 + i % 2]
        items.append(("issue_command", ("net.corda.contracts.asset.Cash$Commands$Issue", rng.randrange(-2**63, 2**63),
                                        keys), 31))
    items += [("String", s, 0) for s in ("", "a", "€" * 70, "x" * 200)]
    return items


def _write_seeds(path):
    items = _seed_items()
    blob, arr, has = _lib.kryo_pack(items)
    blob = np.ascontiguousarray(blob)
    out = bytearray()
    for it, h in zip(arr, has):
        kind, ln = int(it["kind"]), int(it["len"])
        nb = (2 * ln if kind in (9, 12) else ln) if h else 0
        d = int(it["data"])
        out += struct.pack("<IIqQQ", kind, int(it["class_id"]), int(it["value"]), ln, nb) + blob[d:d + nb].tobytes()
    # the bench's cash-issue components (raw payload offsets into their own blob)
    from corda_amd.corpus import cash_issue_items
    r = np.random.default_rng(9)
    cblob, citems, _ = cash_issue_items(r.integers(0, 256, (4, 32), dtype=np.uint8),
                                        r.integers(0, 256, (4, 32), dtype=np.uint8), bytes(range(32)),
                                        r.integers(1, 10**9, 4), r.integers(-2**63, 2**63 - 1, 4))
    cblob = np.ascontiguousarray(cblob)
    for it in citems.reshape(-1):
        kind, ln, d = int(it["kind"]), int(it["len"]), int(it["data"])
        nb = 2 * ln if kind in (9, 12) else ln
        out += struct.pack("<IIqQQ", kind, int(it["class_id"]), int(it["value"]), ln, nb) + cblob[d:d + nb].tobytes()
    with open(path, "wb") as f:
        f.write(out)
    return len(items) + citems.size


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ absent")
def test_kryo_encoder_fuzz_asan_ubsan(tmp_path):
    exe = str(tmp_path / "kryo_fuzz")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-o", exe,
                           os.path.join(ROOT, "tools", "kryo_fuzz.cpp"),
                           os.path.join(ROOT, "corda_amd", "csrc", "kryo.cpp"),
                           os.path.join(ROOT, "tools", "kryo_tmpl_check.cpp")])
    seeds = str(tmp_path / "seeds.bin")
    nseeds = _write_seeds(seeds)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe, seeds, "6000", "20261018"], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    import json
    st = json.loads(p.stdout.strip().splitlines()[-1])
    # the mutants reach both sides: valid leaves and template rebuilds as well as rejections
    assert nseeds > 100 and st["valid"] > st["items"] // 4 and st["templated"] > 1000, st


def test_truncated_composites_through_the_library():
    """Every truncation of a cash state, a party and an issue command through the
    product library (libcordahip.so's cordahip_kryo_encode): rejected or encoded,
    never a read outside the payload. The regression the fuzzer found: a cash
    state cut inside a party's X.500 name left the name pointer null with its
    length set, and the DER check read through it."""
    rng = random.Random(44)
    ref_keys = [bytes.fromhex(v["A"]) for v in _key_vectors()]
    items = [("cash_state", _cash_state(rng, ref_keys), 52), ("party", (x500_der([(O, "P"), (L, "L"), (C, "GB")]),
                                                                        ref_keys[0], 45), 50),
             ("issue_command", ("net.corda.contracts.asset.Cash$Commands$Issue", 5, [(45, ref_keys[1])]), 10)]
    blob, arr, _ = _lib.kryo_pack(items)
    blob = np.ascontiguousarray(blob)
    ok = 0
    for it in arr:
        full = int(it["len"])
        for k in range(full + 1):
            # each cut in its own exact-size buffer: a read past it lands outside the payload
            buf = np.frombuffer(blob[int(it["data"]):int(it["data"]) + k].tobytes(), np.uint8).copy()
            a = np.array([it])
            a["len"] = k
            a["data"] = buf.ctypes.data if k else 0
            try:
                _lib.kryo_encode_array(a)
                ok += 1
            except Exception:
                pass
    assert ok >= 3  # the full payloads themselves encode
