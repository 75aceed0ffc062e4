"""C5 streaming drain (cordahip_stream_verify) on the GPU: a mixed Ed25519 /
secp256k1 / P-256 queue in pinned host memory, streamed through the 3-stage
pipeline, must give exactly the golden statuses lane for lane — including
across chunk boundaries (small chunks forced with CORDAHIP_STREAM_CHUNK)."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sections(ed_vectors, ec_vectors, n_ed, n_ec, seed):
    rng = random.Random(seed)
    eds = [v for v in ed_vectors if len(v["pub"]) == 32 and len(v["sig"]) == 64 and len(v["msg"]) == 32]
    ecs = [v for v in ec_vectors if len(v["pub"]) <= 65 and len(v["sig"]) <= 72 and len(v["msg"]) == 32
           and len(v["pub"]) in (33, 65)]
    E = [eds[rng.randrange(len(eds))] for _ in range(n_ed)]
    C = [ecs[rng.randrange(len(ecs))] for _ in range(n_ec)]
    ek = np.frombuffer(b"".join(v["pub"] for v in E), np.uint8).reshape(n_ed, 32)
    es = np.frombuffer(b"".join(v["sig"] for v in E), np.uint8).reshape(n_ed, 64)
    em = np.frombuffer(b"".join(v["msg"] for v in E), np.uint8).reshape(n_ed, 32)
    sc = np.array([v["scheme"] for v in C], np.uint8)
    ck = np.zeros((n_ec, 65), np.uint8)
    cs = np.zeros((n_ec, 72), np.uint8)
    for i, v in enumerate(C):
        ck[i, :len(v["pub"])] = np.frombuffer(v["pub"], np.uint8)
        cs[i, :len(v["sig"])] = np.frombuffer(v["sig"], np.uint8)
    ckl = np.array([len(v["pub"]) for v in C], np.uint8)
    csl = np.array([len(v["sig"]) for v in C], np.uint8)
    cm = np.frombuffer(b"".join(v["msg"] for v in C), np.uint8).reshape(n_ec, 32)
    return (ek, es, em), (sc, ck, ckl, cs, csl, cm), [v["status"] for v in E], [v["status"] for v in C]


@pytest.mark.parametrize("chunk", [None, "256"])
def test_stream_mixed_golden(engine, ed_vectors, ec_vectors, chunk, monkeypatch):
    torch = pytest.importorskip("torch")
    if chunk:
        monkeypatch.setenv("CORDAHIP_STREAM_CHUNK", chunk)  # 256-lane chunks: ~13 chunks, all 3 stages reused
    (ek, es, em), (sc, ck, ckl, cs, csl, cm), want_ed, want_ec = _sections(ed_vectors, ec_vectors, 2600, 700, 3)
    pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
    ed = [pin(x) for x in (ek, es, em)] + [torch.zeros(len(want_ed), dtype=torch.uint8).pin_memory()]
    ec = [pin(x) for x in (sc, ck, ckl, cs, csl, cm)] + [torch.zeros(len(want_ec), dtype=torch.uint8).pin_memory()]
    engine.stream_verify(ed, ec)
    assert ed[3].numpy().tolist() == want_ed
    assert ec[6].numpy().tolist() == want_ec


def test_stream_one_section_empty(engine, ed_vectors, ec_vectors):
    (ek, es, em), (sc, ck, ckl, cs, csl, cm), want_ed, want_ec = _sections(ed_vectors, ec_vectors, 130, 0, 4)
    st = np.zeros(130, np.uint8)
    empty = np.zeros(0, np.uint8)
    engine.stream_verify((ek, es, em, st), (empty, ck, empty, cs, empty, cm, empty))
    assert st.tolist() == want_ed
