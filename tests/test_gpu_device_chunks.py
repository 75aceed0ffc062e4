"""The device-resident signed-tx calls' Ed25519 section in alternating chunks
(cordahip.cpp ed_verify_device_chunks: the remainder first, then full chunks on
the caller's stream / slot 0 and the device's second Ed25519 stream / slot 1,
forked and joined by events). The default chunk (98,304 signatures) is larger
than a test corpus, so a fresh process forces 192-signature chunks (the size is
read once): ~2,000 signatures in 11 chunks through
cordahip_signed_tx_verify_ed25519_device and
cordahip_signed_txcomp_verify_ed25519_device, every id against the host tx-id
path, every signature status, tx status and first_bad_sig against the
construction (SignedTransaction.kt:95-100: the first failing signature in list
order), and both calls against each other."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import hashlib, json, sys
import numpy as np
import torch
sys.path.insert(0, %(root)r)
sys.path.insert(0, %(root)r + "/tests")
from conftest import load_oracle
from corda_amd import _lib
from corda_amd.corpus import cash_issue_items
from corda_amd.engine import Engine
import ctypes
orc = load_oracle()
eng = Engine(1)
dev = torch.device("cuda:0")
rng = np.random.default_rng(77)
ntx = 1000
blob, items, _ = cash_issue_items(rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                  rng.integers(0, 256, (ntx, 32), dtype=np.uint8), bytes(range(32)),
                                  rng.integers(1, 10**9, ntx), rng.integers(-2**63, 2**63 - 1, ntx))
it = items.reshape(-1).copy()
host_it = it.copy()
host_it["data"] += np.uint64(blob.ctypes.data)
hb, ho = _lib.kryo_encode_array(host_it)
leaves = [[hb[int(ho[5 * t + j]):int(ho[5 * t + j + 1])].tobytes() for j in range(5)] for t in range(ntx)]
ids, _ = eng.tx_ids(leaves)
nsig = rng.integers(1, 4, ntx)
keys, sigs, want_st, want_fb = [], [], [], []
for t in range(ntx):
    bad = -1
    for q in range(int(nsig[t])):
        pub, sg = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        m = ids[t].tobytes()
        orc.oracle_ed25519_sign(hashlib.sha256(b"dc%%d-%%d" %% (t, q)).digest(), m, 32, pub, sg)
        s = sg.raw
        if (t * 3 + q) %% 17 == 5:
            s = s[:9] + bytes([s[9] ^ 16]) + s[10:]
            bad = q if bad < 0 else bad
        keys.append(pub.raw)
        sigs.append(s)
    want_fb.append(bad)
    want_st.append(1 if bad >= 0 else 0)
tso = np.zeros(ntx + 1, np.int64)
tso[1:] = np.cumsum(nsig)
K = torch.tensor(np.frombuffer(b"".join(keys), np.uint8).reshape(-1, 32), device=dev)
S = torch.tensor(np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64), device=dev)
d_so = torch.from_numpy(tso).to(dev)
d_tlo = torch.from_numpy(np.arange(0, 5 * ntx + 1, 5, dtype=np.int64)).to(dev)
out = {}
for name in ("leaf", "comp"):
    txid = torch.zeros((ntx, 32), dtype=torch.uint8, device=dev)
    st = torch.zeros(ntx, dtype=torch.uint8, device=dev)
    fb = torch.zeros(ntx, dtype=torch.int64, device=dev)
    sst = torch.zeros(len(keys), dtype=torch.uint8, device=dev)
    if name == "leaf":
        flat = [x for tx in leaves for x in tx]
        lb = torch.tensor(np.frombuffer(b"".join(flat), np.uint8), device=dev)
        lo = torch.tensor(np.concatenate([[0], np.cumsum([len(x) for x in flat])]).astype(np.int64), device=dev)
        eng.signed_tx_verify_ed25519_device(lb, lo, d_tlo, d_so, K, S, txid, st, fb, sst)
    else:
        d_items = torch.from_numpy(np.ascontiguousarray(it).view(np.uint8).copy()).to(dev)
        d_blob = torch.from_numpy(np.ascontiguousarray(blob)).to(dev)
        eng.signed_txcomp_verify_ed25519_device(d_items, len(it), d_blob, d_tlo, d_so, K, S, txid, st, fb, sst,
                                                group=5)
    torch.cuda.synchronize()
    out[name] = (txid.cpu().numpy(), st.cpu().numpy(), fb.cpu().numpy(), sst.cpu().numpy())
want_sig = np.zeros(len(keys), np.uint8)
for t in range(ntx):
    for q in range(int(nsig[t])):
        if (t * 3 + q) %% 17 == 5:
            want_sig[tso[t] + q] = 1
res = {"sigs": len(keys)}
for name, (txid, st, fb, sst) in out.items():
    res[name] = {"ids": int((txid != ids).any(axis=1).sum()), "tx_status": int((st != np.array(want_st)).sum()),
                 "first_bad": int((fb != np.array(want_fb)).sum()), "sig_status": int((sst != want_sig).sum())}
res["leaf_vs_comp"] = int(sum((a != b).sum() for a, b in zip(out["leaf"], out["comp"])))
print(json.dumps(res))
eng.close()
sys.exit(0 if all(v == 0 for k in ("leaf", "comp") for v in res[k].values()) and res["leaf_vs_comp"] == 0 else 1)
"""


def test_device_calls_in_small_chunks_subprocess():
    env = dict(os.environ, CORDAHIP_DEVICE_ED_CHUNK="192")
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT}], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["sigs"] > 8 * 192  # the remainder chunk and several full ones on both streams
