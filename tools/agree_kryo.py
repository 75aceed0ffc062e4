"""Encoder agreement sweep (dev tool, one MI355X): every leaf of C4's cash-issue
corpus (1.25 M transactions = 6.25 M components, per-rank seeds as bench.py)
encoded by the GPU template encoder (cordahip_kryo_encode_device) against the
host encoder (cordahip_kryo_encode), byte for byte; then every transaction id
of the component-level call (cordahip_signed_txcomp_verify: templates-only chain
and leaf hashes from the templates from the third call) against the ids of the
leaf-level path over the host encoder's leaves. One JSON line ->
profiles/r05_agreement_kryo.json.

usage: python tools/agree_kryo.py [--txs N] [--seeds K]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txs", type=int, default=1_250_000)
    ap.add_argument("--seeds", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_agreement_kryo.json"))
    a = ap.parse_args()
    import torch

    from corda_amd import _lib
    from corda_amd.corpus import cash_issue_items
    from corda_amd.engine import Engine
    dev = torch.device("cuda", 0)
    res = {"txs_per_seed": a.txs, "seeds": [], "leaves_compared": 0, "leaf_mismatches": 0, "ids_compared": 0,
           "id_mismatches": 0}
    t0 = time.time()
    with Engine(1) as eng:
        for seed in range(a.seeds):
            rng = np.random.default_rng(0xC0DA0004 + seed)
            ntx = a.txs
            blob, items, _ = cash_issue_items(rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                              rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                              rng.integers(0, 256, 32, dtype=np.uint8).tobytes(),
                                              rng.integers(1, 10**9, ntx), rng.integers(-2**63, 2**63 - 1, ntx))
            it = items.reshape(-1)
            host_it = it.copy()
            host_it["data"] += np.uint64(blob.ctypes.data)
            hb, ho = _lib.kryo_encode_array(host_it)
            d_blob = torch.from_numpy(blob).to(dev)
            dit = it.copy()
            dit["data"] += np.uint64(d_blob.data_ptr())
            d_items = torch.from_numpy(dit.view(np.uint8)).to(dev)
            n = dit.size
            off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            st = torch.zeros(n, dtype=torch.uint8, device=dev)
            out = torch.empty(int(ho[-1]), dtype=torch.uint8, device=dev)
            eng.kryo_encode_device(d_items, n, out, off, st, group=5)
            torch.cuda.synchronize()
            o = off.cpu().numpy().astype(np.uint64)
            leaf_ok = bool(np.array_equal(o, ho)) and bool(np.array_equal(out.cpu().numpy(), hb)) and int(st.sum()) == 0
            # the leaf path's ids over those leaves (equal to the host encoder's when leaf_ok):
            # the device signed-tx call, one blank signature per transaction (ids are compared)
            tlo = np.arange(0, n + 1, 5, dtype=np.uint64)
            d_tlo = torch.from_numpy(tlo.astype(np.int64)).to(dev)
            d_tso = torch.arange(ntx + 1, dtype=torch.int64, device=dev)
            txid = torch.empty((ntx, 32), dtype=torch.uint8, device=dev)
            tst = torch.empty(ntx, dtype=torch.uint8, device=dev)
            fb = torch.empty(ntx, dtype=torch.int64, device=dev)
            sst = torch.empty(ntx, dtype=torch.uint8, device=dev)
            zk = torch.zeros((ntx, 32), dtype=torch.uint8, device=dev)
            zs = torch.zeros((ntx, 64), dtype=torch.uint8, device=dev)
            eng.signed_tx_verify_ed25519_device(out, off, d_tlo, d_tso, zk, zs, txid, tst, fb, sst)
            torch.cuda.synchronize()
            ids_leaf = txid.cpu().numpy()
            sigs = [[(4, bytes(32), bytes(64))]] * ntx
            bad_ids = 0
            for call in range(3):
                r = eng.signed_txcomp_verify_arrays(blob, it, tlo, sigs, pinned_out=True)
                bad_ids += int((r[0] != ids_leaf[:ntx]).any(axis=1).sum())
            res["seeds"].append({"seed": seed, "leaves_equal": leaf_ok, "id_mismatches_3_calls": bad_ids})
            res["leaves_compared"] += n
            res["leaf_mismatches"] += 0 if leaf_ok else 1
            res["ids_compared"] += 3 * ntx
            res["id_mismatches"] += bad_ids
            del d_blob, d_items, off, st, out, txid, tst, fb, sst, zk, zs, d_tlo, d_tso
            torch.cuda.empty_cache()
    res["wall_s"] = time.time() - t0
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0 if res["leaf_mismatches"] == 0 and res["id_mismatches"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
