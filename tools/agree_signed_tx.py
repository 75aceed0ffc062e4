"""Agreement sweep of the signed-transaction paths at scale:
>= 1e8 signature verdicts through cordahip_tx_submit (leaf bytes; the Ed25519
prep's key half ahead of the ids) and cordahip_txcomp_submit (Kryo components;
ids from the encoder's templates-only chain from the second call on), each
batch's two tickets outstanding together on one device (the overlapped calls);
with --device also through the device-resident calls on the same batch,
cordahip_signed_txcomp_verify_ed25519_device (the device hash chain: leaf
hashes straight from the encoder) and cordahip_signed_tx_verify_ed25519_device
(leaf bytes in HBM), both with the Ed25519 section in alternating chunks;
every output checked against the CPU oracle (oracle/c):

  * every transaction id against oracle_tx_id over the host encoder's leaves
    (SHA-256 + MerkleTree.kt restated in C; the leaves themselves are the
    components' Kryo preimages, cordahip_kryo_encode, whose bytes the r05 sweeps
    pinned against the GPU encoder);
  * every signature status against oracle_ed25519_verify (i2p 0.2.0 restated)
    over the oracle's id of its transaction, and against the construction
    (valid signatures OK; one R bit flipped, or the transaction's owner key
    changed after signing: BAD_SIG);
  * every transaction status and first_bad_sig against the reference's
    per-transaction rule (SignedTransaction.kt:95-100) applied to the oracle's
    signature statuses.

Batches are C4-shaped: TXS cash-issue transactions (5 components, 1-3 Ed25519
signers each), 1% of signatures with one R bit flipped, 0.5% of transactions
with an owner-key byte changed after signing -- fresh seeds per batch.
Test infrastructure: the oracle is the checker, never the thing measured.
Usage (GPU box): python tools/agree_signed_tx.py --batches 20 --out gpurun_out/agree_tx.json
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _pinned(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory()


def reduce_rule(sig_status, tso):
    """SignedTransaction.checkSignaturesAreValid per transaction: the first failing
    signature's index and status (-1 / OK if none); NO_SIGNATURES never occurs here"""
    ntx = len(tso) - 1
    bad = sig_status != 0
    fb = np.full(ntx, -1, np.int64)
    st = np.zeros(ntx, np.uint8)
    idx = np.nonzero(bad)[0]
    tx = np.searchsorted(tso, idx, side="right") - 1
    # the first bad per transaction: idx sorted ascending, keep the first occurrence of each tx
    first = np.unique(tx, return_index=True)
    tfirst, pos = first[0], idx[first[1]]
    fb[tfirst] = pos - tso[tfirst]
    st[tfirst] = sig_status[pos]
    return st, fb


def device_calls(eng, blob, items, lb, lo, tlo, tso, K, S):
    """the batch through the two device-resident signed-tx calls (inputs copied to HBM
    first, outside the checks); returns {name: (ids, tx_status, first_bad, sig_status)}"""
    import torch
    dev = torch.device("cuda:0")
    ntx, ns = len(tlo) - 1, len(K)
    d_so = torch.from_numpy(tso.astype(np.int64)).to(dev)
    d_tlo = torch.from_numpy(tlo.astype(np.int64)).to(dev)
    k = torch.from_numpy(K).to(dev)
    s = torch.from_numpy(S).to(dev)
    out = {}
    for name in ("device_txcomp", "device_leaf"):
        txid = torch.zeros((ntx, 32), dtype=torch.uint8, device=dev)
        st = torch.zeros(ntx, dtype=torch.uint8, device=dev)
        fb = torch.zeros(ntx, dtype=torch.int64, device=dev)
        sst = torch.zeros(ns, dtype=torch.uint8, device=dev)
        if name == "device_txcomp":
            d_items = torch.from_numpy(np.ascontiguousarray(items).view(np.uint8).copy()).to(dev)
            d_blob = torch.from_numpy(np.ascontiguousarray(blob, dtype=np.uint8)).to(dev)
            eng.signed_txcomp_verify_ed25519_device(d_items, len(items), d_blob, d_tlo, d_so, k, s, txid, st, fb, sst,
                                                    group=5)
            del d_items, d_blob
        else:
            d_lb = torch.from_numpy(lb).to(dev)
            d_lo = torch.from_numpy(lo.astype(np.int64)).to(dev)
            eng.signed_tx_verify_ed25519_device(d_lb, d_lo, d_tlo, d_so, k, s, txid, st, fb, sst)
            del d_lb, d_lo
        torch.cuda.synchronize()
        out[name] = (txid.cpu().numpy(), st.cpu().numpy(), sst.cpu().numpy(), fb.cpu().numpy())
    return out


def one_batch(eng, orc, b, seed, ntx, threads, device=False):
    import torch
    from corda_amd import _lib
    from corda_amd._lib import check, lib
    from corda_amd.corpus import cash_issue_items, make_cash_issue_leaves
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(seed)
    nsig = rng.integers(1, 4, ntx)
    tso = np.zeros(ntx + 1, np.uint64)
    tso[1:] = np.cumsum(nsig)
    ns = int(tso[-1])
    tx_of = np.repeat(np.arange(ntx), nsig)
    ik = rng.integers(0, 256, (ntx, 32), dtype=np.uint8)
    okeys = rng.integers(0, 256, (ntx, 32), dtype=np.uint8)
    notary = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    qty = rng.integers(1, 10**9, ntx)
    nonce = rng.integers(-2**63, 2**63 - 1, ntx)
    tlo = np.arange(0, 5 * ntx + 1, 5, dtype=np.uint64)
    # the ids the signers sign: before the owner keys of 0.5% of the transactions change
    lb0, lo0 = make_cash_issue_leaves(ik, okeys, notary, qty, nonce, threads=threads)
    ids_signed = np.zeros((ntx, 32), np.uint8)
    st0 = np.zeros(ntx, np.uint8)
    orc.oracle_tx_id_batch(ntx, lb0.ctypes.data, lo0.ctypes.data, tlo.ctypes.data, ids_signed.ctypes.data,
                           st0.ctypes.data, threads)
    del lb0, lo0
    bad_tx = rng.choice(ntx, max(1, ntx // 200), replace=False)
    okeys_bad = okeys.copy()
    okeys_bad[bad_tx, rng.integers(0, 32, bad_tx.size)] ^= 1
    lb, lo = make_cash_issue_leaves(ik, okeys_bad, notary, qty, nonce, threads=threads)
    ids = np.zeros((ntx, 32), np.uint8)
    st_o = np.zeros(ntx, np.uint8)
    orc.oracle_tx_id_batch(ntx, lb.ctypes.data, lo.ctypes.data, tlo.ctypes.data, ids.ctypes.data, st_o.ctypes.data,
                           threads)
    blob, items, _ = cash_issue_items(ik, okeys_bad, notary, qty, nonce)
    items = np.ascontiguousarray(items.reshape(-1))
    # signers: the GPU signer (corpus generation) over the signed ids; 1% of R bits flipped
    seeds = torch.from_numpy(rng.integers(0, 256, (ns, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(ids_signed[tx_of]).to(dev)
    pubs = torch.empty((ns, 32), dtype=torch.uint8, device=dev)
    sigs = torch.empty((ns, 64), dtype=torch.uint8, device=dev)
    eng.ed25519_sign_device(seeds, msgs, pubs, sigs)
    torch.cuda.synchronize()
    K, S = pubs.cpu().numpy(), sigs.cpu().numpy()
    del seeds, msgs, pubs, sigs
    bad_sig = rng.choice(ns, max(1, ns // 100), replace=False)
    S[bad_sig, rng.integers(0, 32, bad_sig.size)] ^= (1 << rng.integers(0, 8, bad_sig.size)).astype(np.uint8)
    construction = np.zeros(ns, np.uint8)
    construction[bad_sig] = 1
    construction[np.isin(tx_of, bad_tx)] = 1
    # the oracle: every signature over the oracle's id of its transaction
    M = np.ascontiguousarray(ids[tx_of])
    want_sig = np.zeros(ns, np.uint8)
    t0 = time.time()
    orc.oracle_ed25519_verify_batch(ns, K.ctypes.data, S.ctypes.data, M.ctypes.data, 32, want_sig.ctypes.data, threads)
    t_oracle = time.time() - t0
    want_st, want_fb = reduce_rule(want_sig, tso)
    # the two host boundaries, both tickets outstanding at once
    ar = np.arange(ns + 1, dtype=np.uint64)
    sig_arrays = [_pinned(x) for x in (np.full(ns, 4, np.uint8), K.reshape(-1), ar * 32, S.reshape(-1), ar * 64)]
    so_t = _pinned(tso)
    leaf_t = [_pinned(lb), _pinned(lo), _pinned(tlo)]
    comp_t = [_pinned(items.view(np.uint8)), _pinned(tlo), _pinned(blob)]
    outs = []
    for _ in range(2):
        outs.append((_pinned(np.zeros((ntx, 32), np.uint8)), _pinned(np.zeros(ntx, np.uint8)),
                     _pinned(np.zeros(ns, np.uint8)), _pinned(np.zeros(ntx, np.int64))))
    p = [x.data_ptr() for x in sig_arrays]
    o = [[x.data_ptr() for x in out] for out in outs]
    tb = _lib.TxidBatch(ntx, leaf_t[0].data_ptr(), leaf_t[1].data_ptr(), leaf_t[2].data_ptr(), o[0][0], o[0][1],
                        5 * ntx, lb.size)
    b_leaf = _lib.SignedTxBatch(tb, so_t.data_ptr(), *p, o[0][2], o[0][3], ns, K.size, S.size)
    cb = _lib.TxcompBatch(ntx, comp_t[0].data_ptr(), comp_t[1].data_ptr(), comp_t[2].data_ptr(), blob.size, o[1][0],
                          o[1][1], items.size)
    b_comp = _lib.SignedTxcompBatch(cb, so_t.data_ptr(), *p, o[1][2], o[1][3], ns, K.size, S.size)
    t1, t2 = ctypes.c_uint64(), ctypes.c_uint64()
    t0 = time.time()
    check(lib().cordahip_tx_submit(eng.ctx, ctypes.byref(b_leaf), ctypes.byref(t1)), "cordahip_tx_submit")
    check(lib().cordahip_txcomp_submit(eng.ctx, ctypes.byref(b_comp), ctypes.byref(t2)), "cordahip_txcomp_submit")
    check(lib().cordahip_wait(eng.ctx, t1.value, -1), "cordahip_wait")
    check(lib().cordahip_wait(eng.ctx, t2.value, -1), "cordahip_wait")
    t_gpu = time.time() - t0
    rec = {"batch": b, "seed": seed, "txs": ntx, "sigs": ns, "bad_txs": int(bad_tx.size), "bad_sigs": int(bad_sig.size),
           "oracle_vs_construction_mismatches": int((want_sig != construction).sum()),
           "oracle_tx_no_leaves": int((st_o != 0).sum()), "oracle_s": round(t_oracle, 2), "gpu_calls_s": round(t_gpu, 3)}
    results = [(name, tuple(x.numpy() for x in o)) for name, o in zip(("tx_submit", "txcomp_submit"), outs)]
    if device:
        t0 = time.time()
        results += list(device_calls(eng, blob, items, lb, lo, tlo, tso, K, S).items())
        rec["device_calls_s"] = round(time.time() - t0, 3)
    for name, (txid, txst, sst, fb) in results:
        rec[name] = {"id_mismatches": int((txid != ids).any(axis=1).sum()),
                     "sig_status_mismatches": int((sst != want_sig).sum()),
                     "tx_status_mismatches": int((txst != want_st).sum()),
                     "first_bad_mismatches": int((fb != want_fb).sum()),
                     "accepted_txs": int((txst == 0).sum()), "rejected_sigs": int((sst != 0).sum())}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--txs", type=int, default=1_250_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--log", default=None, help="append one JSON line per batch")
    ap.add_argument("--out", default=None)
    ap.add_argument("--device", action="store_true", help="also the two device-resident signed-tx calls")
    args = ap.parse_args()
    from conftest import load_oracle
    from corda_amd.engine import Engine
    orc = load_oracle()
    tot = {"batches": 0, "txs": 0, "sigs": 0, "verdicts_checked": 0, "id_checks": 0, "mismatches": 0,
           "oracle_vs_construction_mismatches": 0}
    t_start = time.time()
    with Engine(1) as eng:
        for k in range(args.batches):
            b = args.first + k
            rec = one_batch(eng, orc, b, 0xA6EE0000 + b, args.txs, args.threads, args.device)
            tot["batches"] += 1
            tot["txs"] += rec["txs"]
            tot["sigs"] += rec["sigs"]
            tot["oracle_vs_construction_mismatches"] += rec["oracle_vs_construction_mismatches"]
            for name in [x for x in ("tx_submit", "txcomp_submit", "device_txcomp", "device_leaf") if x in rec]:
                r = rec[name]
                tot["verdicts_checked"] += rec["sigs"]
                tot["id_checks"] += rec["txs"]
                tot["mismatches"] += (r["id_mismatches"] + r["sig_status_mismatches"] + r["tx_status_mismatches"]
                                      + r["first_bad_mismatches"])
            print(json.dumps(rec), flush=True)
            if args.log:
                with open(args.log, "a") as f:
                    f.write(json.dumps(rec) + "\n")
    tot["wall_s"] = round(time.time() - t_start, 1)
    tot["what"] = ("cordahip_tx_submit + cordahip_txcomp_submit (two tickets outstanding per batch on one device)%s, "
                   "every id, signature status, tx status and first_bad_sig against oracle/c; signature statuses also "
                   "against the construction" % (
                       " + cordahip_signed_txcomp_verify_ed25519_device + cordahip_signed_tx_verify_ed25519_device"
                       if args.device else ""))
    print(json.dumps(tot), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(tot, f, indent=1)
    return 0 if tot["mismatches"] == 0 and tot["oracle_vs_construction_mismatches"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
