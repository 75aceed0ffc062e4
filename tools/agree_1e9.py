"""North-star agreement sweep: >= 1e9 mixed valid/invalid signatures on one MI355X.

BASELINE.json north_star asks for "100% verdict agreement with the reference on
>= 1e9 mixed valid/invalid signatures". This runs ED x 2^LOG2 Ed25519 lanes
(C2 corpora: 1% corrupted / non-canonical / off-curve / small-order / S + kL)
and EC x 2^LOG2 ECDSA lanes (C3 corpora: 50/50 secp256k1 / P-256, DER
malformations, r/s out of range, off-curve and compressed keys, high-S) through
the product kernels, each batch from a fresh seed, and checks EVERY lane's
status byte:
  * against the corpus construction where it fixes the exact status
    (valid lanes, and every corruption whose status is determined);
  * against the CPU oracle (oracle/c, the i2p 0.2.0 / BC 1.57 restatement)
    for every lane the construction leaves open (slide()-dependent S >= 2^255
    cases, "any rejection" ECDSA corruptions) and for a contiguous sample of
    2^SAMPLE lanes per batch (valid and corrupted alike).
Test infrastructure: the oracle is the checker here, never the thing measured.
Usage (GPU box): python tools/agree_1e9.py --out gpurun_out/agree.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def ecdsa_csr(sc, K, KL, S, SL, M):
    """Slot-layout lanes -> the oracle's CSR (bytes in lane order, vectorised)."""
    kl = KL.astype(np.int64)
    sl = SL.astype(np.int64)
    kb = np.ascontiguousarray(K[np.arange(K.shape[1])[None, :] < kl[:, None]])
    sb = np.ascontiguousarray(S[np.arange(S.shape[1])[None, :] < sl[:, None]])
    if kb.size == 0:
        kb = np.zeros(1, np.uint8)
    if sb.size == 0:
        sb = np.zeros(1, np.uint8)
    ko = np.zeros(len(sc) + 1, np.uint64)
    so = np.zeros(len(sc) + 1, np.uint64)
    ko[1:] = np.cumsum(kl)
    so[1:] = np.cumsum(sl)
    mo = np.arange(len(sc) + 1, dtype=np.uint64) * M.shape[1]
    return kb, ko, sb, so, np.ascontiguousarray(M), mo


def _log(args, scheme, b, n, checked, mism_c, mism_o, got, want, rejected, **extra):
    """One JSON line per batch: counts plus SHA-256 digests of the GPU's and the
    oracle's status bytes over the oracle-checked lanes (equal iff they agree)."""
    import hashlib
    if not args.log:
        return
    rec = {"scheme": scheme, "batch": b, "lanes": n, "oracle_checked": checked, "construction_mismatches": mism_c,
           "oracle_mismatches": mism_o, "rejected": rejected,
           "gpu_status_sha256": hashlib.sha256(got.tobytes()).hexdigest(),
           "oracle_status_sha256": hashlib.sha256(want.tobytes()).hexdigest()}
    rec.update(extra)
    with open(args.log, "a") as f:
        f.write(json.dumps(rec) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ed", type=int, default=48, help="Ed25519 batches")
    ap.add_argument("--ec", type=int, default=12, help="ECDSA batches")
    ap.add_argument("--log2", type=int, default=24)
    ap.add_argument("--sample-log2", type=int, default=15)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=None)
    ap.add_argument("--oracle-all", action="store_true",
                    help="oracle-check EVERY lane of every batch (not only the open lanes and a sample)")
    ap.add_argument("--first", type=int, default=0, help="index of the first batch (seeds are per batch index)")
    ap.add_argument("--log", default=None, help="append one JSON line per batch to this file")
    ap.add_argument("--stream-first", type=int, default=None, help="index of the first stream batch (default --first)")
    ap.add_argument("--stream", type=int, default=0,
                    help="C5 verifier-queue batches through cordahip_stream_verify (80%% Ed25519, 10%% P-256, "
                         "10%% secp256k1, pinned host memory), every lane oracle-checked")
    args = ap.parse_args()

    import torch

    from conftest import load_oracle
    from corda_amd.corpus import REJECT_ANY, make_c2_corpus, make_c3_corpus
    from corda_amd.engine import Engine

    orc = load_oracle()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    n = 1 << args.log2
    smp = 1 << args.sample_log2
    tot = {k: dict(lanes=0, construction_checked=0, oracle_checked=0, mismatches=0, rejected=0)
           for k in ("ed25519", "ecdsa", "stream")}

    def ec_oracle(sc, K, KL, S, SL, M, label):
        """C oracle statuses of slot-layout ECDSA lanes (CPU tensors), in 2^20-lane
        pieces with a progress line each (a silent 4-minute oracle call looks hung)."""
        kb, ko, sb, so, Mc, mo = ecdsa_csr(sc.numpy(), K.numpy(), KL.numpy(), S.numpy(), SL.numpy(), M.numpy())
        sch = np.ascontiguousarray(sc.numpy())
        want = np.zeros(len(sch), np.uint8)
        step = 1 << 20
        for p0 in range(0, len(sch), step):
            p1 = min(len(sch), p0 + step)
            orc.oracle_ecdsa_verify_batch(p1 - p0, sch[p0:].ctypes.data, kb.ctypes.data, ko[p0:].ctypes.data,
                                          sb.ctypes.data, so[p0:].ctypes.data, Mc.ctypes.data, mo[p0:].ctypes.data,
                                          want[p0:].ctypes.data, args.threads)
            print("  %s: oracle %d/%d ECDSA lanes (%.0f s)" % (label, p1, len(sch), time.time() - t0), flush=True)
        return want
    t0 = time.time()
    gpu_s = 0.0
    with Engine(1) as eng:
        for b in range(args.first, args.first + args.ed):
            pubs, sigs, msgs, exp, _ = make_c2_corpus(eng, n, 0xA9EE0000 + b, dev, stream=stream)
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            t1 = time.time()
            eng.ed25519_verify_device(pubs, sigs, msgs, st, None, stream=stream)
            torch.cuda.synchronize(dev)
            gpu_s += time.time() - t1
            known = exp >= 0
            mism = int((st[known].to(torch.int16) != exp[known]).sum())
            # oracle: every open lane plus the first `smp` lanes
            if args.oracle_all:
                idx = torch.arange(n, device=dev)
            else:
                idx = torch.nonzero(~known).flatten()
                idx = torch.unique(torch.cat([idx, torch.arange(smp, device=dev)]))
            k = pubs[idx].cpu().numpy().copy()
            s = sigs[idx].cpu().numpy().copy()
            m = msgs[idx].cpu().numpy().copy()
            want = np.zeros(len(idx), np.uint8)
            orc.oracle_ed25519_verify_batch(len(idx), k.ctypes.data, s.ctypes.data, m.ctypes.data, 32,
                                            want.ctypes.data, args.threads)
            got = st[idx].cpu().numpy()
            mism_o = int((got != want).sum())
            _log(args, "ed25519", b, n, len(idx), mism, mism_o, got, want, int((st != 0).sum()))
            r = tot["ed25519"]
            r["lanes"] += n
            r["construction_checked"] += int(known.sum())
            r["oracle_checked"] += len(idx)
            r["mismatches"] += mism + mism_o
            r["rejected"] += int((st != 0).sum())
            print("ed25519 batch %d/%d: %d lanes, construction mism %d, oracle-checked %d mism %d (%.0f s)"
                  % (b + 1, args.ed, n, mism, len(idx), mism_o, time.time() - t0), flush=True)
            del pubs, sigs, msgs, exp, st
        for b in range(args.first, args.first + args.ec):
            sc, K, KL, S, SL, M, exp, _ = make_c3_corpus(eng, n, 0xA9EC0000 + b, dev, stream=stream)
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            t1 = time.time()
            eng.ecdsa_verify_device(sc, K, KL, S, SL, M, st, None, stream=stream)
            torch.cuda.synchronize(dev)
            gpu_s += time.time() - t1
            exact = exp >= 0
            anyrej = exp == REJECT_ANY
            mism = int((st[exact].to(torch.int16) != exp[exact]).sum()) + int((st[anyrej] == 0).sum())
            if args.oracle_all:
                idx = torch.arange(n, device=dev)
            else:
                idx = torch.nonzero(~exact).flatten()
                idx = torch.unique(torch.cat([idx, torch.arange(smp, device=dev)]))
            csr = ecdsa_csr(sc[idx].cpu().numpy(), K[idx].cpu().numpy(), KL[idx].cpu().numpy(),
                            S[idx].cpu().numpy(), SL[idx].cpu().numpy(), M[idx].cpu().numpy())
            sch = np.ascontiguousarray(sc[idx].cpu().numpy())
            kb, ko, sb, so, Mc, mo = csr
            want = np.zeros(len(idx), np.uint8)
            # in pieces with a progress line each (a silent 4-minute oracle call looks hung to the box)
            step = 1 << 20
            for p0 in range(0, len(idx), step):
                p1 = min(len(idx), p0 + step)
                orc.oracle_ecdsa_verify_batch(p1 - p0, sch[p0:].ctypes.data, kb.ctypes.data, ko[p0:].ctypes.data,
                                              sb.ctypes.data, so[p0:].ctypes.data, Mc.ctypes.data, mo[p0:].ctypes.data,
                                              want[p0:].ctypes.data, args.threads)
                print("  ecdsa batch %d: oracle %d/%d lanes (%.0f s)" % (b, p1, len(idx), time.time() - t0), flush=True)
            got = st[idx].cpu().numpy()
            mism_o = int((got != want).sum())
            _log(args, "ecdsa", b, n, len(idx), mism, mism_o, got, want, int((st != 0).sum()))
            r = tot["ecdsa"]
            r["lanes"] += n
            r["construction_checked"] += int(exact.sum() + anyrej.sum())
            r["oracle_checked"] += len(idx)
            r["mismatches"] += mism + mism_o
            r["rejected"] += int((st != 0).sum())
            print("ecdsa batch %d/%d: %d lanes, construction mism %d, oracle-checked %d mism %d (%.0f s)"
                  % (b + 1, args.ec, n, mism, len(idx), mism_o, time.time() - t0), flush=True)
            del sc, K, KL, S, SL, M, exp, st
        # C5 verifier-queue batches: the stream drain (chunked H2D / kernels / D2H
        # through three buffer sets, both sections side by side) over pinned host
        # memory, as bench.py --workload c5 runs it
        sf = args.first if args.stream_first is None else args.stream_first
        for b in range(sf, sf + args.stream):
            n_ec = n // 5
            n_ed = n - n_ec
            pubs, sigs, msgs, exp_ed, _ = make_c2_corpus(eng, n_ed, 0xA9C50000 + b, dev, stream=stream)
            (sc, K, KL, S, SL, M, exp_ec, _) = make_c3_corpus(eng, n_ec, 0xA9C51000 + b, dev, stream=stream)
            torch.cuda.synchronize(dev)
            pin = lambda x: x.cpu().contiguous().pin_memory()  # noqa: E731
            ed = [pin(x) for x in (pubs, sigs, msgs)] + [torch.full((n_ed,), 0xEE, dtype=torch.uint8).pin_memory()]
            ec = [pin(x) for x in (sc, K, KL, S, SL, M)] + [torch.full((n_ec,), 0xEE, dtype=torch.uint8).pin_memory()]
            exp_ed, exp_ec = exp_ed.cpu(), exp_ec.cpu()
            del pubs, sigs, msgs, sc, K, KL, S, SL, M
            t1 = time.time()
            eng.stream_verify(ed, ec)
            gpu_s += time.time() - t1
            st_ed, st_ec = ed[3].numpy(), ec[6].numpy()
            k = (exp_ed >= 0).numpy()
            ex = (exp_ec >= 0).numpy()
            anyrej = (exp_ec == REJECT_ANY).numpy()
            mism = int((st_ed[k] != exp_ed.numpy()[k]).sum()) + int((st_ec[ex] != exp_ec.numpy()[ex]).sum()) \
                + int((st_ec[anyrej] == 0).sum())
            want_ed = np.zeros(n_ed, np.uint8)
            orc.oracle_ed25519_verify_batch(n_ed, ed[0].numpy().ctypes.data, ed[1].numpy().ctypes.data,
                                            ed[2].numpy().ctypes.data, 32, want_ed.ctypes.data, args.threads)
            print("  stream batch %d: oracle %d Ed25519 lanes (%.0f s)" % (b, n_ed, time.time() - t0), flush=True)
            want_ec = ec_oracle(*ec[:6], "stream batch %d" % b)
            got = np.concatenate([st_ed, st_ec])
            want = np.concatenate([want_ed, want_ec])
            mism_o = int((got != want).sum())
            rej = int((got != 0).sum())
            _log(args, "stream", b, n, n, mism, mism_o, got, want, rej, ed25519_lanes=n_ed, ecdsa_lanes=n_ec,
                 ed25519_oracle_mismatches=int((st_ed != want_ed).sum()),
                 ecdsa_oracle_mismatches=int((st_ec != want_ec).sum()))
            r = tot["stream"]
            r["lanes"] += n
            r["construction_checked"] += int(k.sum() + ex.sum() + anyrej.sum())
            r["oracle_checked"] += n
            r["mismatches"] += mism + mism_o
            r["rejected"] += rej
            print("stream batch %d/%d: %d lanes (%d Ed25519, %d ECDSA), construction mism %d, oracle mism %d (%.0f s)"
                  % (b + 1, args.stream, n, n_ed, n_ec, mism, mism_o, time.time() - t0), flush=True)
            del ed, ec, exp_ed, exp_ec
    lanes = sum(t["lanes"] for t in tot.values())
    out = {"lanes": lanes, "mismatches": sum(t["mismatches"] for t in tot.values()),
           "per_scheme": tot, "gpu_verify_s": gpu_s, "wall_s": time.time() - t0,
           "batch": n, "oracle_sample_per_batch": smp,
           "note": ("every lane's status vs the corpus construction where it fixes the status; " +
                    ("every lane vs the C oracle (--oracle-all)" if args.oracle_all else
                     "every open lane (slide()-dependent S, any-rejection ECDSA corruptions) plus a 2^%d-lane "
                     "sample per batch vs the C oracle" % args.sample_log2))}
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0 if out["mismatches"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
