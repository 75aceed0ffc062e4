"""Python handle on a libcordahip context (plumbing for tests and bench.py).

`Engine` owns one `cordahip_ctx`. Host batches go through the C-ABI's
generic CSR batch (`cordahip_sig_verify`, the `Crypto.isValid` batch
replacement) or the dense Ed25519 host path; device batches take torch
tensors that already live in HBM and run on the caller's HIP stream.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (EngineError, FilteredTxBatch, SigBatch, SignedTxBatch, SignedTxcompBatch, StreamBatch, TxcompBatch,
                   TxidBatch, check, lib)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


class Engine:
    def __init__(self, device_mask: int = 0):
        l = lib()
        self._ctx = ctypes.c_void_p()
        check(l.cordahip_init(device_mask, ctypes.byref(self._ctx)), "cordahip_init")

    def close(self):
        if self._ctx:
            lib().cordahip_shutdown(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def ctx(self):
        return self._ctx

    def device_count(self) -> int:
        return lib().cordahip_device_count(self._ctx)

    # ---- generic batch: Crypto.isValid per lane -------------------------------
    @staticmethod
    def _csr(items: Sequence[bytes]):
        off = np.zeros(len(items) + 1, dtype=np.uint64)
        if items:
            off[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
        blob = np.frombuffer(b"".join(items), dtype=np.uint8) if off[-1] else np.zeros(1, np.uint8)
        return np.ascontiguousarray(blob), off

    def verify_batch(self, schemes: Sequence[int], keys: Sequence[bytes], sigs: Sequence[bytes],
                     msgs: Sequence[bytes], async_: bool = False, is_valid: bool = False):
        """Per-lane statuses for (scheme, key, sig, msg) tuples; returns (status, verdict).
        is_valid=False: Crypto.doVerify semantics (empty sig / clear data -> EMPTY);
        is_valid=True: Crypto.isValid semantics (no emptiness checks)."""
        n = len(keys)
        sch = np.ascontiguousarray(np.asarray(schemes, dtype=np.uint8))
        kb, ko = self._csr(list(keys))
        sb, so = self._csr(list(sigs))
        mb, mo = self._csr(list(msgs))
        status = np.zeros(max(n, 1), dtype=np.uint8)
        verdict = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        b = SigBatch(n, _ptr(sch), _ptr(kb), _ptr(ko), _ptr(sb), _ptr(so), _ptr(mb), _ptr(mo),
                     _ptr(status), _ptr(verdict), _lib.FLAG_IS_VALID if is_valid else 0, kb.size, sb.size, mb.size)
        keep = (sch, kb, ko, sb, so, mb, mo, status, verdict, b)
        if async_:
            t = ctypes.c_uint64()
            check(lib().cordahip_sig_submit(self._ctx, ctypes.byref(b), ctypes.byref(t)), "cordahip_sig_submit")
            return Ticket(self, t.value, lambda: (status[:n], verdict), keep)
        check(lib().cordahip_sig_verify(self._ctx, ctypes.byref(b)), "cordahip_sig_verify")
        return status[:n], verdict

    # ---- dense Ed25519 host path ---------------------------------------------
    def ed25519_verify_host(self, keys: np.ndarray, sigs: np.ndarray, msgs: np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, 32)
        n = keys.shape[0]
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(n, 64)
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8).reshape(n, -1)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        verdict = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        check(lib().cordahip_ed25519_verify_host(self._ctx, _ptr(keys), _ptr(sigs), _ptr(msgs), msgs.shape[1], n,
                                                 _ptr(status), _ptr(verdict)), "cordahip_ed25519_verify_host")
        return status[:n], verdict

    # ---- device-resident paths (torch tensors in HBM) -------------------------
    def ed25519_verify_device(self, keys, sigs, msgs, status, verdict=None, device: int = 0, stream=None):
        n = keys.shape[0]
        s = stream.cuda_stream if stream is not None else 0
        check(lib().cordahip_ed25519_verify_device(
            self._ctx, device, keys.data_ptr(), sigs.data_ptr(), msgs.data_ptr(), msgs.shape[1], n,
            status.data_ptr(), verdict.data_ptr() if verdict is not None else None, s),
            "cordahip_ed25519_verify_device")

    def ed25519_sign_device(self, seeds, msgs, pubs, sigs, device: int = 0, stream=None):
        n = seeds.shape[0]
        s = stream.cuda_stream if stream is not None else 0
        check(lib().cordahip_ed25519_sign_device(self._ctx, device, seeds.data_ptr(), msgs.data_ptr(),
                                                 msgs.shape[1], n, pubs.data_ptr(), sigs.data_ptr(), s),
              "cordahip_ed25519_sign_device")

    def ecdsa_sign_device(self, scheme, seeds, msgs, keys, key_len, sigs, sig_len, device: int = 0, stream=None):
        """Device tensors: scheme[n] u8 (2/3), seeds[n,32], msgs[n,L] -> keys[n,65], key_len[n], sigs[n,72], sig_len[n]."""
        n = seeds.shape[0]
        s = stream.cuda_stream if stream is not None else 0
        check(lib().cordahip_ecdsa_sign_device(self._ctx, device, scheme.data_ptr(), seeds.data_ptr(), msgs.data_ptr(),
                                               msgs.shape[1], n, keys.data_ptr(), key_len.data_ptr(), sigs.data_ptr(),
                                               sig_len.data_ptr(), s), "cordahip_ecdsa_sign_device")

    # ---- transactions: WireTransaction.id and SignedTransaction verification ---
    def _tx_arrays(self, txs: Sequence[Sequence[bytes]]):
        leaves = [leaf for tx in txs for leaf in tx]
        lb, lo = self._csr(leaves)
        to = np.zeros(len(txs) + 1, dtype=np.uint64)
        if txs:
            to[1:] = np.cumsum([len(tx) for tx in txs], dtype=np.uint64)
        txid = np.zeros((max(len(txs), 1), 32), dtype=np.uint8)
        st = np.zeros(max(len(txs), 1), dtype=np.uint8)
        b = TxidBatch(len(txs), _ptr(lb), _ptr(lo), _ptr(to), _ptr(txid), _ptr(st), len(leaves), lb.size)
        return b, (lb, lo, to, txid, st)

    def tx_ids(self, txs: Sequence[Sequence[bytes]], async_: bool = False):
        """txs: per transaction, the serialised components (leaf preimages). Returns (ids[ntx,32], status[ntx])
        (or a Ticket whose wait() returns them)."""
        b, keep = self._tx_arrays(txs)
        res = lambda: (keep[3][:len(txs)], keep[4][:len(txs)])  # noqa: E731
        if async_:
            t = ctypes.c_uint64()
            check(lib().cordahip_txid_submit(self._ctx, ctypes.byref(b), ctypes.byref(t)), "cordahip_txid_submit")
            return Ticket(self, t.value, res, (b, keep))
        check(lib().cordahip_tx_ids(self._ctx, ctypes.byref(b)), "cordahip_tx_ids")
        return res()

    def signed_tx_verify(self, txs: Sequence[Sequence[bytes]], sigs: Sequence[Sequence[tuple]],
                         async_: bool = False):
        """sigs[t] = [(scheme, key, sig), ...] in list order. Returns (ids, tx_status, first_bad, sig_status)
        (or, async_, a Ticket from cordahip_tx_submit whose wait() returns them)."""
        b, keep = self._tx_arrays(txs)
        flat = [x for per in sigs for x in per]
        so = np.zeros(len(txs) + 1, dtype=np.uint64)
        if txs:
            so[1:] = np.cumsum([len(per) for per in sigs], dtype=np.uint64)
        sch = np.ascontiguousarray(np.asarray([x[0] for x in flat] or [0], dtype=np.uint8))
        kb, ko = self._csr([x[1] for x in flat])
        sb, sgo = self._csr([x[2] for x in flat])
        sst = np.zeros(max(len(flat), 1), dtype=np.uint8)
        fb = np.zeros(max(len(txs), 1), dtype=np.int64)
        sbatch = SignedTxBatch(b, _ptr(so), _ptr(sch), _ptr(kb), _ptr(ko), _ptr(sb), _ptr(sgo), _ptr(sst), _ptr(fb),
                               len(flat), kb.size, sb.size)
        n = len(txs)
        res = lambda: (keep[3][:n], keep[4][:n], fb[:n], sst[:len(flat)])  # noqa: E731
        if async_:
            t = ctypes.c_uint64()
            check(lib().cordahip_tx_submit(self._ctx, ctypes.byref(sbatch), ctypes.byref(t)), "cordahip_tx_submit")
            return Ticket(self, t.value, res, (keep, so, sch, kb, ko, sb, sgo, sst, fb, sbatch))
        check(lib().cordahip_signed_tx_verify(self._ctx, ctypes.byref(sbatch)), "cordahip_signed_tx_verify")
        return res()

    def signed_txcomp_verify(self, txs, sigs, async_: bool = False):
        """cordahip_signed_txcomp_verify / cordahip_txcomp_submit: txs[t] = the transaction's components
        as (kind, value, class_id) tuples (_lib.kryo_pack's form, availableComponents order) -- the GPU
        writes their leaves; sigs as in signed_tx_verify. Returns (ids, tx_status, first_bad, sig_status)."""
        comps = [c for tx in txs for c in tx]
        blob, items, has = _lib.kryo_pack(comps)
        items = items.copy()
        items["data"] = np.where(has, items["data"], 0)  # offsets into the payload
        tio = np.zeros(len(txs) + 1, dtype=np.uint64)
        if txs:
            tio[1:] = np.cumsum([len(tx) for tx in txs], dtype=np.uint64)
        return self.signed_txcomp_verify_arrays(np.ascontiguousarray(blob), items, tio, sigs, async_=async_)

    def signed_txcomp_verify_arrays(self, payload, items, tx_item_off, sigs, async_: bool = False,
                                    pinned_out: bool = False):
        """The array form: payload uint8, items KRYO_ITEM_DTYPE whose `data` are offsets into payload,
        tx_item_off uint64[ntx + 1]; sigs[t] = [(scheme, key, sig), ...]. pinned_out: txid and
        tx_status in page-locked memory (the library's kernels then store them through their
        device mapping, as for a JVM's pinned direct buffers)."""
        n = len(tx_item_off) - 1
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        items = np.ascontiguousarray(items)
        tio = np.ascontiguousarray(tx_item_off, dtype=np.uint64)
        pins = ()
        if pinned_out:
            import torch
            pins = (torch.zeros((max(n, 1), 32), dtype=torch.uint8).pin_memory(),
                    torch.zeros(max(n, 1), dtype=torch.uint8).pin_memory())
            txid, st = pins[0].numpy(), pins[1].numpy()
        else:
            txid = np.zeros((max(n, 1), 32), dtype=np.uint8)
            st = np.zeros(max(n, 1), dtype=np.uint8)
        tb = TxcompBatch(n, _ptr(items) if len(items) else None, _ptr(tio), _ptr(payload) if payload.size else None,
                         payload.size, _ptr(txid), _ptr(st), len(items))
        flat = [x for per in sigs for x in per]
        so = np.zeros(n + 1, dtype=np.uint64)
        if n:
            so[1:] = np.cumsum([len(per) for per in sigs], dtype=np.uint64)
        sch = np.ascontiguousarray(np.asarray([x[0] for x in flat] or [0], dtype=np.uint8))
        kb, ko = self._csr([x[1] for x in flat])
        sb, sgo = self._csr([x[2] for x in flat])
        sst = np.zeros(max(len(flat), 1), dtype=np.uint8)
        fb = np.zeros(max(n, 1), dtype=np.int64)
        sbatch = SignedTxcompBatch(tb, _ptr(so), _ptr(sch), _ptr(kb), _ptr(ko), _ptr(sb), _ptr(sgo), _ptr(sst),
                                   _ptr(fb), len(flat), kb.size, sb.size)
        res = lambda: (txid[:n], st[:n], fb[:n], sst[:len(flat)])  # noqa: E731
        keep = (payload, items, tio, txid, st, so, sch, kb, ko, sb, sgo, sst, fb, tb, sbatch, pins)
        if async_:
            t = ctypes.c_uint64()
            check(lib().cordahip_txcomp_submit(self._ctx, ctypes.byref(sbatch), ctypes.byref(t)),
                  "cordahip_txcomp_submit")
            return Ticket(self, t.value, res, keep)
        check(lib().cordahip_signed_txcomp_verify(self._ctx, ctypes.byref(sbatch)), "cordahip_signed_txcomp_verify")
        return res()

    def signed_tx_verify_ed25519_device(self, leaf_bytes, leaf_off, tx_leaf_off, tx_sig_off, keys, sigs,
                                        txid, tx_status, first_bad, sig_status, device: int = 0, stream=None):
        s = stream.cuda_stream if stream is not None else 0
        check(lib().cordahip_signed_tx_verify_ed25519_device(
            self._ctx, device, leaf_bytes.data_ptr(), leaf_off.data_ptr(), leaf_off.shape[0] - 1,
            tx_leaf_off.data_ptr(), tx_leaf_off.shape[0] - 1, tx_sig_off.data_ptr(), keys.data_ptr(),
            sigs.data_ptr(), keys.shape[0], txid.data_ptr(), tx_status.data_ptr(), first_bad.data_ptr(),
            sig_status.data_ptr(), s), "cordahip_signed_tx_verify_ed25519_device")

    def signed_txcomp_verify_ed25519_device(self, items, n_items: int, payload, tx_item_off, tx_sig_off, keys, sigs,
                                            txid, tx_status, first_bad, sig_status, group: int = 1, device: int = 0,
                                            stream=None):
        """cordahip_signed_txcomp_verify_ed25519_device: items (device tensor of n_items
        cordahip_kryo_item records whose `data` are offsets into payload), payload (uint8 device
        tensor), tx_item_off / tx_sig_off (int64 [ntx + 1]), keys [nsig, 32], sigs [nsig, 64];
        outputs as in signed_tx_verify_ed25519_device."""
        s = stream.cuda_stream if stream is not None else 0
        check(lib().cordahip_signed_txcomp_verify_ed25519_device(
            self._ctx, device, items.data_ptr(), n_items, group, payload.data_ptr() if payload.numel() else None,
            payload.numel(), tx_item_off.data_ptr(), tx_item_off.shape[0] - 1, tx_sig_off.data_ptr(),
            keys.data_ptr(), sigs.data_ptr(), keys.shape[0], txid.data_ptr(), tx_status.data_ptr(),
            first_bad.data_ptr(), sig_status.data_ptr(), s), "cordahip_signed_txcomp_verify_ed25519_device")

    def device_mem(self, device: int = 0):
        """cordahip_device_mem: (bytes the library holds on the device's GPU, their peak, the budget)"""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().cordahip_device_mem(self._ctx, device, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
              "cordahip_device_mem")
        return a.value, b.value, c.value

    def trim(self):
        """cordahip_trim: release every device's grow-only buffers now"""
        check(lib().cordahip_trim(self._ctx), "cordahip_trim")

    def kryo_encode_device(self, items, n: int, out, off, status, group: int = 1, device: int = 0, stream=None):
        """cordahip_kryo_encode_device: leaf preimages of n components on the GPU. items: a
        device tensor holding n cordahip_kryo_item records (_lib.KRYO_ITEM_DTYPE) whose data
        pointers are device addresses; out: uint8 device tensor (its size is the cap); off:
        n + 1 int64; status: n uint8 (0 written, 1 invalid item, 2 beyond cap)."""
        s = stream.cuda_stream if stream is not None else 0
        check(lib().cordahip_kryo_encode_device(self._ctx, device, items.data_ptr(), n, group,
                                                out.data_ptr() if out is not None else None,
                                                out.numel() if out is not None else 0, off.data_ptr(),
                                                status.data_ptr(), s), "cordahip_kryo_encode_device")

    def kryo_encode_packed_device(self, blob, items, has, group: int = 1, cap=None, device: int = 0, stream=None):
        """_lib.kryo_pack output (payload blob, items with blob offsets, has-payload mask) encoded on
        the GPU: the blob and the rebased items go to the device, then cordahip_kryo_encode_device.
        cap None: sized by a first pass. Synchronous (returns host-visible results): (leaves uint8
        device tensor, off int64 device tensor [n + 1], status uint8 device tensor [n])."""
        import contextlib

        import torch
        dev = torch.device("cuda", device)
        # the copies and zero fills are ordered before the encoder on `stream`
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            d_blob = torch.from_numpy(np.ascontiguousarray(blob)).to(dev)
            a = np.array(items, copy=True)
            a["data"] = np.where(has, a["data"] + np.uint64(d_blob.data_ptr()), 0)
            d_items = torch.from_numpy(a.view(np.uint8)).to(dev)
            n = len(a)
            off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            status = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        if cap is None:
            self.kryo_encode_device(d_items, n, None, off, status, group, device, stream)
            torch.cuda.synchronize(dev)
            cap = int(off[n])
        out = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
        self.kryo_encode_device(d_items, n, out, off, status, group, device, stream)
        torch.cuda.synchronize(dev)
        return out[:cap], off, status[:n]

    def ecdsa_verify_device(self, scheme, keys, key_len, sigs, sig_len, msgs, status, verdict=None, device: int = 0,
                            stream=None):
        """Dense mixed secp256k1/P-256 batch in HBM: keys [n,65] + key_len, DER sigs [n,72] + sig_len."""
        s = stream.cuda_stream if stream is not None else 0
        check(lib().cordahip_ecdsa_verify_device(
            self._ctx, device, scheme.data_ptr(), keys.data_ptr(), key_len.data_ptr(), sigs.data_ptr(),
            sig_len.data_ptr(), msgs.data_ptr(), msgs.shape[1], scheme.shape[0], status.data_ptr(),
            verdict.data_ptr() if verdict is not None else None, s), "cordahip_ecdsa_verify_device")

    # ---- FilteredTransaction.verify / PartialMerkleTree.verify ----------------
    def filtered_tx_verify(self, ftxs, async_: bool = False):
        """ftxs[t] = (leaves: [bytes], tokens: [(tok, hash32 or None)], root: bytes32), tokens being the
        post-order stream of the PartialMerkleTree (oracle/partial_merkle.py tokens()). Returns tx_status."""
        leaves = [leaf for f in ftxs for leaf in f[0]]
        lb, lo = self._csr(leaves)
        to = np.zeros(len(ftxs) + 1, dtype=np.uint64)
        ko = np.zeros(len(ftxs) + 1, dtype=np.uint64)
        if ftxs:
            to[1:] = np.cumsum([len(f[0]) for f in ftxs], dtype=np.uint64)
            ko[1:] = np.cumsum([len(f[1]) for f in ftxs], dtype=np.uint64)
        toks = [t for f in ftxs for t in f[1]]
        tok = np.ascontiguousarray(np.array([t[0] for t in toks] or [0], dtype=np.uint8))
        th = np.frombuffer(b"".join((t[1] or bytes(32)) for t in toks) or bytes(32), dtype=np.uint8).copy()
        root = np.frombuffer(b"".join(f[2] for f in ftxs) or bytes(32), dtype=np.uint8).copy()
        st = np.zeros(max(len(ftxs), 1), dtype=np.uint8)
        b = FilteredTxBatch(len(ftxs), _ptr(lb), _ptr(lo), _ptr(to), _ptr(tok), _ptr(th), _ptr(ko), _ptr(root),
                            _ptr(st), len(leaves), lb.size, len(toks))
        if async_:
            t = ctypes.c_uint64()
            check(lib().cordahip_filtered_tx_submit(self._ctx, ctypes.byref(b), ctypes.byref(t)),
                  "cordahip_filtered_tx_submit")
            return Ticket(self, t.value, lambda: st[:len(ftxs)], (lb, lo, to, tok, th, ko, root, st, b))
        check(lib().cordahip_filtered_tx_verify(self._ctx, ctypes.byref(b)), "cordahip_filtered_tx_verify")
        return st[:len(ftxs)]

    # ---- C5: streaming mixed-scheme drain (host, ideally pinned, memory) -------
    def stream_verify(self, ed, ec):
        """ed = (keys[n,32], sigs[n,64], msgs[n,L], status[n]) and ec = (scheme[n], keys[n,65],
        key_len[n], sigs[n,72], sig_len[n], msgs[n,L], status[n]): host arrays (numpy or CPU torch
        tensors; pin them for overlapped copies). Statuses are written in place."""
        def p(x):
            return x.data_ptr() if hasattr(x, "data_ptr") else x.ctypes.data

        ek, es, em, est = ed
        sc, ck, ckl, cs, csl, cm, cst = ec
        b = StreamBatch(ek.shape[0], p(ek), p(es), p(em), em.shape[1] if ek.shape[0] else 0, p(est),
                        sc.shape[0], p(sc), p(ck), p(ckl), p(cs), p(csl), p(cm), cm.shape[1] if sc.shape[0] else 0,
                        p(cst))
        check(lib().cordahip_stream_verify(self._ctx, ctypes.byref(b)), "cordahip_stream_verify")

    def last_kernel_ms(self, device: int = 0) -> float:
        return lib().cordahip_last_kernel_ms(self._ctx, device)


class Ticket:
    """A submitted batch (cordahip_*_submit). wait() releases the ticket and returns the
    batch's results; poll() only reports completion. `keep` pins the host buffers."""

    def __init__(self, eng: Engine, ticket: int, result, keep):
        self.eng, self.ticket, self._result, self._keep = eng, ticket, result, keep
        self._waited = False

    def __del__(self):
        # a ticket dropped without wait(): the pool may still be writing into the
        # buffers self._keep pins, so wait for it before they can be freed
        if not getattr(self, "_waited", True) and self.eng.ctx:
            lib().cordahip_wait(self.eng.ctx, self.ticket, -1)

    def poll(self) -> bool:
        r = lib().cordahip_poll(self.eng.ctx, self.ticket)
        if r < 0:
            raise EngineError(r, "cordahip_poll")
        return r == 1

    def wait(self, timeout_ns: int = -1):
        rc = lib().cordahip_wait(self.eng.ctx, self.ticket, timeout_ns)
        if rc != _lib.ERR_TIMEOUT:
            self._waited = True  # released by the library (successfully or not)
        check(rc, "cordahip_wait")
        return self._result()
