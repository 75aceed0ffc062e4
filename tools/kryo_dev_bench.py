"""GPU Kryo encoder on the C4 cash-issue corpus (1.25 M transactions = 6.25 M
components in HBM): ms per cordahip_kryo_encode_device call (HIP events around
its launches, cordahip_last_kernel_ms), first-call (templates built) and
steady-state (templates cached) separately, and the leaves of the first 20,000
transactions against the host encoder. One JSON line.
usage: python tools/kryo_dev_bench.py [--txs N] [--calls K]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txs", type=int, default=1_250_000)
    ap.add_argument("--calls", type=int, default=10)
    args = ap.parse_args()
    import torch

    from corda_amd import _lib
    from corda_amd.corpus import cash_issue_items
    from corda_amd.engine import Engine
    ntx = args.txs
    rng = np.random.default_rng(0xC0DA0004)
    blob, items, _ = cash_issue_items(rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                      rng.integers(0, 256, (ntx, 32), dtype=np.uint8),
                                      rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(1, 10**9, ntx),
                                      rng.integers(-2**63, 2**63 - 1, ntx))
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(blob).to(dev)
    it = items.reshape(-1).copy()
    it["data"] += np.uint64(d_blob.data_ptr())
    d_items = torch.from_numpy(it.view(np.uint8)).to(dev)
    n = it.size
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    with Engine(1) as eng:
        eng.kryo_encode_device(d_items, n, None, off, st, group=5)  # sizes only (also builds the templates)
        torch.cuda.synchronize()
        out = torch.empty(int(off[-1]), dtype=torch.uint8, device=dev)
        ms = []
        for _ in range(args.calls):
            eng.kryo_encode_device(d_items, n, out, off, st, group=5)
            ms.append(_lib.lib().cordahip_last_kernel_ms(eng._ctx, 0))
        torch.cuda.synchronize()
        k = min(ntx, 20000) * 5
        host_it = items.reshape(-1)[:k].copy()
        host_it["data"] += np.uint64(blob.ctypes.data)
        hb, ho = _lib.kryo_encode_array(host_it)
        ok = (np.array_equal(off[:k + 1].cpu().numpy().astype(np.uint64), ho)
              and np.array_equal(out[:int(ho[-1])].cpu().numpy(), hb))
    res = {"txs": ntx, "leaves": n, "leaf_bytes": int(off[-1]), "bytes_per_tx": int(off[-1]) / ntx,
           "ms_first_call_sizes_only": None, "ms_per_call": ms, "ms_median": float(np.median(ms)),
           "txs_per_s": ntx / (float(np.median(ms)) * 1e-3), "item_errors": int((st != 0).sum()),
           "leaves_checked_vs_host": k, "leaves_equal_host": bool(ok)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
