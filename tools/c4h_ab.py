"""Interleaved A/B of the signed-tx pipeline's per-call knobs on ONE corpus in ONE
process (dev tool): builds bench.py's c4h workload once (--components or
leaves), then for R rounds runs K timed calls under each configuration in turn
(environment variables the library reads per call: CORDAHIP_TX_SIG_CHUNK,
CORDAHIP_TX_SIG_CHUNK_MAX, CORDAHIP_TX_SLICE_AHEAD, CORDAHIP_TX_SLICES), so box
and clock drift hit every configuration alike. One JSON line: per configuration
the median and min/max of its per-round sig/s, and the check of the last call.

usage: python tools/c4h_ab.py [--components] [--rounds R] [--calls K] CFG [CFG ...]
  CFG: name:VAR=VALUE,VAR=VALUE  (e.g. c17a1:CORDAHIP_TX_SIG_CHUNK=131072)"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--components", action="store_true")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--workload", default="c4h")
    ap.add_argument("cfg", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from corda_amd.engine import Engine
    args = bench.parse_args(["--workload", a.workload] + (["--components"] if a.components else []))
    device = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    eng = Engine(1)
    stream = torch.cuda.Stream(device)
    torch.cuda.set_stream(stream)
    wl = bench.WORKLOADS[a.workload](eng, device, stream, 0, args)
    torch.cuda.synchronize(device)
    cfgs = []
    for c in a.cfg:
        name, _, kv = c.partition(":")
        cfgs.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    keys = sorted({k for _, e in cfgs for k in e})
    rates = {n: [] for n, _ in cfgs}
    for r in range(a.rounds):
        for name, env in cfgs:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            wl.step()  # one untimed call under this configuration
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            for _ in range(a.calls):
                wl.step()
            torch.cuda.synchronize(device)
            rates[name].append(wl.units * a.calls / (time.perf_counter() - t0))
    for k in keys:
        os.environ.pop(k, None)
    chk = wl.check()
    out = {"workload": a.workload, "components": a.components, "rounds": a.rounds, "calls": a.calls,
           "units": wl.units, "check": chk,
           "sig_per_s": {n: {"median": float(np.median(v)), "min": min(v), "max": max(v)} for n, v in rates.items()},
           "configs": {n: e for n, e in cfgs}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
