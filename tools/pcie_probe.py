"""H2D / D2H bandwidth of the box from page-locked host memory (the bound of
the host-batch paths: c4h moves ~1.37 GB per 1.25 M cash-issue transactions).
One and two concurrent copy streams, 256 MiB and 1 GiB copies; prints one JSON line."""
import json
import time

import torch


def rate(nbytes, streams, direction, reps=5):
    dev = torch.device("cuda", 0)
    per = nbytes // streams
    hs = [torch.empty(per, dtype=torch.uint8).pin_memory() for _ in range(streams)]
    ds = [torch.empty(per, dtype=torch.uint8, device=dev) for _ in range(streams)]
    ss = [torch.cuda.Stream(dev) for _ in range(streams)]
    for _ in range(2):
        for h, d, s in zip(hs, ds, ss):
            with torch.cuda.stream(s):
                (d.copy_(h, non_blocking=True) if direction == "h2d" else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        for h, d, s in zip(hs, ds, ss):
            with torch.cuda.stream(s):
                (d.copy_(h, non_blocking=True) if direction == "h2d" else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize()
    return per * streams * reps / (time.perf_counter() - t) / 1e9


out = {}
for size in (256 << 20, 1 << 30):
    for st in (1, 2):
        for dr in ("h2d", "d2h"):
            out["%s_%dMiB_%dstream_GBps" % (dr, size >> 20, st)] = round(rate(size, st, dr), 2)
print(json.dumps(out))
