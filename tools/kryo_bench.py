"""Host Kryo leaf encoder throughput (cordahip_kryo_encode) on the C4 cash-issue
transactions of bench.py --native-leaves: the C call alone over prepared items
(one thread), and the whole corpus builder with 1 and 8 threads. Optional
argument: another libcordahip.so to time (A/B). Output bytes are digested so
variants can be compared."""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import _lib, corpus  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = sys.argv[1]
_lib.lib()
n = 200000
rng = np.random.default_rng(1)
ik = rng.integers(0, 256, (n, 32), dtype=np.uint8)
ok = rng.integers(0, 256, (n, 32), dtype=np.uint8)
q = rng.integers(1, 10**9, n).astype(np.int64)
nz = rng.integers(0, 2**62, n).astype(np.int64)
corpus.make_cash_issue_leaves(ik[:1000], ok[:1000], bytes(32), q[:1000], nz[:1000], threads=1)  # warm
# the C call alone: time kryo_encode_array inside a one-thread build
spent = [0.0]
orig = _lib.kryo_encode_array


def timed(items):
    t0 = time.perf_counter()
    r = orig(items)
    spent[0] += time.perf_counter() - t0
    return r


_lib.kryo_encode_array = timed
b, o = corpus.make_cash_issue_leaves(ik, ok, bytes(32), q, nz, threads=1)
_lib.kryo_encode_array = orig
print("C call, 1 thread: %.3f us/tx (%d B/tx)" % (spent[0] / n * 1e6, b.size // n))
for th in (1, 8):
    t = time.perf_counter()
    b, o = corpus.make_cash_issue_leaves(ik, ok, bytes(32), q, nz, threads=th)
    dt = time.perf_counter() - t
    print("builder, %d threads: %.3f us/tx, sha256 %s" % (th, dt / n * 1e6, hashlib.sha256(b.tobytes()).hexdigest()[:16]))
