"""Synthetic, seeded corpora for the benchmark configs.

C2: a batch of Ed25519 (key, sig, 32-byte txId) tuples, all made on the GPU by
libcordahip's RFC 8032 signer (cordahip_ed25519_sign_device, the analogue of
Crypto.doSign / deriveKeyPairFromEntropy), then 1% of lanes corrupted with the
fixed catalogue mix of SURVEY §8(d) C2. Everything stays in HBM.

The special encodings below are DATA (derived once from the curve equation and
listed here so the corpus is reproducible without any curve arithmetic):
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

L = 2**252 + 27742317777372353535851937790883648493
P = 2**255 - 19

# the 8 small-order points of edwards25519 (canonical encodings)
SMALL_ORDER_KEYS = [
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0000000000000000000000000000000000000000000000000000000000000080",
    "0100000000000000000000000000000000000000000000000000000000000000",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
]
# y + p encodings (y < 19) that decode to curve points: non-canonical keys
NONCANONICAL_KEYS = ["%02xffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff%s" % (0xED + y, s)
                     for y in (0, 1) for s in ("7f", "ff")]
# small y values that are NOT on the curve: decode fails (BAD_KEY)
OFF_CURVE_KEYS = ["%02x" % y + "00" * 31 for y in (2, 7, 8, 11, 12, 13, 17, 20)]
# y + p encodings used as R: never equal to a canonical encode(R')
NONCANONICAL_R = ["%02xffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff%s" % (0xED + y, s)
                  for y in range(0, 19) for s in ("7f", "ff") if 0xED + y <= 0xFF]

# C2 mix (fractions of the corrupted lanes)
C2_MIX = [("r_bitflip", 0.30), ("s_bitflip", 0.20), ("msg_bitflip", 0.10), ("wrong_key", 0.10),
          ("s_plus_kL", 0.10), ("r_noncanonical", 0.05), ("key_noncanonical", 0.05),
          ("key_off_curve", 0.05), ("key_small_order", 0.05)]
# expected status per category; None = decided by slide() (checked against the oracle in tests)
C2_EXPECTED = {"r_bitflip": 1, "s_bitflip": 1, "msg_bitflip": 1, "wrong_key": 1, "s_plus_kL": None,
               "r_noncanonical": 1, "key_noncanonical": 1, "key_off_curve": 3, "key_small_order": 1}


def _consts(hexes, torch, device):
    return torch.tensor(np.frombuffer(bytes.fromhex("".join(hexes)), np.uint8).reshape(len(hexes), 32),
                        device=device)


def make_c2_corpus(engine, n: int, seed: int, device, corrupt_frac: float = 0.01, stream=None,
                   dev_index: int = 0):
    """Returns (pubs[n,32], sigs[n,64], msgs[n,32], expected[n] int16 (-1 = slide-dependent), categories)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=device, generator=g)
    msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=device, generator=g)
    pubs = torch.empty((n, 32), dtype=torch.uint8, device=device)
    sigs = torch.empty((n, 64), dtype=torch.uint8, device=device)
    engine.ed25519_sign_device(seeds, msgs, pubs, sigs, device=dev_index, stream=stream)
    torch.cuda.synchronize(device)
    del seeds
    expected, cats = corrupt_c2(pubs, sigs, msgs, seed, g, corrupt_frac)
    torch.cuda.synchronize(device)
    return pubs, sigs, msgs, expected, cats


def corrupt_c2(pubs, sigs, msgs, seed: int, g, corrupt_frac: float = 0.01):
    """Apply the C2 corruption catalogue in place (works on CPU or GPU tensors)."""
    import torch

    n, device = pubs.shape[0], pubs.device
    expected = torch.zeros(n, dtype=torch.int16, device=device)
    ncor = int(n * corrupt_frac)
    perm = torch.randperm(n, device=device, generator=g)[:ncor]
    cats: Dict[str, torch.Tensor] = {}
    start = 0
    for i, (name, frac) in enumerate(C2_MIX):
        cnt = ncor - start if i == len(C2_MIX) - 1 else int(round(ncor * frac))
        cats[name] = perm[start:start + cnt]
        start += cnt
    orig_pubs = pubs.clone()

    def flip(t, idx, lo_byte, nbits):
        bit = torch.randint(0, nbits, (idx.numel(),), device=device, generator=g)
        byte = lo_byte + bit // 8
        mask = (1 << (bit % 8)).to(torch.uint8)
        t[idx, byte] ^= mask

    flip(sigs, cats["r_bitflip"], 0, 256)
    flip(sigs, cats["s_bitflip"], 32, 253)
    flip(msgs, cats["msg_bitflip"], 0, 256)
    wk = cats["wrong_key"]
    pubs[wk] = orig_pubs[(wk + 1) % n]
    # S + kL (k random in [1, kmax]); includes S >= 2^255 lanes where slide() may drop a carry
    sk = cats["s_plus_kL"]
    if sk.numel():
        s_host = sigs[sk, 32:].cpu().numpy()
        rng = np.random.default_rng(seed ^ 0x5EED)
        out = np.empty_like(s_host)
        for j in range(s_host.shape[0]):
            S = int.from_bytes(s_host[j].tobytes(), "little")
            kmax = (2**256 - 1 - S) // L
            S2 = S + int(rng.integers(1, kmax + 1)) * L
            out[j] = np.frombuffer(S2.to_bytes(32, "little"), np.uint8)
        sigs[sk, 32:] = torch.from_numpy(out).to(device)
    for name, table, col in (("r_noncanonical", NONCANONICAL_R, "sig"), ("key_noncanonical", NONCANONICAL_KEYS, "key"),
                             ("key_off_curve", OFF_CURVE_KEYS, "key"), ("key_small_order", SMALL_ORDER_KEYS, "key")):
        idx = cats[name]
        if not idx.numel():
            continue
        c = _consts(table, torch, device)
        pick = torch.randint(0, c.shape[0], (idx.numel(),), device=device, generator=g)
        if col == "sig":
            sigs[idx, :32] = c[pick]
        else:
            pubs[idx] = c[pick]
    for name, idx in cats.items():
        e = C2_EXPECTED[name]
        expected[idx] = -1 if e is None else e
    return expected, cats
