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


# ---- C3: mixed secp256k1 / P-256 ECDSA --------------------------------------
N_K1 = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
N_R1 = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
CURVE_N = {2: N_K1, 3: N_R1}
REJECT_ANY = -2  # expected "some rejection status" (exact status decided by the oracle in tests)

# C3 mix (fractions of the corrupted lanes), SURVEY §8(d)
C3_MIX = [("sig_bitflip", 0.30), ("msg_bitflip", 0.10), ("wrong_key", 0.10), ("key_off_curve", 0.10),
          ("r_zero", 0.05), ("s_zero", 0.05), ("r_ge_n", 0.05), ("s_ge_n", 0.05), ("der_trailing", 0.05),
          ("der_wrong_tag", 0.05), ("der_nonminimal", 0.05), ("der_long_len", 0.05)]
C3_EXPECTED = {"sig_bitflip": REJECT_ANY, "msg_bitflip": 1, "wrong_key": 1, "key_off_curve": 3, "r_zero": 1,
               "s_zero": 1, "r_ge_n": 1, "s_ge_n": 1, "der_trailing": 2, "der_wrong_tag": 2, "der_nonminimal": 2,
               "der_long_len": 2}
C3_COMPRESSED_FRAC = 0.10  # valid lanes re-encoded as 33-byte compressed keys (must still accept)


def der_ints(sig: bytes):
    """(r, s) of a minimal DER SEQUENCE{INTEGER r, INTEGER s} as written by the device signer."""
    lr = sig[3]
    r = int.from_bytes(sig[4:4 + lr], "big")
    ls = sig[5 + lr]
    return r, int.from_bytes(sig[6 + lr:6 + lr + ls], "big")


def _der_int(v: int, extra_zero: bool = False) -> bytes:
    b = v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big")
    if b[0] & 0x80:
        b = b"\x00" + b
    if extra_zero:
        b = b"\x00" + b
    return b"\x02" + bytes([len(b)]) + b


def der_sig(r: int, s: int, nonminimal_r: bool = False, long_len: bool = False) -> bytes:
    body = _der_int(r, nonminimal_r) + _der_int(s)
    return b"\x30" + (b"\x81" if long_len else b"") + bytes([len(body)]) + body


def make_c3_corpus(engine, n: int, seed: int, device, corrupt_frac: float = 0.01, stream=None, dev_index: int = 0):
    """Returns (scheme[n], keys[n,65], key_len[n], sigs[n,72], sig_len[n], msgs[n,32], expected[n] int16, cats).
    Schemes alternate secp256k1 / P-256 lane by lane; keys and sigs are made by the device signer."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    scheme = (2 + (torch.arange(n, device=device) & 1)).to(torch.uint8)
    seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=device, generator=g)
    msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=device, generator=g)
    keys = torch.zeros((n, 65), dtype=torch.uint8, device=device)
    key_len = torch.zeros(n, dtype=torch.uint8, device=device)
    sigs = torch.zeros((n, 72), dtype=torch.uint8, device=device)
    sig_len = torch.zeros(n, dtype=torch.uint8, device=device)
    engine.ecdsa_sign_device(scheme, seeds, msgs, keys, key_len, sigs, sig_len, device=dev_index, stream=stream)
    torch.cuda.synchronize(device)
    del seeds
    expected, cats = corrupt_c3(scheme, keys, key_len, sigs, sig_len, msgs, seed, g, corrupt_frac)
    torch.cuda.synchronize(device)
    return scheme, keys, key_len, sigs, sig_len, msgs, expected, cats


def corrupt_c3(scheme, keys, key_len, sigs, sig_len, msgs, seed: int, g, corrupt_frac: float = 0.01):
    """Apply the C3 catalogue in place (CPU or GPU tensors); then compress a share of the untouched keys."""
    import torch

    n, device = keys.shape[0], keys.device
    expected = torch.zeros(n, dtype=torch.int16, device=device)
    ncor = int(n * corrupt_frac)
    perm = torch.randperm(n, device=device, generator=g)
    cor = perm[:ncor]
    cats: Dict[str, torch.Tensor] = {}
    start = 0
    for i, (name, frac) in enumerate(C3_MIX):
        cnt = ncor - start if i == len(C3_MIX) - 1 else int(round(ncor * frac))
        cats[name] = cor[start:start + cnt]
        start += cnt
    orig_keys = keys.clone()

    idx = cats["sig_bitflip"]
    if idx.numel():
        ln = sig_len[idx].to(torch.int64)
        bit = (torch.rand(idx.numel(), device=device, generator=g) * (ln * 8).to(torch.float32)).to(torch.int64)
        bit = torch.minimum(bit, ln * 8 - 1)
        sigs[idx, bit // 8] ^= (1 << (bit % 8)).to(torch.uint8)
    idx = cats["msg_bitflip"]
    if idx.numel():
        bit = torch.randint(0, 256, (idx.numel(),), device=device, generator=g)
        msgs[idx, bit // 8] ^= (1 << (bit % 8)).to(torch.uint8)
    idx = cats["wrong_key"]  # lane +- 2 has the same curve (schemes alternate)
    keys[idx] = orig_keys[(idx + 2) % n if n > 2 else idx]
    idx = cats["key_off_curve"]
    if idx.numel():
        bit = torch.randint(0, 256, (idx.numel(),), device=device, generator=g)
        keys[idx, 33 + bit // 8] ^= (1 << (bit % 8)).to(torch.uint8)

    # DER / range edits: re-encoded on the host (a few hundred lanes per 2^24)
    edit = [nm for nm in ("r_zero", "s_zero", "r_ge_n", "s_ge_n", "der_trailing", "der_wrong_tag",
                          "der_nonminimal", "der_long_len") if cats[nm].numel()]
    if edit:
        all_idx = torch.cat([cats[nm] for nm in edit])
        S = sigs[all_idx].cpu().numpy()
        SL = sig_len[all_idx].cpu().numpy()
        SC = scheme[all_idx].cpu().numpy()
        outS, outL, pos = S.copy(), SL.copy(), 0
        for nm in edit:
            for _ in range(cats[nm].numel()):
                sig = S[pos, :SL[pos]].tobytes()
                r, s = der_ints(sig)
                nn = CURVE_N[int(SC[pos])]
                if nm == "r_zero":
                    new = der_sig(0, s)
                elif nm == "s_zero":
                    new = der_sig(r, 0)
                elif nm == "r_ge_n":
                    new = der_sig(r + nn if r + nn < 2**256 else nn, s)
                elif nm == "s_ge_n":
                    new = der_sig(r, s + nn if s + nn < 2**256 else nn)
                elif nm == "der_trailing":
                    new = sig + b"\x00" if len(sig) < 72 else b"\x31" + sig[1:]
                elif nm == "der_wrong_tag":
                    new = b"\x31" + sig[1:]
                elif nm == "der_nonminimal":
                    new = der_sig(r, s, nonminimal_r=True)
                    if len(new) > 72:
                        new = b"\x30" + sig[1:2] + b"\x03" + sig[3:]  # INTEGER tag -> BIT STRING
                else:  # der_long_len: sequence length in long form (BER, not DER)
                    new = der_sig(r, s, long_len=True)
                    if len(new) > 72:
                        new = b"\x30\x81" + sig[1:-1]  # long form, body truncated by one byte
                outS[pos] = 0
                outS[pos, :len(new)] = np.frombuffer(new, np.uint8)
                outL[pos] = len(new)
                pos += 1
        sigs[all_idx] = torch.from_numpy(outS).to(device)
        sig_len[all_idx] = torch.from_numpy(outL).to(device)

    for name, idx in cats.items():
        expected[idx] = C3_EXPECTED[name]
    # compressed keys on a share of the valid lanes: 02/03 || X
    ncomp = int((n - ncor) * C3_COMPRESSED_FRAC)
    comp = perm[ncor:ncor + ncomp]
    if comp.numel():
        keys[comp, 0] = 2 + (keys[comp, 64] & 1)
        keys[comp, 33:] = 0
        key_len[comp] = 33
    cats["compressed_valid"] = comp
    return expected, cats


# ---- C4 with native Kryo leaves ------------------------------------
# The five components of a cash-issue WireTransaction in availableComponents
# order (MerkleTransaction.kt:51-62; CashIssueFlow.kt:52-54): the
# TransactionState<Cash.State> output, the issue Command, the notary Party, the
# mustSign key, TransactionType.General -- written by cordahip_kryo_encode, no JVM.
KRYO_IDS = {"ed25519_key": 45, "x500_name": 52, "arrays_as_list": 10}  # registration ids on the node (parameters)
TRANSACTION_TYPE_GENERAL = "net.corda.core.contracts.TransactionType$General"  # TransactionTypes.kt:64
CASH_ISSUE_COMMAND = "net.corda.contracts.asset.Cash$Commands$Issue"  # Cash.kt:148


def _der(tag: int, body: bytes) -> bytes:
    n = len(body)
    if n < 128:
        return bytes([tag, n]) + body
    nb = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([tag, 0x80 | len(nb)]) + nb + body


def x500_name(org: str, locality: str, country: str) -> bytes:
    """DER of O=<org>, L=<locality>, C=<country> (UTF8String / PrintableString values)."""
    out = b""
    for oid, val, tag in ((b"\x55\x04\x0a", org, 0x0C), (b"\x55\x04\x07", locality, 0x0C), (b"\x55\x04\x06", country, 0x13)):
        out += _der(0x31, _der(0x30, _der(0x06, oid) + _der(tag, val.encode())))
    return _der(0x30, out)


def cash_issue_items(issuer_keys: np.ndarray, owner_keys: np.ndarray, notary_key: bytes, quantities: np.ndarray,
                     nonces: np.ndarray):
    """The five cordahip_kryo_items of each of ntx cash-issue transactions (TransactionState<Cash.State>,
    the issue Command, the notary Party, the mustSign key, TransactionType.General) with their payloads
    in ONE byte blob: returns (blob uint8, items KRYO_ITEM_DTYPE[ntx, 5]) whose `data` fields are
    OFFSETS into the blob (add the blob's address -- host or device -- before encoding), and the
    blob layout of the owner keys ({"owner_key": tx 0's offset, "cash_stride": bytes per tx}). The blob
    is tx-major: the shared payloads, then each transaction's cash state, command and key.
    issuer_keys[t] (Ed25519 A) issues quantities[t] USD cents (issue reference 01) to the anonymised
    owner_keys[t] (an AnonymousParty, as CashIssueFlow's default confidential recipient), notary
    "Notary Service, Zurich, CH"; the command signer and mustSign key = the issuer key."""
    from corda_amd import _lib
    ntx = len(issuer_keys)
    ik = np.ascontiguousarray(issuer_keys, np.uint8).reshape(ntx, 32)
    ok = np.ascontiguousarray(owner_keys, np.uint8).reshape(ntx, 32)
    bank = x500_name("Bank A", "London", "GB")
    notary = x500_name("Notary Service", "Zurich", "CH")
    legal = __import__("hashlib").sha256(b"https://www.big-book-of-banking-law.gov/cash-claims.html").digest()
    ed = KRYO_IDS["ed25519_key"]
    mark_i, mark_o = b"\xa5" * 32, b"\x5a" * 32
    cash_t = np.frombuffer(_lib.pack_cash_state(
        {"issuer": (bank, mark_i, ed), "reference": b"\x01", "owner": (b"", mark_o, ed), "notary": (notary, notary_key, ed),
         "currency": "USD", "digits": 2, "legal_ref": legal, "encumbrance": None}), np.uint8)
    nm = CASH_ISSUE_COMMAND.encode()
    cmd_t = np.frombuffer(bytes([len(nm)]) + nm + bytes([1]) + ed.to_bytes(2, "little") + (32).to_bytes(2, "little")
                          + mark_i, np.uint8)
    oi = bytes(cash_t).index(mark_i)
    oo = bytes(cash_t).index(mark_o)
    oc = bytes(cmd_t).index(mark_i)
    cash = np.tile(cash_t, (ntx, 1))
    cash[:, oi:oi + 32] = ik
    cash[:, oo:oo + 32] = ok
    cmd = np.tile(cmd_t, (ntx, 1))
    cmd[:, oc:oc + 32] = ik
    party = np.frombuffer(notary + bytes(notary_key), np.uint8)
    gen = np.frombuffer(TRANSACTION_TYPE_GENERAL.encode("utf-16-le"), np.uint8)
    # tx-major, as a JVM writing one transaction's components after another would: the shared
    # payloads (the notary Party, the TransactionType name) first, then per transaction its
    # cash state, command and key -- every id slice's components then lie in one prefix of the
    # blob (what cordahip_txcomp_submit copies ahead of each slice)
    shared = np.concatenate([party, gen])
    rec = np.concatenate([cash, cmd, ik], axis=1)
    stride = rec.shape[1]
    blob = np.concatenate([shared, rec.reshape(-1)])
    items = np.zeros((ntx, 5), _lib.KRYO_ITEM_DTYPE)
    kinds = [_lib.KRYO_KINDS[k] for k in ("cash_state", "issue_command", "party", "ed25519_key", "kotlin_object")]
    items["kind"] = kinds
    items["class_id"] = [KRYO_IDS["x500_name"], KRYO_IDS["arrays_as_list"], KRYO_IDS["x500_name"], ed, 0]
    items["value"][:, 0] = quantities
    items["value"][:, 1] = nonces
    items["value"][:, 2] = ed  # the notary key's class
    t0 = shared.size + np.arange(ntx, dtype=np.uint64) * stride
    items["data"][:, 0] = t0
    items["len"][:, 0] = cash.shape[1]
    items["data"][:, 1] = t0 + cash.shape[1]
    items["len"][:, 1] = cmd.shape[1]
    items["data"][:, 2] = 0
    items["len"][:, 2] = party.size
    items["data"][:, 3] = t0 + cash.shape[1] + cmd.shape[1]
    items["len"][:, 3] = 32
    items["data"][:, 4] = party.size
    items["len"][:, 4] = gen.size // 2
    # where transaction t's owner key sits in the blob (bench corruption: a flipped
    # key byte changes the output leaf and so the id, as a flipped leaf byte does)
    layout = {"owner_key": shared.size + oo, "cash_stride": stride}
    return blob, items, layout


def make_cash_issue_leaves(issuer_keys: np.ndarray, owner_keys: np.ndarray, notary_key: bytes,
                           quantities: np.ndarray, nonces: np.ndarray, threads: int = 8):
    """CSR leaf bytes of the ntx cash-issue transactions of cash_issue_items, encoded on the host
    (cordahip_kryo_encode, `threads` at a time). Returns (leaf_bytes uint8, leaf_off uint64[5 * ntx + 1])."""
    from concurrent.futures import ThreadPoolExecutor

    from corda_amd import _lib
    ntx = len(issuer_keys)
    blob, items, _ = cash_issue_items(issuer_keys, owner_keys, notary_key, quantities, nonces)
    items["data"] += np.uint64(blob.ctypes.data)
    flat = items.reshape(-1)
    per = max(1, -(-ntx // (threads * 4)))
    parts = [(a * 5, min(ntx, a + per) * 5) for a in range(0, ntx, per)]
    with ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(lambda r: _lib.kryo_encode_array(flat[r[0]:r[1]]), parts))
    out = np.concatenate([b for b, _ in outs]) if outs else np.zeros(0, np.uint8)
    off = np.zeros(5 * ntx + 1, np.uint64)
    base = 0
    for (a, b), (bb, oo_) in zip(parts, outs):
        off[a + 1:b + 1] = oo_[1:] + base
        base += len(bb)
    del blob  # the encoder copied everything
    return out, off
