"""Benchmark corpora (corda_amd/corpus.py) on the CPU: the corruption catalogue's
expected statuses must be what the oracle says, so bench.py's construction
check is meaningful. The GPU signers are replaced here by the oracle signers
with the same key/nonce derivation."""
import hashlib

import numpy as np
import torch

from corda_amd import corpus


def _c3_rows(n, seed):
    import bc_ecdsa as ec
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    scheme = (2 + (np.arange(n) & 1)).astype(np.uint8)
    keys = np.zeros((n, 65), np.uint8)
    sigs = np.zeros((n, 72), np.uint8)
    sl = np.zeros(n, np.uint8)
    for i in range(n):
        c = ec.CURVES[int(scheme[i])]
        d = int.from_bytes(hashlib.sha256(seeds[i].tobytes()).digest(), "big") % c.n or 1
        k = int.from_bytes(hashlib.sha256(seeds[i].tobytes() + msgs[i].tobytes()).digest(), "big") % c.n or 1
        keys[i] = np.frombuffer(ec.keypair(int(scheme[i]), d), np.uint8)
        sig = ec.der_encode(*ec.sign(int(scheme[i]), d, msgs[i].tobytes(), k))
        sigs[i, :len(sig)] = np.frombuffer(sig, np.uint8)
        sl[i] = len(sig)
    t = torch.from_numpy
    return t(scheme), t(keys), t(np.full(n, 65, np.uint8)), t(sigs), t(sl), t(msgs)


def test_c3_catalogue_matches_oracle(oracle):
    n = 320
    scheme, keys, kl, sigs, sl, msgs = _c3_rows(n, 3)
    for i in range(n):  # the oracle signer's DER matches the device signer's minimal form
        r, s = corpus.der_ints(sigs[i, :sl[i]].numpy().tobytes())
        assert corpus.der_sig(r, s) == sigs[i, :sl[i]].numpy().tobytes()
    g = torch.Generator()
    g.manual_seed(7)
    expected, cats = corpus.corrupt_c3(scheme, keys, kl, sigs, sl, msgs, 7, g, corrupt_frac=0.5)
    assert all(cats[nm].numel() > 0 for nm, _ in corpus.C3_MIX)
    assert cats["compressed_valid"].numel() > 0
    got = np.array([oracle.oracle_ecdsa_verify(int(scheme[i]), keys[i, :kl[i]].numpy().tobytes(), int(kl[i]),
                                               sigs[i, :sl[i]].numpy().tobytes(), int(sl[i]),
                                               msgs[i].numpy().tobytes(), 32) for i in range(n)])
    exp = expected.numpy()
    exact = exp >= 0
    assert np.array_equal(got[exact], exp[exact]), [(i, got[i], exp[i]) for i in np.where(exact & (got != exp))[0]]
    assert (got[exp == corpus.REJECT_ANY] != 0).all()
    assert (got[cats["compressed_valid"].numpy()] == 0).all()
