"""CPU model of the Ed25519 prep's lattice reduction (ed25519.hip
half_scalars): Lehmer rounds over 52-bit leading parts in doubles must hand
over exactly the plain Euclid state (same quotients, same stopping point)."""
import importlib.util
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("lehmer", os.path.join(ROOT, "tools", "proto", "lehmer.py"))
lehmer = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(lehmer)


def test_lehmer_hands_over_euclid_state():
    rng = random.Random(11)
    L, T = lehmer.L, lehmer.T
    hs = [0, 1, 2, 3, L - 1, L - 2, T - 1, T, T + 1, 2 * T, (1 << 252) - 1, 1 << 200, (1 << 128) + 1]
    hs += [rng.randrange(L) for _ in range(3000)]
    stats = {}
    for h in hs:
        *ref, _ = lehmer.euclid_state(h)
        assert tuple(lehmer.lehmer_state(h, stats)) == tuple(ref), h
    assert stats["max_finish"] <= 3 and stats["max_rounds"] <= 8
