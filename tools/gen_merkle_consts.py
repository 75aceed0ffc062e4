#!/usr/bin/env python3
"""Constants of the Merkle node hash (corda_amd/csrc/tx.hip): K[i] + W[i] for the
constant second SHA-256 block of a 64-byte message, and the zero-tree roots
Z_j (Z_0 = 32 zero bytes, Z_{j+1} = SHA-256(Z_j || Z_j), MerkleTree.kt:33-41).
Prints the two C initialiser bodies (kPadKW, then kZeroHash) separated by a
line holding '--'. (dev tool)"""
import hashlib
import struct

K = [0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
     0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
     0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
     0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
     0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
     0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
     0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
     0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
M = 0xffffffff


def ror(x, n):
    return ((x >> n) | (x << (32 - n))) & M


def pad_kw():
    w = [0x80000000] + [0] * 14 + [512]
    for i in range(16, 64):
        s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3)
        s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10)
        w.append((w[i - 16] + s0 + w[i - 7] + s1) & M)
    return [(K[i] + w[i]) & M for i in range(64)]


def zero_roots(n=64):
    z, out = bytes(32), []
    for _ in range(n):
        out.append(struct.unpack(">8I", z))
        z = hashlib.sha256(z + z).digest()
    return out


def main():
    kw = pad_kw()
    print("\n".join("    " + ", ".join("0x%08x" % x for x in kw[i:i + 8]) + "," for i in range(0, 64, 8)))
    print("--")
    print("\n".join("    {" + ", ".join("0x%08x" % x for x in z) + "}," for z in zero_roots()))


if __name__ == "__main__":
    main()
