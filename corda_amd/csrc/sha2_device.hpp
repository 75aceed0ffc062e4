// SHA-256 / SHA-512 compression functions for gfx950 lanes (FIPS 180-4).
// One lane hashes one message; blocks are assembled in registers by the
// caller (the hot shapes are single-block: Ed25519's R||A||txId is 96 bytes,
// a Merkle node is SHA-256 of 64 bytes = 2 blocks, the 2nd constant).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef CDEV
#define CDEV __device__ __forceinline__
#endif

namespace cordahip {

__device__ __constant__ static const uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

__device__ __constant__ static const uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

CDEV uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
CDEV uint32_t ror32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
CDEV uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

CDEV void sha512_init(uint64_t h[8]) {
  h[0] = 0x6a09e667f3bcc908ULL; h[1] = 0xbb67ae8584caa73bULL;
  h[2] = 0x3c6ef372fe94f82bULL; h[3] = 0xa54ff53a5f1d36f1ULL;
  h[4] = 0x510e527fade682d1ULL; h[5] = 0x9b05688c2b3e6c1fULL;
  h[6] = 0x1f83d9abfb41bd6bULL; h[7] = 0x5be0cd19137e2179ULL;
}

// w[16]: the block as big-endian 64-bit words (clobbered)
CDEV void sha512_block(uint64_t h[8], uint64_t w[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 80; i++) {
    uint64_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint64_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint64_t s0 = ror64(w15, 1) ^ ror64(w15, 8) ^ (w15 >> 7);
      const uint64_t s1 = ror64(w2, 19) ^ ror64(w2, 61) ^ (w2 >> 6);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint64_t t1 = hh + (ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41)) + ((e & f) ^ (~e & g)) + kSha512K[i] + wi;
    const uint64_t t2 = (ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

CDEV void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
  h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
}

// w[16]: the block as big-endian 32-bit words (clobbered)
CDEV void sha256_block(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = ror32(w15, 7) ^ ror32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = ror32(w2, 17) ^ ror32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t t1 = hh + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + kSha256K[i] + wi;
    const uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// big-endian word at byte pos of the SHA-256-padded message p[0..len)
CDEV uint32_t sha256_padded_word(const uint8_t* __restrict__ p, uint64_t len, uint64_t pos, uint64_t total_bits,
                                 uint64_t padded_len) {
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t q = pos + k;
    uint32_t b;
    if (q < len) b = p[q];
    else if (q == len) b = 0x80;
    else if (q >= padded_len - 8) b = (uint32_t)((total_bits >> (8 * (padded_len - 1 - q))) & 0xff);
    else b = 0;
    w = (w << 8) | b;
  }
  return w;
}

// SHA-256 of an arbitrary byte string in global memory (one lane).
// Leaves sit at arbitrary byte offsets (CSR), so each 64-byte block is read as
// 17 ALIGNED dwords (only those holding at least one message byte: an aligned
// dword around a valid byte never crosses a page) and re-aligned with a funnel
// shift + byte swap: 17 loads and ~2 ALU ops per word instead of 64 byte loads
// and 3 ops per byte. FIPS 180-4 padding is applied per word in registers.
CDEV void sha256_bytes(uint32_t h[8], const uint8_t* __restrict__ p, uint64_t len) {
  sha256_init(h);
  const uint64_t padded = ((len + 9 + 63) / 64) * 64;
  const uint64_t bits = len * 8;
  const uint32_t a = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
  const uint32_t* __restrict__ wp = reinterpret_cast<const uint32_t*>(p - a);  // aligned
  const uint32_t sh = 8u * a;
  uint32_t w[16];
  for (uint64_t blk = 0; blk < padded; blk += 64) {
    // dword k of this block covers message bytes [blk - a + 4k, blk - a + 4k + 4)
    uint32_t d[17];
    const uint64_t d0 = blk >> 2;
    if (blk + 64 + 4 <= len + a) {  // all 17 dwords hold message bytes
#pragma unroll
      for (int k = 0; k < 17; k++) d[k] = wp[d0 + k];
    } else {
#pragma unroll
      for (int k = 0; k < 17; k++) d[k] = (blk + 4 * k < len + a) ? wp[d0 + k] : 0u;
    }
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const uint32_t le = (uint32_t)(((((uint64_t)d[q + 1]) << 32) | d[q]) >> sh);  // bytes pos..pos+3
      w[q] = __builtin_bswap32(le);
    }
    if (blk + 64 > len) {  // block holds the end of the message: mask, 0x80, length
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const uint64_t pos = blk + 4 * q;
        if (pos + 4 > len) {
          const uint32_t nv = pos < len ? (uint32_t)(len - pos) : 0u;  // 0..3 valid bytes
          const uint32_t keep = nv ? ~0u << (32 - 8 * nv) : 0u;
          w[q] = (w[q] & keep) | (pos <= len ? 0x80000000u >> (8 * nv) : 0u);
        }
      }
      if (blk + 64 == padded) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
      }
    }
    sha256_block(h, w);
  }
}

}  // namespace cordahip
