// BLAKE2b-256 (RFC 7693, unkeyed, 32-byte digest), one message per lane, and
// the BDLS SignedProto.Hash framing:
//   vendor/github.com/BDLS-bft/bdls/message.go:97-138
//   H = BLAKE2b-256("BDLS_CONSENSUS_SIGNATURE" || Version (u32 LE) || X (32 B)
//                   || Y (32 B) || len(Message) (u32 LE) || Message)
// Replaces vendor/github.com/BDLS-bft/bdls/crypto/blake2b (Go + AVX2 asm) on
// the consensus-message verify path.
#pragma once
#include "bh_common.h"

namespace bh {

#if defined(__HIPCC__)
__device__ __constant__ static const uint64_t kB2IV[8] = {
#else
static const uint64_t kB2IV[8] = {
#endif
    0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
    0x510e527fade682d1ull, 0x9b05688c2b3e6c1full, 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

// Message schedule. Used only with compile-time indices (the round loop
// below is fully unrolled), so every m[] access folds to a register.
struct B2Sigma {
  static constexpr uint8_t s[12][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
      {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
      {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
      {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
      {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
};

BH_HD uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

BH_HD void b2_g(uint64_t v[16], int a, int b, int c, int d, uint64_t x, uint64_t y) {
  v[a] = v[a] + v[b] + x;
  v[d] = rotr64(v[d] ^ v[a], 32);
  v[c] = v[c] + v[d];
  v[b] = rotr64(v[b] ^ v[c], 24);
  v[a] = v[a] + v[b] + y;
  v[d] = rotr64(v[d] ^ v[a], 16);
  v[c] = v[c] + v[d];
  v[b] = rotr64(v[b] ^ v[c], 63);
}

// m: the block as 32 little-endian u32 words.
BH_HD void b2_compress(uint64_t h[8], const uint32_t mw[32], uint64_t t, bool last) {
  uint64_t m[16], v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = (uint64_t)mw[2 * i] | ((uint64_t)mw[2 * i + 1] << 32);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = kB2IV[i];
  }
  v[12] ^= t;  // byte counter (messages < 2^64 bytes: high word stays 0)
  if (last) v[14] = ~v[14];
#pragma unroll
  for (int r = 0; r < 12; r++) {
    b2_g(v, 0, 4, 8, 12, m[B2Sigma::s[r][0]], m[B2Sigma::s[r][1]]);
    b2_g(v, 1, 5, 9, 13, m[B2Sigma::s[r][2]], m[B2Sigma::s[r][3]]);
    b2_g(v, 2, 6, 10, 14, m[B2Sigma::s[r][4]], m[B2Sigma::s[r][5]]);
    b2_g(v, 3, 7, 11, 15, m[B2Sigma::s[r][6]], m[B2Sigma::s[r][7]]);
    b2_g(v, 0, 5, 10, 15, m[B2Sigma::s[r][8]], m[B2Sigma::s[r][9]]);
    b2_g(v, 1, 6, 11, 12, m[B2Sigma::s[r][10]], m[B2Sigma::s[r][11]]);
    b2_g(v, 2, 7, 8, 13, m[B2Sigma::s[r][12]], m[B2Sigma::s[r][13]]);
    b2_g(v, 3, 4, 9, 14, m[B2Sigma::s[r][14]], m[B2Sigma::s[r][15]]);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

constexpr uint32_t kBdlsHeader = 96;  // prefix 24 + version 4 + X 32 + Y 32 + len 4

// Little-endian word at byte q (multiple of 4) of msg[0..mlen), zero-padded
// past the end (bytes loaded one at a time only for the straddling word).
BH_HD uint32_t b2_tail_word(const uint8_t* msg, uint32_t mlen, uint32_t q) {
  if (q + 4 <= mlen) {
    return (uint32_t)msg[q] | ((uint32_t)msg[q + 1] << 8) | ((uint32_t)msg[q + 2] << 16) |
           ((uint32_t)msg[q + 3] << 24);
  }
  uint32_t v = 0;
  for (uint32_t b = 0; b < 4; b++)
    if (q + b < mlen) v |= (uint32_t)msg[q + b] << (8 * b);
  return v;
}

// out[0..31] = SignedProto.Hash() for (version, X, Y, msg[0..mlen)).
// Stream = header (96 B, 24 words built in registers) || msg. Block 0 holds
// the header and msg[0..32); block k >= 1 holds msg[128 k - 96, 128 k + 32).
// Every block but the last is read with dword loads + funnel shifts.
BH_HD void bdls_signed_proto_hash(uint8_t out[32], uint32_t version, const uint8_t* x32,
                                  const uint8_t* y32, const uint8_t* msg, uint32_t mlen) {
  uint32_t blk[32];
  // "BDLS_CONSENSUS_SIGNATURE" as little-endian words
  blk[0] = 0x534c4442u;  // "BDLS"
  blk[1] = 0x4e4f435fu;  // "_CON"
  blk[2] = 0x534e4553u;  // "SENS"
  blk[3] = 0x535f5355u;  // "US_S"
  blk[4] = 0x414e4749u;  // "IGNA"
  blk[5] = 0x45525554u;  // "TURE"
  blk[6] = version;
  load_le_words<8>(blk + 7, x32);
  load_le_words<8>(blk + 15, y32);
  blk[23] = mlen;

  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = kB2IV[i];
  h[0] ^= 0x01010000ull ^ 32ull;  // digest length 32, no key
  const uint64_t total = kBdlsHeader + (uint64_t)mlen;
  for (uint64_t pos = 0;; pos += 128) {  // one compression call site
    const bool last = total - pos <= 128;
    if (pos == 0) {
      if (!last) {
        load_le_words<8>(blk + 24, msg);
      } else {
#pragma unroll
        for (int i = 0; i < 8; i++) blk[24 + i] = b2_tail_word(msg, mlen, 4u * i);
      }
    } else {
      const uint32_t q = (uint32_t)(pos - kBdlsHeader);
      if (!last) {
        load_le_words<32>(blk, msg + q);
      } else {
        for (int i = 0; i < 32; i++) blk[i] = b2_tail_word(msg, mlen, q + 4u * i);
      }
    }
    b2_compress(h, blk, last ? total : pos + 128, last);
    if (last) break;
  }
#pragma unroll
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(h[i >> 3] >> (8 * (i & 7)));
}

}  // namespace bh
