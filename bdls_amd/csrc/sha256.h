// SHA-256 (FIPS 180-4), one message per lane, message bytes read straight
// from HBM. Replaces bccsp/sw/hash.go:29-33 (Go crypto/sha256, SHA-NI asm) as
// reached from msp/identities.go:179 (identity.Verify hashes the message with
// the SHA2 family before CSP.Verify).
#pragma once
#include "bh_common.h"

namespace bh {

#if defined(__HIPCC__)
__device__ __constant__ static const uint32_t kSha256K[64] = {
#else
static const uint32_t kSha256K[64] = {
#endif
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

BH_HD uint32_t rotr32(uint32_t x, uint32_t n) { return (x >> n) | (x << (32 - n)); }

// The round's operations in the forms CDNA4 issues in one instruction each:
// a rotation is v_alignbit_b32, a three-way xor one v_bitop3_b32 (truth table
// 0x96; the compiler forms bitop3 for Ch / Maj but not for these sums), Ch a
// v_bfi_b32. Host builds (the CPU harness) take the plain expressions.
BH_HD uint32_t sha_rotr(uint32_t x, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(x, x, n);
#else
  return rotr32(x, n);
#endif
}
BH_HD uint32_t sha_xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return a ^ b ^ c;
#endif
}

// one round; wk = W[t] + K[t]
BH_HD void sha256_round(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                        uint32_t& f, uint32_t& g, uint32_t& hh, uint32_t wk) {
  const uint32_t S1 = sha_xor3(sha_rotr(e, 6), sha_rotr(e, 11), sha_rotr(e, 25));
  const uint32_t ch = g ^ (e & (f ^ g));
  const uint32_t t1 = (hh + wk) + S1 + ch;
  const uint32_t S0 = sha_xor3(sha_rotr(a, 2), sha_rotr(a, 13), sha_rotr(a, 22));
  const uint32_t mj = (a & b) | (c & (a | b));
  hh = g;
  g = f;
  f = e;
  e = d + t1;
  d = c;
  c = b;
  b = a;
  a = t1 + S0 + mj;
}

// schedule word t >= 16 into the 16-word ring
BH_HD uint32_t sha256_sched(uint32_t w[16], int i) {
  const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
  const uint32_t s0 = sha_xor3(sha_rotr(w15, 7), sha_rotr(w15, 18), w15 >> 3);
  const uint32_t s1 = sha_xor3(sha_rotr(w2, 17), sha_rotr(w2, 19), w2 >> 10);
  const uint32_t wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
  w[i & 15] = wi;
  return wi;
}

BH_HD void sha256_block(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const uint32_t wi = i < 16 ? w[i] : sha256_sched(w, i);
    sha256_round(a, b, c, d, e, f, g, hh, wi + kSha256K[i]);
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// Big-endian 32-bit word at message byte position pos of a padded stream:
// bytes [0, len) are the message, then 0x80, zeros, 64-bit bit length.
BH_HD uint32_t sha256_word(const uint8_t* m, uint64_t len, uint64_t total, uint64_t pos) {
  // fast path: the word lies fully inside the message
  if (pos + 4 <= len) {
    return ((uint32_t)m[pos] << 24) | ((uint32_t)m[pos + 1] << 16) | ((uint32_t)m[pos + 2] << 8) |
           (uint32_t)m[pos + 3];
  }
  uint32_t w = 0;
  const uint64_t bits = len * 8;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint64_t p = pos + k;
    uint32_t byte;
    if (p < len) byte = m[p];
    else if (p == len) byte = 0x80u;
    else if (p >= total - 8) byte = (uint32_t)(bits >> (8 * (total - 1 - p))) & 0xffu;
    else byte = 0;
    w = (w << 8) | byte;
  }
  return w;
}

// out = SHA-256(m[0..len)) as 8 big-endian words (out[0] = most significant).
BH_HD void sha256_msg(uint32_t out[8], const uint8_t* m, uint64_t len) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t total = ((len + 9 + 63) / 64) * 64;
  for (uint64_t blk = 0; blk < total; blk += 64) {
    uint32_t w[16];
    if (blk + 64 <= len) {  // full message block, any alignment
      load_le_words<16>(w, m + blk);
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = bswap32(w[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = sha256_word(m, len, total, blk + 4 * i);
    }
    sha256_block(h, w);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = h[i];
}

// ---- two-span messages: m1[0, l1) || m2[0, l2) hashed as one message (a
// Fabric SignedData prp || endorser, validator_keylevel.go:246-260, without a
// host-side concatenation). Blocks inside one span load as above; only the
// block straddling the seam and the padding go byte by byte.
BH_HD uint32_t msg2_byte(const uint8_t* m1, uint64_t l1, const uint8_t* m2, uint64_t p) {
  return p < l1 ? m1[p] : m2[p - l1];
}

BH_HD uint32_t sha256_word2(const uint8_t* m1, uint64_t l1, const uint8_t* m2, uint64_t len,
                            uint64_t total, uint64_t pos) {
  uint32_t w = 0;
  const uint64_t bits = len * 8;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t p = pos + k;
    uint32_t byte;
    if (p < len) byte = msg2_byte(m1, l1, m2, p);
    else if (p == len) byte = 0x80u;
    else if (p >= total - 8) byte = (uint32_t)(bits >> (8 * (total - 1 - p))) & 0xffu;
    else byte = 0;
    w = (w << 8) | byte;
  }
  return w;
}

// ---- split compression (round 5): the message schedule of a block depends on
// the block alone, so it can be expanded by other lanes ahead of the serial
// chain of rounds (k_digest_grp). sched: wk[t] = W[t] + K[t], t < 64;
// rounds: the 64 rounds over a precomputed wk. sha256_rounds_wk(h,
// sha256_sched_wk(w)) == sha256_block(h, w).
BH_HD void sha256_sched_wk(uint32_t wk[64], uint32_t w[16]) {
#pragma unroll
  for (int i = 0; i < 64; i++) wk[i] = (i < 16 ? w[i] : sha256_sched(w, i)) + kSha256K[i];
}

BH_HD void sha256_rounds_wk(uint32_t h[8], const uint32_t wk[64]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) sha256_round(a, b, c, d, e, f, g, hh, wk[i]);
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// The 16 big-endian words of padded block blk (byte offset) of the two-span
// message m1[0, l1) || m2[0, len - l1) (one span: l1 = len, m2 unused).
BH_HD void sha256_load_block(uint32_t w[16], const uint8_t* m1, uint64_t l1, const uint8_t* m2,
                             uint64_t len, uint64_t total, uint64_t blk);

BH_HD void sha256_msg2(uint32_t out[8], const uint8_t* m1, uint64_t l1, const uint8_t* m2,
                       uint64_t l2) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t len = l1 + l2;
  const uint64_t total = ((len + 9 + 63) / 64) * 64;
  for (uint64_t blk = 0; blk < total; blk += 64) {
    uint32_t w[16];
    const uint8_t* src = blk + 64 <= l1 ? m1 + blk
                         : (blk >= l1 && blk + 64 <= len) ? m2 + (blk - l1)
                                                          : nullptr;
    if (src) {
      load_le_words<16>(w, src);
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = bswap32(w[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = sha256_word2(m1, l1, m2, len, total, blk + 4 * i);
    }
    sha256_block(h, w);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = h[i];
}

BH_HD void sha256_load_block(uint32_t w[16], const uint8_t* m1, uint64_t l1, const uint8_t* m2,
                             uint64_t len, uint64_t total, uint64_t blk) {
  const uint8_t* src = blk + 64 <= l1 ? m1 + blk
                       : (blk >= l1 && blk + 64 <= len) ? m2 + (blk - l1)
                                                        : nullptr;
  if (src) {
    load_le_words<16>(w, src);
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = bswap32(w[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = sha256_word2(m1, l1, m2, len, total, blk + 4 * i);
  }
}

}  // namespace bh
