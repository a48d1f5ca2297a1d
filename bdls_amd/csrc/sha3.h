// SHA3-256 (FIPS 202: Keccak-f[1600], rate 136 bytes, domain byte 0x06), one
// message per lane, message bytes read straight from HBM. Replaces
// bccsp/sw/hash.go:29-33 with sha3.New256 (registered at bccsp/sw/new.go:72;
// vendor/golang.org/x/crypto/sha3/hashes.go:28-32, x/crypto v0.14.0:
// rate 136, outputLen 32, dsbyte 0x06) as selected by
// msp/identities.go:219-227 when the MSP's SignatureHashFamily is SHA3.
//
// gfx950 has no 64-bit rotate: each Keccak lane is kept as two u32 halves and
// a 64-bit rotation is two v_alignbit_b32 (funnel shifts). The state is 50
// VGPRs; with the round loop fully unrolled rho/pi is register renaming.
#pragma once
#include <utility>

#include "bh_common.h"

namespace bh {

// Keccak round constants (FIPS 202 iota), low / high 32 bits.
struct KeccakConst {
  static constexpr uint32_t rc_lo[24] = {
      0x00000001u, 0x00008082u, 0x0000808au, 0x80008000u, 0x0000808bu, 0x80000001u,
      0x80008081u, 0x00008009u, 0x0000008au, 0x00000088u, 0x80008009u, 0x8000000au,
      0x8000808bu, 0x0000008bu, 0x00008089u, 0x00008003u, 0x00008002u, 0x00000080u,
      0x0000800au, 0x8000000au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
  static constexpr uint32_t rc_hi[24] = {
      0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u,
      0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u,
      0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u,
      0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};
  // rho offsets r[x + 5 y]
  static constexpr int rho[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                  25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
  // pi: lane (x, y) moves to (y, 2x + 3y mod 5)
  static constexpr int pi_dst(int i) { return (i / 5) + 5 * ((2 * (i % 5) + 3 * (i / 5)) % 5); }
};

struct K64 {
  uint32_t lo, hi;
};

// (hi:lo) rotated left by N (compile-time, 0 < N < 64)
template <int N>
BH_HD K64 rotl64(K64 x) {
  static_assert(N > 0 && N < 64, "N");
  if constexpr (N == 32) {
    return K64{x.hi, x.lo};
  } else if constexpr (N > 32) {
    return rotl64<N - 32>(K64{x.hi, x.lo});
  } else {
#if defined(__HIP_DEVICE_COMPILE__)
    return K64{__builtin_amdgcn_alignbit(x.lo, x.hi, 32 - N),
               __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - N)};
#else
    return K64{(x.lo << N) | (x.hi >> (32 - N)), (x.hi << N) | (x.lo >> (32 - N))};
#endif
  }
}

BH_HD K64 kxor(K64 a, K64 b) { return K64{a.lo ^ b.lo, a.hi ^ b.hi}; }
// a ^ (~b & c)
BH_HD K64 kchi(K64 a, K64 b, K64 c) { return K64{a.lo ^ (~b.lo & c.lo), a.hi ^ (~b.hi & c.hi)}; }

template <int I>
BH_HD K64 rho_lane(K64 v) {
  constexpr int r = KeccakConst::rho[I];
  if constexpr (r == 0) return v;
  else return rotl64<r>(v);
}

template <int... I>
BH_HD void rho_pi(K64 b[25], const K64 a[25], std::integer_sequence<int, I...>) {
  ((b[KeccakConst::pi_dst(I)] = rho_lane<I>(a[I])), ...);
}

template <int R>
BH_HD void keccak_round(K64 a[25]) {
  K64 c[5], d[5], b[25];
#pragma unroll
  for (int x = 0; x < 5; x++)
    c[x] = kxor(kxor(kxor(a[x], a[x + 5]), kxor(a[x + 10], a[x + 15])), a[x + 20]);
#pragma unroll
  for (int x = 0; x < 5; x++) d[x] = kxor(c[(x + 4) % 5], rotl64<1>(c[(x + 1) % 5]));
#pragma unroll
  for (int i = 0; i < 25; i++) a[i] = kxor(a[i], d[i % 5]);
  rho_pi(b, a, std::make_integer_sequence<int, 25>{});
#pragma unroll
  for (int y = 0; y < 5; y++)
#pragma unroll
    for (int x = 0; x < 5; x++)
      a[x + 5 * y] = kchi(b[x + 5 * y], b[(x + 1) % 5 + 5 * y], b[(x + 2) % 5 + 5 * y]);
  a[0].lo ^= KeccakConst::rc_lo[R];
  a[0].hi ^= KeccakConst::rc_hi[R];
}

template <int... R>
BH_HD void keccak_rounds(K64 a[25], std::integer_sequence<int, R...>) {
  (keccak_round<R>(a), ...);
}

BH_HD void keccak_f1600(K64 a[25]) { keccak_rounds(a, std::make_integer_sequence<int, 24>{}); }

constexpr uint32_t kSha3Rate = 136;  // bytes (17 lanes)

// Little-endian word at byte pos of the padded stream: message bytes [0, len),
// the domain/pad byte 0x06 at len, 0x80 ORed into the last byte of the rate
// block (sha3.go padAndPermute).
BH_HD uint32_t sha3_word(const uint8_t* m, uint64_t len, uint64_t total, uint64_t pos) {
  if (pos + 4 <= len)
    return (uint32_t)m[pos] | ((uint32_t)m[pos + 1] << 8) | ((uint32_t)m[pos + 2] << 16) |
           ((uint32_t)m[pos + 3] << 24);
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t p = pos + k;
    uint32_t byte = 0;
    if (p < len) byte = m[p];
    else if (p == len) byte = 0x06u;
    if (p == total - 1) byte |= 0x80u;
    v |= byte << (8 * k);
  }
  return v;
}

// out = SHA3-256(m[0..len)), 32 bytes.
BH_HD void sha3_256_msg(uint8_t out[32], const uint8_t* m, uint64_t len) {
  K64 a[25];
#pragma unroll
  for (int i = 0; i < 25; i++) a[i] = K64{0u, 0u};
  const uint64_t total = (len / kSha3Rate + 1) * kSha3Rate;  // padding adds 1..136 bytes
  for (uint64_t blk = 0; blk < total; blk += kSha3Rate) {  // one permutation call site
    uint32_t w[34];
    if (blk + kSha3Rate <= len) {  // a full message block, any alignment
      load_le_words<34>(w, m + blk);
    } else {
#pragma unroll
      for (int i = 0; i < 34; i++) w[i] = sha3_word(m, len, total, blk + 4 * i);
    }
#pragma unroll
    for (int i = 0; i < 17; i++) {
      a[i].lo ^= w[2 * i];
      a[i].hi ^= w[2 * i + 1];
    }
    keccak_f1600(a);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      out[8 * i + k] = (uint8_t)(a[i].lo >> (8 * k));
      out[8 * i + 4 + k] = (uint8_t)(a[i].hi >> (8 * k));
    }
  }
}

// Two-span message (see sha256.h sha256_msg2): m1[0, l1) || m2[0, l2).
BH_HD uint32_t sha3_word2(const uint8_t* m1, uint64_t l1, const uint8_t* m2, uint64_t len,
                          uint64_t total, uint64_t pos) {
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t p = pos + k;
    uint32_t byte = 0;
    if (p < len) byte = p < l1 ? m1[p] : m2[p - l1];
    else if (p == len) byte = 0x06u;
    if (p == total - 1) byte |= 0x80u;
    v |= byte << (8 * k);
  }
  return v;
}

BH_HD void sha3_256_msg2(uint8_t out[32], const uint8_t* m1, uint64_t l1, const uint8_t* m2,
                         uint64_t l2) {
  K64 a[25];
#pragma unroll
  for (int i = 0; i < 25; i++) a[i] = K64{0u, 0u};
  const uint64_t len = l1 + l2;
  const uint64_t total = (len / kSha3Rate + 1) * kSha3Rate;
  for (uint64_t blk = 0; blk < total; blk += kSha3Rate) {
    uint32_t w[34];
    const uint8_t* src = blk + kSha3Rate <= l1 ? m1 + blk
                         : (blk >= l1 && blk + kSha3Rate <= len) ? m2 + (blk - l1)
                                                                 : nullptr;
    if (src) {
      load_le_words<34>(w, src);
    } else {
#pragma unroll
      for (int i = 0; i < 34; i++) w[i] = sha3_word2(m1, l1, m2, len, total, blk + 4 * i);
    }
#pragma unroll
    for (int i = 0; i < 17; i++) {
      a[i].lo ^= w[2 * i];
      a[i].hi ^= w[2 * i + 1];
    }
    keccak_f1600(a);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      out[8 * i + k] = (uint8_t)(a[i].lo >> (8 * k));
      out[8 * i + 4 + k] = (uint8_t)(a[i].hi >> (8 * k));
    }
  }
}

}  // namespace bh
