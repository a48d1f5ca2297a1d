// 256-bit modular arithmetic on 8 x 32-bit little-endian limbs, Montgomery form
// (R = 2^256), one field element per lane.
//
// Replaces the field layer of Go's crypto/internal/nistec (P-256) and
// crypto/internal/bigmod (mod-n scalars) reached from bccsp/sw/ecdsa.go:56, and
// btcec's fieldVal (vendor/github.com/BDLS-bft/bdls/crypto/btcec/field.go:149)
// for secp256k1. Designed for gfx950 VALU: the product terms are
// v_mad_u64_u32 (32x32+64 -> 64) whose 64-bit result can absorb one extra
// 32-bit addend without overflow, so each CIOS step is one mad + one 64-bit
// add; the modulus is a compile-time constant so zero / one / all-ones limbs
// of p (P-256: p = {-1,-1,-1,0,0,0,1,-1}, -p^-1 = 1 mod 2^32) fold away.
#pragma once
#include "bh_common.h"
#include "curve_consts.h"

namespace bh {

// ---------------------------------------------------------------- raw limbs
BH_HD uint32_t add8(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = __builtin_addc(a[i], b[i], c, &c);
  return c;
}

BH_HD uint32_t sub8(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = __builtin_subc(a[i], b[i], c, &c);
  return c;
}

// a >= b (unsigned 256-bit)
BH_HD bool geq8(const uint32_t a[8], const uint32_t b[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)__builtin_subc(a[i], b[i], c, &c);
  return c == 0;
}

BH_HD bool is_zero8(const uint32_t a[8]) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a[i];
  return x == 0;
}

BH_HD bool eq8(const uint32_t a[8], const uint32_t b[8]) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a[i] ^ b[i];
  return x == 0;
}

BH_HD void copy8(uint32_t r[8], const uint32_t a[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = a[i];
}

BH_HD void sel8(uint32_t r[8], bool c, const uint32_t a[8], const uint32_t b[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = c ? a[i] : b[i];
}

template <class C>
BH_HD void load_const8(uint32_t r[8], const C& c) {
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = c[i];
}

// ------------------------------------------------------ modular add / sub
// Inputs canonical (< m); outputs canonical.
template <class M>
BH_HD void mod_add(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t s[8], d[8];
  uint32_t c = add8(s, a, b);
  uint32_t bo = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = __builtin_subc(s[i], M::m[i], bo, &bo);
  // s - m is the answer iff (carry out of a+b) or (no borrow in s-m)
  bool use_d = c | (bo ^ 1u);
  sel8(r, use_d, d, s);
}

template <class M>
BH_HD void mod_sub(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t d[8], e[8];
  uint32_t bo = sub8(d, a, b);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = __builtin_addc(d[i], M::m[i], c, &c);
  sel8(r, bo != 0, e, d);
}

template <class M>
BH_HD void mod_dbl(uint32_t r[8], const uint32_t a[8]) { mod_add<M>(r, a, a); }

template <class M>
BH_HD void mod_neg(uint32_t r[8], const uint32_t a[8]) {
  uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  mod_sub<M>(r, z, a);
}

// ------------------------------------------------ Montgomery multiplication
// CIOS (coarsely integrated operand scanning). t stays < 2m between rows;
// one conditional subtraction at the end gives a canonical result.
template <class M>
BH_HD void mont_mul(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t t8 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t uv = (uint64_t)a[j] * b[i] + t[j] + c;  // <= 2^64 - 1
      t[j] = (uint32_t)uv;
      c = uv >> 32;
    }
    uint64_t uv = (uint64_t)t8 + c;
    t8 = (uint32_t)uv;
    uint32_t t9 = (uint32_t)(uv >> 32);
    const uint32_t m = t[0] * M::n0;
    uv = (uint64_t)m * M::m[0] + t[0];
    c = uv >> 32;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      uv = (uint64_t)m * M::m[j] + t[j] + c;
      t[j - 1] = (uint32_t)uv;
      c = uv >> 32;
    }
    uv = (uint64_t)t8 + c;
    t[7] = (uint32_t)uv;
    t8 = t9 + (uint32_t)(uv >> 32);
  }
  uint32_t d[8];
  uint32_t bo = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = __builtin_subc(t[i], M::m[i], bo, &bo);
  bool use_d = (t8 != 0) | (bo == 0);
  sel8(r, use_d, d, t);
}

template <class M>
BH_HD void mont_sqr(uint32_t r[8], const uint32_t a[8]) {
  mont_mul<M>(r, a, a);
}

template <class M>
BH_HD void to_mont(uint32_t r[8], const uint32_t a[8]) {
  uint32_t r2[8];
  load_const8(r2, M::r2);
  mont_mul<M>(r, a, r2);
}

template <class M>
BH_HD void from_mont(uint32_t r[8], const uint32_t a[8]) {
  uint32_t one[8] = {1, 0, 0, 0, 0, 0, 0, 0};
  mont_mul<M>(r, a, one);
}

// a^(m-2) in the Montgomery domain: input aR, output a^-1 R (a != 0).
// Left-to-right binary exponentiation over the compile-time exponent; the
// per-bit branch is wave-uniform.
template <class M>
BH_HDNI void mont_inv(uint32_t r[8], const uint32_t a[8]) {
  uint32_t acc[8];
  load_const8(acc, M::r1);  // 1 in Montgomery form
  for (int i = 255; i >= 0; i--) {
    mont_sqr<M>(acc, acc);
    if ((M::mm2[i >> 5] >> (i & 31)) & 1u) mont_mul<M>(acc, acc, a);
  }
  copy8(r, acc);
}

// 32 big-endian bytes -> limbs
BH_HD void be32_to_limbs(uint32_t r[8], const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t* p = b + 28 - 4 * i;
    r[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  }
}

BH_HD void limbs_to_be32(uint8_t* b, const uint32_t a[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint8_t* p = b + 28 - 4 * i;
    p[0] = (uint8_t)(a[i] >> 24);
    p[1] = (uint8_t)(a[i] >> 16);
    p[2] = (uint8_t)(a[i] >> 8);
    p[3] = (uint8_t)a[i];
  }
}

}  // namespace bh
