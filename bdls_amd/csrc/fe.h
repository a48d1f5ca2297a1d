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

// ------------------------------------------- safegcd (divsteps) inversion
// Bernstein-Yang constant-iteration modular inversion (the "safegcd" divstep
// recurrence, "Fast constant-time gcd computation and modular inversion",
// 2019) on signed radix-2^30 limbs: 20 batches of 30 branch-free divsteps
// (600 >= 590, the iteration bound for 256-bit moduli), each batch applied to
// (f, g) and (d, e) as a 2x2 matrix of 31-bit integers. About 14k simple VALU
// instructions per inversion against ~77k for the Fermat ladder above, with
// no data-dependent branch (every lane of a wave runs the same schedule).
// The inputs are public (signature scalars), so no side-channel rule applies;
// constant iteration is chosen for SIMT uniformity.
struct Div2x2 {
  int32_t u, v, q, r;
};

// 30 divsteps on the low words of f (odd) and g; returns the new zeta
// (= -(delta + 1/2)). Matrix entries stay within [-2^30, 2^30].
BH_HD int32_t divsteps30(int32_t zeta, uint32_t f, uint32_t g, Div2x2& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; i++) {
    uint32_t m1 = (uint32_t)(zeta >> 31);  // zeta < 0
    const uint32_t m2 = 0u - (g & 1u);     // g odd
    const uint32_t x = (f ^ m1) - m1, y = (u ^ m1) - m1, z = (v ^ m1) - m1;
    g += x & m2;
    q += y & m2;
    r += z & m2;
    m1 &= m2;
    zeta = (zeta ^ (int32_t)m1) - 1;
    f += g & m1;
    u += q & m1;
    v += r & m1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return zeta;
}

// Variable-time form of divsteps30 for a lane that inverts ONE public scalar
// alone (the latency kernel k_small: no other lane waits on its schedule).
// Same 30 divsteps and the same transition matrix, computed in runs: a run of
// zero low bits of g is one shift, and up to min(eta + 1, i, 6) low bits of g
// are cancelled at once by adding w f, w = -g f^-1 mod 2^limit (f^-1 mod 64 by
// one Newton step from f, valid mod 8 for odd f). eta = -delta (starts at -1).
// The published variable-time optimisation of Bernstein-Yang's divsteps.
BH_HD int32_t divsteps30_var(int32_t eta, uint32_t f, uint32_t g, Div2x2& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 30;
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xffffffffu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    // g is odd here
    if (eta < 0) {
      const uint32_t x = f, y = u, z = v;
      eta = -eta;
      f = g;
      u = q;
      v = r;
      g = 0u - x;
      q = 0u - y;
      r = 0u - z;
    }
    int limit = eta + 1 < i ? eta + 1 : i;
    if (limit > 6) limit = 6;
    const uint32_t m = (0xffffffffu >> (32 - limit)) & 63u;
    const uint32_t finv = f * (2u - f * f);   // f^-1 mod 64
    const uint32_t w = (0u - g * finv) & m;   // g + w f = 0 mod 2^limit
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}

constexpr int32_t kS30Mask = 0x3fffffff;

// [d, e] <- (t [d, e] + m [md, me]) / 2^30 with md, me chosen so the division
// is exact; keeps d, e in (-2m, m).
template <class M>
BH_HD void divsteps_update_de(int32_t d[9], int32_t e[9], const Div2x2& t) {
  const int32_t sd = d[8] >> 31, se = e[8] >> 31;
  int32_t md = (t.u & sd) + (t.v & se);
  int32_t me = (t.q & sd) + (t.r & se);
  int64_t cd = (int64_t)t.u * d[0] + (int64_t)t.v * e[0];
  int64_t ce = (int64_t)t.q * d[0] + (int64_t)t.r * e[0];
  md -= (int32_t)((M::inv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)kS30Mask);
  me -= (int32_t)((M::inv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)kS30Mask);
  cd += (int64_t)M::s30[0] * md;
  ce += (int64_t)M::s30[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    const int32_t di = d[i], ei = e[i];
    cd += (int64_t)t.u * di + (int64_t)t.v * ei + (int64_t)M::s30[i] * md;
    ce += (int64_t)t.q * di + (int64_t)t.r * ei + (int64_t)M::s30[i] * me;
    d[i - 1] = (int32_t)cd & kS30Mask;
    e[i - 1] = (int32_t)ce & kS30Mask;
    cd >>= 30;
    ce >>= 30;
  }
  d[8] = (int32_t)cd;
  e[8] = (int32_t)ce;
}

// [f, g] <- t [f, g] / 2^30 (exact by construction of the divsteps).
BH_HD void divsteps_update_fg(int32_t f[9], int32_t g[9], const Div2x2& t) {
  int64_t cf = (int64_t)t.u * f[0] + (int64_t)t.v * g[0];
  int64_t cg = (int64_t)t.q * f[0] + (int64_t)t.r * g[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    const int32_t fi = f[i], gi = g[i];
    cf += (int64_t)t.u * fi + (int64_t)t.v * gi;
    cg += (int64_t)t.q * fi + (int64_t)t.r * gi;
    f[i - 1] = (int32_t)cf & kS30Mask;
    g[i - 1] = (int32_t)cg & kS30Mask;
    cf >>= 30;
    cg >>= 30;
  }
  f[8] = (int32_t)cf;
  g[8] = (int32_t)cg;
}

// d <- d + (c ? m : 0), then (neg ? -d : d), carries propagated (limbs 0..7
// in [0, 2^30), limb 8 signed).
template <class M>
BH_HD void s30_addm_neg(int32_t d[9], bool c, bool neg) {
  int64_t cy = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    int64_t v = (int64_t)d[i] + (c ? M::s30[i] : 0);
    cy += neg ? -v : v;
    if (i < 8) {
      d[i] = (int32_t)cy & kS30Mask;
      cy >>= 30;
    } else {
      d[8] = (int32_t)cy;
    }
  }
}

// r = a^-1 mod m for plain canonical a in [1, m) (32-bit limbs in and out).
// VAR: divsteps30_var batches, stopping once g = 0 (the remaining batches
// would leave d mod m and f unchanged).
template <class M, bool VAR = false>
BH_HD void mod_inv_sg(uint32_t r[8], const uint32_t a[8]) {
  int32_t d[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int32_t e[9] = {1, 0, 0, 0, 0, 0, 0, 0, 0};
  int32_t f[9], g[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    f[i] = M::s30[i];
    const int b = 30 * i, w = b >> 5, s = b & 31;
    uint64_t x = a[w];
    if (w + 1 < 8) x |= (uint64_t)a[w + 1] << 32;
    g[i] = (int32_t)((x >> s) & (i < 8 ? (uint64_t)kS30Mask : 0xffffffffull));
  }
  // divsteps30: zeta = -(delta + 1/2), delta = 1/2 (600 >= 590 steps suffice);
  // divsteps30_var: eta = -delta, Bernstein-Yang's original delta = 1, whose
  // bound for 256-bit inputs is (49 * 256 + 57) / 17 = 741 <= 25 * 30 steps
  int32_t zeta = -1;
  for (int it = 0; it < (VAR ? 25 : 20); it++) {
    Div2x2 t;
    if constexpr (VAR) {
      int32_t any = 0;
#pragma unroll
      for (int k = 0; k < 9; k++) any |= g[k];
      if (!any) break;
      zeta = divsteps30_var(zeta, (uint32_t)f[0], (uint32_t)g[0], t);
    } else {
      zeta = divsteps30(zeta, (uint32_t)f[0], (uint32_t)g[0], t);
    }
    divsteps_update_de<M>(d, e, t);
    divsteps_update_fg(f, g, t);
  }
  // g == 0, f == +-1, d == +-a^-1 in (-2m, m): bring to [0, m)
  s30_addm_neg<M>(d, d[8] < 0, f[8] < 0);
  s30_addm_neg<M>(d, d[8] < 0, false);
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const int b = 32 * w, i = b / 30, s = b % 30;
    uint64_t x = (uint64_t)(uint32_t)d[i] >> s;
    if (i + 1 < 9) x |= (uint64_t)(uint32_t)d[i + 1] << (30 - s);  // 60 - s >= 32 bits
    r[w] = (uint32_t)x;
  }
}

// Montgomery-domain inverse by safegcd: input aR, output a^-1 R
// ((aR)^-1 * R^3 * R^-1). VAR: variable-time divsteps with an early exit
// once g = 0 (a lane inverting alone; the result is the same).
template <class M, bool VAR = false>
BH_HD void mont_inv_sg(uint32_t r[8], const uint32_t a[8]) {
  uint32_t t[8], r3[8];
  mod_inv_sg<M, VAR>(t, a);
  load_const8(r3, M::r3);
  mont_mul<M>(r, t, r3);
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
