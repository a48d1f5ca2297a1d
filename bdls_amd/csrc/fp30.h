// Base-field arithmetic for the verify ladder: 9 x 30-bit limbs in u32 lanes,
// Montgomery form with R = 2^270, LAZY reduction.
//
// Why this shape (gfx950, measured): a Montgomery product is issue-bound, and
// with 30-bit limbs a column accumulates <= 9 products + the reduction terms
// in one u64 without ever overflowing, so each product term is exactly one
// in-place v_mad_u64_u32 (no carry flags, no register-pair shuffling). The
// 32-bit-limb CIOS version needed ~530 VALU instructions per product; this one
// ~150. R/p ~ 2^14 leaves headroom for values far above p, so add / sub never
// compare against p: they only carry-normalise limbs.
//
// Value contract ("beta"): every element is a non-negative integer < beta * p
// whose limbs 0..7 are < 2^30 ("normalised"; limb 8 holds the rest).
//   f_mul(a, b)  requires beta_a * beta_b <= 16000 and normalised limbs;
//                returns beta 2 (t < ab/R + p < 2p).
//   f_add        beta_a + beta_b
//   f_sub<K>     a - b + K p, K in {32, 64}: requires beta_b <= K - 1;
//                returns beta_a + K
//   f_mulc<c>    c * beta_a
// The formulas in ec30.h annotate the beta of every intermediate.
//
// Replaces the field layer of Go crypto/internal/nistec (P-256) reached from
// bccsp/sw/ecdsa.go:56 and btcec's fieldVal (vendor/github.com/BDLS-bft/bdls/
// crypto/btcec/field.go:149) for secp256k1.
#pragma once
#include "bh_common.h"
#include "curve_consts.h"

// BH_ZFILTER (default 0): test limb 0 first in f_is_zero2. It saves ~50
// VALU instructions per comb step, but the early return is divergent control
// flow inside the hot formulas and the register allocator pays for it:
// k_ktab_ladder 116 -> 132 VGPRs (3 waves per SIMD instead of 4; config 5's
// ladder -6 %, the build kernel +24 % cycles), k_keycomb 88 -> 112 (round 6,
// hipcc -S variants in DESIGN 4.8). Off.
#ifndef BH_ZFILTER
#define BH_ZFILTER 0
#endif

namespace bh {

constexpr uint32_t kM30 = 0x3fffffffu;
constexpr int kL = 9;  // limbs per base-field element

BH_HD void f_copy(uint32_t r[9], const uint32_t a[9]) {
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = a[i];
}

BH_HD void f_sel(uint32_t r[9], bool c, const uint32_t a[9], const uint32_t b[9]) {
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = c ? a[i] : b[i];
}

template <class C>
BH_HD void f_const(uint32_t r[9], const C& c) {
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = c[i];
}

// Montgomery product t = a b / 2^270 mod p (lazy, beta 2).
// Two phases for instruction-level parallelism: (1) the 17 product columns are
// accumulated independently (17 parallel v_mad_u64_u32 chains of <= 9), then
// (2) one short sequential pass folds the carries and the reduction terms
// (critical path ~2 instructions per column; column bounds in f_redc).
// c += m * k as ONE v_mad_u64_u32. For power-of-two k hipcc otherwise emits a
// 64-bit shift of the whole column plus two masks and an add (4 instructions),
// so k is hidden behind an empty asm that claims to rewrite it in an SGPR:
// the multiply stays a multiply (k in an SGPR operand). An inline-asm mad with
// an explicit VCC carry-out instead made the hazard recognizer put an s_nop
// between consecutive mads (1,414 in k_ktab_ladder).
template <uint32_t K>
BH_HD void mac_k(uint64_t& c, uint32_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t k = K;
  asm("" : "+s"(k));
  c += (uint64_t)m * k;
#else
  c += (uint64_t)m * K;
#endif
}

// Phase 2 of the Montgomery product: fold carries and reduction into r.
template <class F>
BH_HD void f_redc(uint32_t r[9], uint64_t C[17]) {
  uint64_t acc = 0;
  if constexpr (F::sparse_p256) {
    // p = 2^256 - 2^224 + 2^192 + 2^96 - 1 and -p^-1 = 1 mod 2^30, so any m_k
    // congruent to the running column mod 2^30 works, and m_k p, limb-aligned
    // at column k, is
    //   -m_k               (col k)
    //   + m_k 2^96  = m_k << 6   at col k+3
    //   + m_k 2^192 = m_k << 12  at col k+6
    //   + m_k (2^256 - 2^224) = m_k p[7] at col k+7 + m_k p[8] at col k+8
    // Columns 0..7 take m_k = the column's whole LOW WORD (< 2^32): -m_k then
    // clears 32 bits, and the carry into column k+1 is 4 x the high word, one
    // v_mad_u64_u32 instead of a 64-bit shift, a mask and a 64-bit add. Column
    // bound: m_k p[7] < 2^62, so <= 9 products + 2^62 + 2^48 + 2^44 + 2^38 + the
    // carry 2^34 < 13.01 x 2^60. Column 8 takes the masked 30-bit m_8, so
    // M = sum m_k 2^(30k) < 2^270 + 2^242 and t < ab/R + (1 + 2^-28) p, which is
    // < 2p for beta_a beta_b <= 16000 (the formulas stay <= 9604).
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t m = (uint32_t)C[k];
      mac_k<64u>(C[k + 3], m);
      mac_k<4096u>(C[k + 6], m);
      mac_k<F::p[7]>(C[k + 7], m);
      mac_k<F::p[8]>(C[k + 8], m);
      mac_k<4u>(C[k + 1], (uint32_t)(C[k] >> 32));
    }
#pragma unroll
    for (int k = 8; k < 17; k++) {
      acc += C[k];
      const uint32_t m = (uint32_t)acc & kM30;
      if (k == 8) {
        mac_k<64u>(C[11], m);
        mac_k<4096u>(C[14], m);
        mac_k<F::p[7]>(C[15], m);
        mac_k<F::p[8]>(C[16], m);
      } else {
        r[k - 9] = m;
      }
      acc >>= 30;
    }
  } else {
    // generic: m_k = low limb * (-p^-1) mod 2^30; m_k p added column-wise
#pragma unroll
    for (int k = 0; k < 17; k++) {
      acc += C[k];
      if (k < 9) {
        const uint32_t m = ((uint32_t)acc * F::n0) & kM30;
        acc += (uint64_t)m * F::p[0];  // low 30 bits become zero
#pragma unroll
        for (int j = 1; j < 9; j++)
          if (F::p[j]) C[k + j] += (uint64_t)m * F::p[j];
      } else {
        r[k - 9] = (uint32_t)acc & kM30;
      }
      acc >>= 30;
    }
  }
  r[8] = (uint32_t)acc;
}

template <class F>
BH_HD void f_mul(uint32_t r[9], const uint32_t a[9], const uint32_t b[9]) {
  uint64_t C[17];
#pragma unroll
  for (int k = 0; k < 17; k++) C[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) C[i + j] += (uint64_t)a[i] * b[j];
  f_redc<F>(r, C);
}

// Squaring: 9 squares + 36 doubled cross products (2 a_i) a_j. A column holds
// <= 4 cross products < 2^61 plus one square < 2^60: the same < 2^64 bound.
// Precondition as f_mul, and limb 8 < 2^30 (always: beta <= 2^14).
template <class F>
BH_HD void f_sqr(uint32_t r[9], const uint32_t a[9]) {
  uint64_t C[17];
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a[i] << 1;
#pragma unroll
  for (int k = 0; k < 17; k++) C[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    C[2 * i] += (uint64_t)a[i] * a[i];
#pragma unroll
    for (int j = i + 1; j < 9; j++) C[i + j] += (uint64_t)d[i] * a[j];
  }
  f_redc<F>(r, C);
}

// r = a + b, limbs re-normalised.
BH_HD void f_add(uint32_t r[9], const uint32_t a[9], const uint32_t b[9]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a[i] + b[i] + c;
    r[i] = t & kM30;
    c = t >> 30;
  }
  r[8] = a[8] + b[8] + c;
}

// r = a - b + K p (K = 32 or 64), limbs re-normalised. Every limb of the
// borrowed K p exceeds the matching limb of b, so no intermediate goes negative.
template <class F, int K>
BH_HD void f_sub(uint32_t r[9], const uint32_t a[9], const uint32_t b[9]) {
  static_assert(K == 32 || K == 64, "K");
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t kk = (K == 32) ? F::k32[i] : F::k64[i];
    const uint32_t t = a[i] + kk - b[i] + c;
    r[i] = t & kM30;
    c = t >> 30;
  }
  const uint32_t k8 = (K == 32) ? F::k32[8] : F::k64[8];
  r[8] = a[8] + k8 - b[8] + c;
}

// K p in a borrowed form that lends B 2^30 to every limb below the top:
// limb 0 = n_0 + B 2^30, limbs 1..7 = n_i + B 2^30 - B, limb 8 = n_8 - B
// (n = K p's normalised limbs). B = 1 is the k32 / k64 form; B = 2 leaves
// every limb >= 2^31 - 2, so TWO normalised limbs can be subtracted from it in
// one pass (round 6: the fused passes below, one carry chain where the
// formulas had two or three).
struct Limbs9 {
  uint32_t v[9];
};
template <class F, int K, int B>
constexpr Limbs9 kp_borrowed() {
  Limbs9 r{};
  uint64_t c = 0;
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)F::p[i] * (uint64_t)K + c;
    const uint64_t n = i < 8 ? (t & kM30) : t;
    c = i < 8 ? (t >> 30) : 0;
    r.v[i] = (uint32_t)(n + (i < 8 ? ((uint64_t)B << 30) : 0) - (i > 0 ? (uint64_t)B : 0));
  }
  return r;
}
template <class F, int K, int B>
struct KpB {
  static constexpr Limbs9 k = kp_borrowed<F, K, B>();
  static_assert(k.v[8] < (1u << 26), "K p's top limb covers the borrow");
};

// r = a + 2 b, limbs re-normalised (beta_a + 2 beta_b): H^3 + 2V of the
// additions in one pass (t < 3 * 2^30 + 3).
BH_HD void f_add2x(uint32_t r[9], const uint32_t a[9], const uint32_t b[9]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a[i] + (b[i] << 1) + c;
    r[i] = t & kM30;
    c = t >> 30;
  }
  r[8] = a[8] + (b[8] << 1) + c;
}

// r = a + b - c + K p (K = 32 or 64) in one pass instead of f_add then f_sub.
// Requires value(c) <= K p; returns beta_a + beta_b + K. A limb never leaves
// u32: a_i + b_i + kk_i + carry <= 2 (2^30 - 1) + (2^31 - 2) + 3 < 2^32 (the
// B = 1 borrowed limbs are <= n_i + 2^30 - 1), and kk_i >= c_i.
template <class F, int K>
BH_HD void f_addsub(uint32_t r[9], const uint32_t a[9], const uint32_t b[9], const uint32_t c[9]) {
  static_assert(K == 32 || K == 64, "K");
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t kk = (K == 32) ? F::k32[i] : F::k64[i];
    const uint32_t t = a[i] + b[i] + kk + cy - c[i];
    r[i] = t & kM30;
    cy = t >> 30;
  }
  const uint32_t k8 = (K == 32) ? F::k32[8] : F::k64[8];
  r[8] = a[8] + b[8] + k8 + cy - c[8];
}

// r = a - b - c + K p in one pass (the B = 2 borrowed K p: kk_i >= b_i + c_i,
// and a_i + kk_i + carry <= (2^30 - 1) + (2^31 + 2^30 - 3) + 3 < 2^32).
// Requires value(b) + value(c) <= K p; returns beta_a + K.
template <class F, int K>
BH_HD void f_sub2(uint32_t r[9], const uint32_t a[9], const uint32_t b[9], const uint32_t c[9]) {
  constexpr Limbs9 kk = KpB<F, K, 2>::k;
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a[i] + kk.v[i] + cy - b[i] - c[i];
    r[i] = t & kM30;
    cy = t >> 30;
  }
  r[8] = a[8] + kk.v[8] + cy - b[8] - c[8];
}

// r = (neg ? -s : s) - y + K p in one pass: a table point's sign folded into
// the subtraction that consumes its y (the additions' r = S2 - Y1), instead of
// negating y and selecting first. Per limb the true value kk_i +- s_i - y_i +
// carry lies in [0, 2^32) (B = 2 borrowed K p), so the u32 wrap of -s_i is
// exact. Requires value(s) + value(y) <= K p when neg, value(y) <= K p else;
// returns K (neg) or beta_s + K.
template <class F, int K>
BH_HD void f_csub(uint32_t r[9], bool neg, const uint32_t s[9], const uint32_t y[9]) {
  constexpr Limbs9 kk = KpB<F, K, 2>::k;
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t x = neg ? 0u - s[i] : s[i];
    const uint32_t t = kk.v[i] + x + cy - y[i];
    r[i] = t & kM30;
    cy = t >> 30;
  }
  const uint32_t x8 = neg ? 0u - s[8] : s[8];
  r[8] = kk.v[8] + x8 + cy - y[8];
}

// r = K p - a
template <class F, int K>
BH_HD void f_neg(uint32_t r[9], const uint32_t a[9]) {
  const uint32_t z[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  f_sub<F, K>(r, z, a);
}

// r = c a for a small constant c (c * 2^30 + carry < 2^64 trivially).
template <uint32_t C>
BH_HD void f_mulc(uint32_t r[9], const uint32_t a[9]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = (uint64_t)a[i] * C + c;
    r[i] = (uint32_t)t & kM30;
    c = t >> 30;
  }
  r[8] = a[8] * C + (uint32_t)c;
}

// For beta <= 2: canonical representative in [0, p).
template <class F>
BH_HD void f_canon(uint32_t r[9], const uint32_t a[9]) {
  uint32_t d[9];
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int32_t t = (int32_t)a[i] - (int32_t)F::p[i] + c;
    d[i] = (uint32_t)t & kM30;
    c = t >> 30;  // arithmetic: 0 or -1
  }
  const int32_t t8 = (int32_t)a[8] - (int32_t)F::p[8] + c;
  d[8] = (uint32_t)t8;
  f_sel(r, t8 >= 0, d, a);
}

// Any beta (<= 8192): a mod p in [0, p) in the same domain, via a Montgomery
// product with R mod p (= 1 in Montgomery form) and one conditional subtract.
template <class F>
BH_HD void f_reduce(uint32_t r[9], const uint32_t a[9]) {
  uint32_t one[9];
  f_const(one, F::r1);
  f_mul<F>(r, a, one);
  f_canon<F>(r, r);
}

BH_HD bool f_eq(const uint32_t a[9], const uint32_t b[9]) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) x |= a[i] ^ b[i];
  return x == 0;
}

// beta <= 2 and normalised: value == 0 mod p  <=>  a in {0, p}
// (BH_ZFILTER: limb 0 filters first -- a value in {0, p} has limb 0 in
// {0, p_0} -- measured and left off, see its definition)
template <class F>
BH_HD bool f_is_zero2(const uint32_t a[9]) {
#if BH_ZFILTER
  if (a[0] != 0u && a[0] != F::p[0]) return false;
#endif
  uint32_t z = 0, q = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    z |= a[i];
    q |= a[i] ^ F::p[i];
  }
  return z == 0 || q == 0;
}

// 8 x 32-bit little-endian limbs (value < 2^256) <-> 9 x 30-bit limbs
BH_HD void f_from_u256(uint32_t r[9], const uint32_t a[8]) {
  r[0] = a[0] & kM30;
#pragma unroll
  for (int i = 1; i < 8; i++) {
    const int lo = 30 * i;  // bit offset
    const int w = lo >> 5, s = lo & 31;
    uint32_t v = a[w] >> s;
    if (s > 2 && w + 1 < 8) v |= a[w + 1] << (32 - s);
    r[i] = v & kM30;
  }
  r[8] = a[7] >> 16;
}

BH_HD void f_to_u256(uint32_t r[8], const uint32_t a[9]) {  // a normalised, < 2^256
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const int bit = 32 * w;
    const int i = bit / 30, s = bit % 30;
    uint32_t v = a[i] >> s;
    if (i + 1 < 9) v |= a[i + 1] << (30 - s);
    if (s > 28 && i + 2 < 9) v |= a[i + 2] << (60 - s);
    r[w] = v;
  }
}

template <class F>
BH_HD void f_to_mont(uint32_t r[9], const uint32_t a[9]) {
  uint32_t r2[9];
  f_const(r2, F::r2);
  f_mul<F>(r, a, r2);
}

// r = a^(2^k) (k squarings; a loop, so the code stays one f_sqr body)
template <class F>
BH_HD void f_sqrn(uint32_t r[9], const uint32_t a[9], int k) {
  f_copy(r, a);
#pragma unroll 1
  for (int i = 0; i < k; i++) f_sqr<F>(r, r);
}

// r = a^(2^k) * b
template <class F>
BH_HD void f_sqrn_mul(uint32_t r[9], const uint32_t a[9], int k, const uint32_t b[9]) {
  f_sqrn<F>(r, a, k);
  f_mul<F>(r, r, b);
}

// a^(p-2) (Fermat inverse in the Montgomery domain; a != 0 mod p) by an
// addition chain over e_k = a^(2^k - 1): 255 squarings + 12 (P-256) / 15
// (secp256k1) multiplications instead of the binary method's ~128 / ~250.
//   P-256  p-2 = [32 ones][31 zeros, 1][96 zeros][64 ones][30 ones, 0, 1]
//   k1     p-2 = [223 ones][0][22 ones][0000 1][0 11][0 1]
template <class F>
BH_HD void f_inv(uint32_t r[9], const uint32_t a[9]) {
  uint32_t e2[9], e3[9], t[9], u[9], acc[9];
  f_sqrn_mul<F>(e2, a, 1, a);            // e2
  f_sqrn_mul<F>(e3, e2, 1, a);           // e3
  if constexpr (F::sparse_p256) {
    uint32_t e15[9], e32[9];
    f_sqrn_mul<F>(t, e3, 3, e3);         // e6
    f_sqrn_mul<F>(u, t, 6, t);           // e12
    f_sqrn_mul<F>(e15, u, 3, e3);        // e15
    f_sqrn_mul<F>(t, e15, 15, e15);      // e30
    f_sqrn_mul<F>(e32, t, 2, e2);        // e32
    f_sqrn_mul<F>(acc, e32, 32, a);      // [32 ones][31 zeros, 1]
    f_sqrn<F>(acc, acc, 96);
    f_sqrn_mul<F>(acc, acc, 32, e32);
    f_sqrn_mul<F>(acc, acc, 32, e32);
    f_sqrn_mul<F>(acc, acc, 30, t);      // 30 ones
    f_sqrn_mul<F>(acc, acc, 2, a);       // 0 1
  } else {
    uint32_t e11[9], e22[9], e44[9];
    f_sqrn_mul<F>(t, e3, 3, e3);         // e6
    f_sqrn_mul<F>(u, t, 3, e3);          // e9
    f_sqrn_mul<F>(e11, u, 2, e2);        // e11
    f_sqrn_mul<F>(e22, e11, 11, e11);    // e22
    f_sqrn_mul<F>(e44, e22, 22, e22);    // e44
    f_sqrn_mul<F>(t, e44, 44, e44);      // e88
    f_sqrn_mul<F>(u, t, 88, t);          // e176
    f_sqrn_mul<F>(t, u, 44, e44);        // e220
    f_sqrn_mul<F>(acc, t, 3, e3);        // e223
    f_sqrn_mul<F>(acc, acc, 23, e22);    // 0, 22 ones
    f_sqrn_mul<F>(acc, acc, 5, a);       // 0000 1
    f_sqrn_mul<F>(acc, acc, 3, e2);      // 0 11
    f_sqrn_mul<F>(acc, acc, 2, a);       // 0 1
  }
  f_copy(r, acc);
}

}  // namespace bh
