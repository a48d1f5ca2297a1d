// Jacobian point arithmetic on the radix-2^30 lazy field (fp30.h).
//
// Replaces the point layer of Go crypto/internal/nistec P-256 (ScalarMult /
// ScalarBaseMult / Add behind crypto/ecdsa verifyNISTEC, called at
// bccsp/sw/ecdsa.go:56) and btcec addJacobian / doubleJacobian
// (vendor/github.com/BDLS-bft/bdls/crypto/btcec/btcec.go:461-482, 765-887).
//
// Formulas (EFD g1p/auto-shortw-jacobian*): dbl-2001-b (a=-3, 3M+5S),
// dbl-2009-l (a=0, 2M+5S), add-1998-cmo-2 (12M+4S), madd (8M+3S).
// [bN] = value bound in units of p after the step (see fp30.h). Coordinates
// leaving any function here have beta <= 66; inputs are required to satisfy the
// bounds stated per function (all call sites in verify.h do).
// The add formulas are incomplete and REPORT the degenerate case (equal x):
// callers resolve doubling / infinity explicitly.
#pragma once
#include "fp30.h"

namespace bh {

struct J30 {
  uint32_t X[9], Y[9], Z[9];
};

BH_HD void j_copy(J30& r, const J30& p) {
  f_copy(r.X, p.X);
  f_copy(r.Y, p.Y);
  f_copy(r.Z, p.Z);
}

BH_HD void j_sel(J30& r, bool c, const J30& a, const J30& b) {
  f_sel(r.X, c, a.X, b.X);
  f_sel(r.Y, c, a.Y, b.Y);
  f_sel(r.Z, c, a.Z, b.Z);
}

// Requires beta(X) <= 100, beta(Y) + beta(Z) <= 128. Output beta (34/66, 34, 34/4).
template <class F>
BH_HD void j_dbl(J30& r, const J30& p) {
  if constexpr (F::a_is_minus3) {
    uint32_t delta[9], gamma[9], bt[9], t0[9], t1[9], u[9], alpha[9];
    f_sqr<F>(delta, p.Z);                 // [b2]
    f_sqr<F>(gamma, p.Y);                 // [b2]
    f_mul<F>(bt, p.X, gamma);             // [b2]
    f_sub<F, 32>(t0, p.X, delta);         // [bX+32]
    f_add(t1, p.X, delta);                // [bX+2]
    f_mul<F>(u, t0, t1);                  // [b2]  (bX+32)(bX+2) <= 13464
    f_mulc<3>(alpha, u);                  // [b6]
    // Z3 = (Y + Z)^2 - gamma - delta
    f_add(t0, p.Y, p.Z);                  // [bY+bZ]
    f_sqr<F>(t0, t0);                     // [b2]
    f_sub2<F, 32>(r.Z, t0, gamma, delta); // [b34] (one pass)
    // X3 = alpha^2 - 8 beta
    f_sqr<F>(u, alpha);                   // [b2]  36
    f_mulc<8>(t0, bt);                    // [b16]
    f_sub<F, 32>(r.X, u, t0);             // [b34]
    // Y3 = alpha (4 beta - X3) - 8 gamma^2 = alpha (12 beta - alpha^2) - 8 gamma^2
    f_mulc<12>(t0, bt);                   // [b24]
    f_sub<F, 32>(t0, t0, u);              // [b56]
    f_mul<F>(t0, alpha, t0);              // [b2]  6*56
    f_sqr<F>(gamma, gamma);               // [b2]
    f_mulc<8>(gamma, gamma);              // [b16]
    f_sub<F, 32>(r.Y, t0, gamma);         // [b34]
  } else {
    // a = 0: A = X^2, B = Y^2, C = B^2, D = 2((X+B)^2 - A - C), E = 3A,
    // X3 = E^2 - 2D, Y3 = E(D - X3) - 8C = E(3D - E^2) - 8C, Z3 = 2 Y Z
    uint32_t A[9], B[9], Cc[9], D[9], E[9], t[9], t2[9];
    f_sqr<F>(A, p.X);                     // [b2]
    f_sqr<F>(B, p.Y);                     // [b2]
    f_mul<F>(t, p.Y, p.Z);                // [b2]  bY*bZ <= 16000
    f_sqr<F>(Cc, B);                      // [b2]
    f_add(t2, p.X, B);                    // [bX+2]
    f_sqr<F>(t2, t2);                     // [b2]
    f_mulc<2>(r.Z, t);                    // [b4]
    f_add(t, A, Cc);                      // [b4]
    f_sub<F, 32>(t2, t2, t);              // [b34]
    f_mulc<2>(D, t2);                     // [b68]
    f_mulc<3>(E, A);                      // [b6]
    f_sqr<F>(t, E);                       // [b2]  F = E^2
    f_mulc<3>(t2, D);                     // [b204]
    f_sub<F, 32>(t2, t2, t);              // [b236] 3D - F
    f_mulc<2>(D, D);                      // [b136] 2D
    // X3 = F - 2D: reduce 2D first (beta 136 > 63)
    f_reduce<F>(D, D);                    // [b1]
    f_sub<F, 32>(r.X, t, D);              // [b34]
    f_mul<F>(t, E, t2);                   // [b2]  6*236
    f_mulc<8>(Cc, Cc);                    // [b16]
    f_sub<F, 32>(r.Y, t, Cc);             // [b34]
  }
}

// Co-Z doubling (DBLU): r = 2p and pp = p rescaled to r's Z, i.e.
// (X (2Y)^2, Y (2Y)^3, 2YZ) = (4 X Y^2, 8 Y^4, Z3), both intermediates of the
// doubling. Requires beta(X) <= 63, beta(Y) + beta(Z) <= 128. Output r as
// j_dbl (a = -3: (34, 34, 34); a = 0: (34, 34, 4)); pp beta (8, 16) / (2, 16).
template <class F>
BH_HD void j_dblu(J30& r, J30& pp, const J30& p) {
  if constexpr (F::a_is_minus3) {
    uint32_t delta[9], gamma[9], bt[9], t0[9], t1[9], u[9], alpha[9];
    f_sqr<F>(delta, p.Z);                 // [b2]
    f_sqr<F>(gamma, p.Y);                 // [b2]
    f_mul<F>(bt, p.X, gamma);             // [b2]
    f_sub<F, 32>(t0, p.X, delta);         // [bX+32]
    f_add(t1, p.X, delta);                // [bX+2]
    f_mul<F>(u, t0, t1);                  // [b2]
    f_mulc<3>(alpha, u);                  // [b6]
    f_add(t0, p.Y, p.Z);                  // [bY+bZ]
    f_sqr<F>(t0, t0);                     // [b2]
    f_sub2<F, 32>(r.Z, t0, gamma, delta); // [b34]  2YZ (one pass)
    f_sqr<F>(u, alpha);                   // [b2]
    f_mulc<8>(t0, bt);                    // [b16]
    f_sub<F, 32>(r.X, u, t0);             // [b34]
    f_mulc<4>(pp.X, bt);                  // [b8]   4 X Y^2
    f_mulc<12>(t0, bt);                   // [b24]
    f_sub<F, 32>(t0, t0, u);              // [b56]
    f_mul<F>(t0, alpha, t0);              // [b2]
    f_sqr<F>(gamma, gamma);               // [b2]
    f_mulc<8>(pp.Y, gamma);               // [b16]  8 Y^4
    f_sub<F, 32>(r.Y, t0, pp.Y);          // [b34]
    f_copy(pp.Z, r.Z);
  } else {
    uint32_t A[9], B[9], Cc[9], D[9], E[9], t[9], t2[9];
    f_sqr<F>(A, p.X);                     // [b2]
    f_sqr<F>(B, p.Y);                     // [b2]
    f_mul<F>(t, p.Y, p.Z);                // [b2]
    f_sqr<F>(Cc, B);                      // [b2]
    f_add(t2, p.X, B);                    // [bX+2]
    f_sqr<F>(t2, t2);                     // [b2]
    f_mulc<2>(r.Z, t);                    // [b4]   2YZ
    f_add(t, A, Cc);                      // [b4]
    f_sub<F, 32>(t2, t2, t);              // [b34]
    f_mulc<2>(D, t2);                     // [b68]  D = 4 X Y^2
    f_reduce<F>(D, D);                    // [b1]
    f_copy(pp.X, D);                      // [b1]
    f_mulc<3>(E, A);                      // [b6]
    f_sqr<F>(t, E);                       // [b2]   F = E^2
    f_mulc<3>(t2, D);                     // [b3]
    f_sub<F, 32>(t2, t2, t);              // [b35]  3D - F
    f_mulc<2>(D, D);                      // [b2]
    f_sub<F, 32>(r.X, t, D);              // [b34]  X3 = F - 2D
    f_mul<F>(t, E, t2);                   // [b2]   6*35
    f_mulc<8>(pp.Y, Cc);                  // [b16]  8 Y^4
    f_sub<F, 32>(r.Y, t, pp.Y);           // [b34]
    f_copy(pp.Z, r.Z);
  }
}

// Co-Z addition (ZADDU, Meloni 2007): p, q share Z; r = p + q and p is
// rescaled in place to r's Z (5M + 2S instead of 12M + 4S). Requires
// beta(X1), beta(Y1) <= 64, beta(X2), beta(Y2) <= 63, beta(Z) <= 34.
// Output r beta (34, 34, 2), p beta (2, 2, 2). Incomplete: p = +-q is not
// detected (callers guarantee it cannot happen).
template <class F>
BH_HD void j_zaddu(J30& r, J30& p, const J30& q) {
  uint32_t t1[9], c[9], w1[9], w2[9], t2[9], d[9], t3[9];
  f_sub<F, 64>(t1, p.X, q.X);             // [b128]
  f_sqr<F>(c, t1);                        // [b2]   C = (X1 - X2)^2
  f_mul<F>(w1, p.X, c);                   // [b2]   W1 = X1 C
  f_mul<F>(w2, q.X, c);                   // [b2]   W2 = X2 C
  f_sub<F, 64>(t2, p.Y, q.Y);             // [b128]
  f_sqr<F>(d, t2);                        // [b2]   D = (Y1 - Y2)^2
  f_sub<F, 32>(t3, w1, w2);               // [b34]
  f_mul<F>(p.Y, p.Y, t3);                 // [b2]   A1 = Y1 (W1 - W2)
  f_sub2<F, 32>(r.X, d, w1, w2);          // [b34]  X3 = D - W1 - W2 (one pass)
  f_sub<F, 64>(t3, w1, r.X);              // [b66]
  f_mul<F>(t3, t2, t3);                   // [b2]   128*66
  f_sub<F, 32>(r.Y, t3, p.Y);             // [b34]  Y3 = (Y1 - Y2)(W1 - X3) - A1
  f_mul<F>(r.Z, p.Z, t1);                 // [b2]   Z3 = Z (X1 - X2): 34*128
  f_copy(p.X, w1);                        // [b2]
  f_copy(p.Z, r.Z);
}

// Degenerate-case resolution shared by the additions: called only when Z3 is
// 0 mod p (x1 == x2); same_y from the canonical r = S2 - S1.
template <class F>
BH_HD bool j_degenerate(const uint32_t z3[9], const uint32_t rr[9], bool* same_y) {
  const bool degenerate = f_is_zero2<F>(z3);
  if (degenerate) {  // rare: decide double vs infinity on the canonical r
    uint32_t t[9];
    f_reduce<F>(t, rr);
    uint32_t z = 0;
    for (int i = 0; i < 9; i++) z |= t[i];
    *same_y = (z == 0);
  } else {
    *same_y = false;
  }
  return degenerate;
}

// r = p + (+-q) (Jacobian, neither at infinity; neg adds -q: q's sign folded
// into r = S2 - S1, f_csub). With CO, pz = p rescaled to r's Z, (U1 H^2,
// S1 H^3, Z3) -- both intermediates of the addition, the co-Z partner j_zaddu
// needs for 2 p + q = (p + q) + p. Requires beta <= 63 on X1, Y1, X2, Y2 and
// beta <= 34 on Z1, Z2 (products below stay <= 16000). Output beta (34, 34,
// 2), pz (2, 2, 2). Returns true iff x(p) == x(q) (degenerate); then r is
// garbage and *same_y says p == +-q (double) vs p == -(+-q) (infinity). r may
// alias p. Round 6: H^3 + 2V once (f_add2x), X3 and V - X3 from it in one
// pass each (was five passes), the sign in the r pass (was a negation + select).
template <class F, bool CO>
BH_HD bool j_add_impl(J30& r, J30* pz, const J30& p, const J30& q, bool neg, bool* same_y) {
  uint32_t z1z1[9], z2z2[9], u1[9], u2[9], s1[9], s2[9], h[9], rr[9], t[9], hh[9], hhh[9], w[9];
  f_sqr<F>(z1z1, p.Z);                    // [b2]
  f_sqr<F>(z2z2, q.Z);                    // [b2]
  f_mul<F>(u1, p.X, z2z2);                // [b2]
  f_mul<F>(u2, q.X, z1z1);                // [b2]
  f_mul<F>(t, q.Z, z2z2);                 // [b2]
  f_mul<F>(s1, p.Y, t);                   // [b2]
  f_mul<F>(t, p.Z, z1z1);                 // [b2]
  f_mul<F>(s2, q.Y, t);                   // [b2]
  f_sub<F, 32>(h, u2, u1);                // [b34]
  f_csub<F, 32>(rr, neg, s2, s1);         // [b34]  +-S2 - S1
  f_sqr<F>(hh, h);                        // [b2]
  f_mul<F>(hhh, hh, h);                   // [b2]
  f_mul<F>(u1, u1, hh);                   // [b2]  V = U1 H^2
  f_sqr<F>(t, rr);                        // [b2]  r^2
  f_add2x(w, hhh, u1);                    // [b6]  H^3 + 2V
  f_sub<F, 32>(r.X, t, w);                // [b34] X3 = r^2 - H^3 - 2V
  f_addsub<F, 32>(u2, w, u1, t);          // [b40] V - X3 = 3V + H^3 - r^2
  f_mul<F>(u2, rr, u2);                   // [b2]  34*40
  f_mul<F>(s1, s1, hhh);                  // [b2]  S1 H^3
  f_sub<F, 32>(r.Y, u2, s1);              // [b34] Y3 = r (V - X3) - S1 H^3
  f_mul<F>(t, p.Z, q.Z);                  // [b2]
  f_mul<F>(r.Z, t, h);                    // [b2]  Z3 = Z1 Z2 H
  if constexpr (CO) {
    f_copy(pz->X, u1);
    f_copy(pz->Y, s1);
    f_copy(pz->Z, r.Z);
  }
  return j_degenerate<F>(r.Z, rr, same_y);
}

template <class F>
BH_HD bool j_add(J30& r, const J30& p, const J30& q, bool* same_y) {
  return j_add_impl<F, false>(r, nullptr, p, q, false, same_y);
}
template <class F>
BH_HD bool j_add_co(J30& r, J30& pz, const J30& p, const J30& q, bool* same_y, bool neg = false) {
  return j_add_impl<F, true>(r, &pz, p, q, neg, same_y);
}

// r = p + (x2, +-y2, 1) (mixed; neg adds (x2, -y2)). Requires beta <= 63 on X1
// and beta <= 94 on Y1 (the sign pass needs S2 + Y1 <= 96 p; a point whose y
// was negated by f_neg<64> has beta 64), beta(Z1) <= 34, beta(x2),
// beta(y2) <= 64. Output beta (34, 34, 2); with CO, pz = (X1 H^2, Y1 H^3, Z3) beta
// (2, 2, 2) (j_madd_co: the composite 2 p + q = (p + q) + p). Degenerate
// contract as j_add_impl; r may alias p.
template <class F, bool CO>
BH_HD bool j_madd_impl(J30& r, J30* pz, const J30& p, const uint32_t x2[9], const uint32_t y2[9],
                       bool neg, bool* same_y) {
  uint32_t z1z1[9], u2[9], s2[9], h[9], rr[9], t[9], hh[9], hhh[9], v[9], w[9];
  f_sqr<F>(z1z1, p.Z);                    // [b2]
  f_mul<F>(u2, x2, z1z1);                 // [b2]
  f_mul<F>(t, p.Z, z1z1);                 // [b2]
  f_mul<F>(s2, y2, t);                    // [b2]
  f_sub<F, 64>(h, u2, p.X);               // [b66]
  f_csub<F, 96>(rr, neg, s2, p.Y);        // [b98]  +-S2 - Y1 (96 p: Y1 may be a negated
                                          // table y, < 64 p, and S2 < 2 p)
  f_sqr<F>(hh, h);                        // [b2]  4356
  f_mul<F>(hhh, hh, h);                   // [b2]
  f_mul<F>(v, p.X, hh);                   // [b2]  V = X1 H^2
  f_sqr<F>(t, rr);                        // [b2]  9604
  f_add2x(w, hhh, v);                     // [b6]  H^3 + 2V
  f_sub<F, 32>(r.X, t, w);                // [b34] X3 = r^2 - H^3 - 2V
  f_addsub<F, 32>(s2, w, v, t);           // [b40] V - X3
  f_mul<F>(s2, rr, s2);                   // [b2]  98*40
  f_mul<F>(t, p.Y, hhh);                  // [b2]  Y1 H^3
  f_sub<F, 32>(r.Y, s2, t);               // [b34]
  f_mul<F>(r.Z, p.Z, h);                  // [b2]  34*66
  if constexpr (CO) {
    f_copy(pz->X, v);
    f_copy(pz->Y, t);
    f_copy(pz->Z, r.Z);
  }
  return j_degenerate<F>(r.Z, rr, same_y);
}

template <class F>
BH_HD bool j_madd(J30& r, const J30& p, const uint32_t x2[9], const uint32_t y2[9], bool* same_y,
                  bool neg = false) {
  return j_madd_impl<F, false>(r, nullptr, p, x2, y2, neg, same_y);
}
template <class F>
BH_HD bool j_madd_co(J30& r, J30& pz, const J30& p, const uint32_t x2[9], const uint32_t y2[9],
                     bool* same_y, bool neg = false) {
  return j_madd_impl<F, true>(r, &pz, p, x2, y2, neg, same_y);
}

// y^2 == x^3 + a x + b for Montgomery-domain x, y with beta <= 2.
template <class F>
BH_HD bool j_on_curve(const uint32_t x[9], const uint32_t y[9]) {
  uint32_t l[9], rhs[9], t[9], b[9];
  f_sqr<F>(l, y);                         // [b2]
  f_sqr<F>(t, x);                         // [b2]
  f_mul<F>(rhs, t, x);                    // [b2]
  if constexpr (F::a_is_minus3) {
    f_mulc<3>(t, x);                      // [b6]
    f_sub<F, 32>(rhs, rhs, t);            // [b34]
  }
  f_const(b, F::b_m);
  f_add(rhs, rhs, b);                     // [b35]
  f_reduce<F>(rhs, rhs);
  f_canon<F>(l, l);
  return f_eq(l, rhs);
}

}  // namespace bh
