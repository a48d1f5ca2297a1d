// Jacobian-coordinate point arithmetic over a short-Weierstrass curve, all
// coordinates in the Montgomery domain of the base field.
//
// Replaces the point layer of Go's crypto/internal/nistec P-256 (ScalarMult /
// ScalarBaseMult / Add reached from crypto/ecdsa verifyNISTEC, called at
// bccsp/sw/ecdsa.go:56) and btcec's addJacobian/doubleJacobian
// (vendor/github.com/BDLS-bft/bdls/crypto/btcec/btcec.go:461-482, 765-887).
//
// Formulas (EFD, hyperelliptic.org/EFD/g1p/auto-shortw-jacobian*.html):
//   dbl  a = -3 : dbl-2001-b        3M + 5S
//   dbl  a =  0 : dbl-2009-l        2M + 5S
//   add         : add-1998-cmo-2   12M + 4S
//   madd (Z2=1) : madd-1998-cmo     8M + 3S
// The add formulas are incomplete: they report H == 0 (equal x) to the caller,
// which resolves doubling / infinity explicitly (see the ladder in verify.hip).
#pragma once
#include "fe.h"

namespace bh {

struct Jac {
  uint32_t X[8], Y[8], Z[8];
};

template <class F, class C>
BH_HD void pt_dbl(Jac& r, const Jac& p) {
  if constexpr (C::a_is_minus3) {
    uint32_t delta[8], gamma[8], beta[8], alpha[8], t0[8], t1[8];
    mont_sqr<F>(delta, p.Z);
    mont_sqr<F>(gamma, p.Y);
    mont_mul<F>(beta, p.X, gamma);
    mod_sub<F>(t0, p.X, delta);
    mod_add<F>(t1, p.X, delta);
    mont_mul<F>(t0, t0, t1);
    mod_add<F>(alpha, t0, t0);
    mod_add<F>(alpha, alpha, t0);  // alpha = 3 (X - delta)(X + delta)
    // Z3 = (Y + Z)^2 - gamma - delta
    mod_add<F>(t1, p.Y, p.Z);
    mont_sqr<F>(t1, t1);
    mod_sub<F>(t1, t1, gamma);
    mod_sub<F>(r.Z, t1, delta);
    // X3 = alpha^2 - 8 beta
    mod_add<F>(beta, beta, beta);
    mod_add<F>(beta, beta, beta);  // 4 beta
    mont_sqr<F>(t0, alpha);
    mod_add<F>(t1, beta, beta);    // 8 beta
    mod_sub<F>(r.X, t0, t1);
    // Y3 = alpha (4 beta - X3) - 8 gamma^2
    mod_sub<F>(t0, beta, r.X);
    mont_mul<F>(t0, alpha, t0);
    mont_sqr<F>(gamma, gamma);
    mod_add<F>(gamma, gamma, gamma);
    mod_add<F>(gamma, gamma, gamma);
    mod_add<F>(gamma, gamma, gamma);
    mod_sub<F>(r.Y, t0, gamma);
  } else {
    // a = 0: A = X^2, B = Y^2, C = B^2, D = 2((X+B)^2 - A - C), E = 3A,
    // X3 = E^2 - 2D, Y3 = E(D - X3) - 8C, Z3 = 2 Y Z
    uint32_t A[8], B[8], Cc[8], D[8], E[8], t[8];
    mont_sqr<F>(A, p.X);
    mont_sqr<F>(B, p.Y);
    mont_mul<F>(t, p.Y, p.Z);
    mod_add<F>(r.Z, t, t);
    mont_sqr<F>(Cc, B);
    mod_add<F>(t, p.X, B);
    mont_sqr<F>(t, t);
    mod_sub<F>(t, t, A);
    mod_sub<F>(t, t, Cc);
    mod_add<F>(D, t, t);
    mod_add<F>(E, A, A);
    mod_add<F>(E, E, A);
    mont_sqr<F>(t, E);
    mod_sub<F>(t, t, D);
    mod_sub<F>(r.X, t, D);
    mod_sub<F>(t, D, r.X);
    mont_mul<F>(t, E, t);
    mod_add<F>(Cc, Cc, Cc);
    mod_add<F>(Cc, Cc, Cc);
    mod_add<F>(Cc, Cc, Cc);
    mod_sub<F>(r.Y, t, Cc);
  }
}

// r = p + q (both Jacobian, neither infinity). Returns true iff H == 0, i.e.
// x(p) == x(q); then *same_y tells p == q (caller must double) vs p == -q
// (result is infinity). r is garbage when true is returned.
template <class F>
BH_HD bool pt_add(Jac& r, const Jac& p, const Jac& q, bool* same_y) {
  uint32_t z1z1[8], z2z2[8], u1[8], u2[8], s1[8], s2[8], h[8], rr[8], t[8], hh[8], hhh[8];
  mont_sqr<F>(z1z1, p.Z);
  mont_sqr<F>(z2z2, q.Z);
  mont_mul<F>(u1, p.X, z2z2);
  mont_mul<F>(u2, q.X, z1z1);
  mont_mul<F>(t, q.Z, z2z2);
  mont_mul<F>(s1, p.Y, t);
  mont_mul<F>(t, p.Z, z1z1);
  mont_mul<F>(s2, q.Y, t);
  mod_sub<F>(h, u2, u1);
  mod_sub<F>(rr, s2, s1);
  bool degenerate = is_zero8(h);
  *same_y = is_zero8(rr);
  mont_sqr<F>(hh, h);
  mont_mul<F>(hhh, hh, h);
  mont_mul<F>(u1, u1, hh);  // U1 H^2
  mont_sqr<F>(t, rr);
  mod_sub<F>(t, t, hhh);
  mod_sub<F>(t, t, u1);
  mod_sub<F>(r.X, t, u1);   // X3 = r^2 - H^3 - 2 U1 H^2
  mod_sub<F>(t, u1, r.X);
  mont_mul<F>(t, rr, t);
  mont_mul<F>(s1, s1, hhh);
  mod_sub<F>(r.Y, t, s1);   // Y3 = r (U1 H^2 - X3) - S1 H^3
  mont_mul<F>(t, p.Z, q.Z);
  mont_mul<F>(r.Z, t, h);   // Z3 = Z1 Z2 H
  return degenerate;
}

// r = p + (qx, qy, 1). Same degenerate-case contract as pt_add.
template <class F>
BH_HD bool pt_madd(Jac& r, const Jac& p, const uint32_t qx[8], const uint32_t qy[8],
                   bool* same_y) {
  uint32_t z1z1[8], u2[8], s2[8], h[8], rr[8], t[8], hh[8], hhh[8];
  mont_sqr<F>(z1z1, p.Z);
  mont_mul<F>(u2, qx, z1z1);
  mont_mul<F>(t, p.Z, z1z1);
  mont_mul<F>(s2, qy, t);
  mod_sub<F>(h, u2, p.X);
  mod_sub<F>(rr, s2, p.Y);
  bool degenerate = is_zero8(h);
  *same_y = is_zero8(rr);
  mont_sqr<F>(hh, h);
  mont_mul<F>(hhh, hh, h);
  mont_mul<F>(u2, p.X, hh);  // X1 H^2
  mont_sqr<F>(t, rr);
  mod_sub<F>(t, t, hhh);
  mod_sub<F>(t, t, u2);
  mod_sub<F>(r.X, t, u2);
  mod_sub<F>(t, u2, r.X);
  mont_mul<F>(t, rr, t);
  mont_mul<F>(s2, p.Y, hhh);
  mod_sub<F>(r.Y, t, s2);
  mont_mul<F>(r.Z, p.Z, h);
  return degenerate;
}

BH_HD void jac_copy(Jac& r, const Jac& p) {
  copy8(r.X, p.X);
  copy8(r.Y, p.Y);
  copy8(r.Z, p.Z);
}

BH_HD void jac_sel(Jac& r, bool c, const Jac& a, const Jac& b) {
  sel8(r.X, c, a.X, b.X);
  sel8(r.Y, c, a.Y, b.Y);
  sel8(r.Z, c, a.Z, b.Z);
}

// y^2 == x^3 + a x + b (Montgomery-domain affine x, y)
template <class F, class C>
BH_HD bool on_curve(const uint32_t x[8], const uint32_t y[8]) {
  uint32_t l[8], rhs[8], t[8], b[8];
  mont_sqr<F>(l, y);
  mont_sqr<F>(t, x);
  mont_mul<F>(rhs, t, x);
  if constexpr (C::a_is_minus3) {
    mod_sub<F>(rhs, rhs, x);
    mod_sub<F>(rhs, rhs, x);
    mod_sub<F>(rhs, rhs, x);
  }
  load_const8(b, C::b_m);
  mod_add<F>(rhs, rhs, b);
  return eq8(l, rhs);
}

}  // namespace bh
