// Go-exact DER decoding of an ECDSA signature SEQUENCE { r INTEGER, s INTEGER }.
//
// Restates bccsp/utils/ecdsa.go:41-65 UnmarshalECDSASignature, i.e.
// encoding/asn1.Unmarshal(raw, &struct{R, S *big.Int}) from Go 1.21.4 (pinned
// by the reference Makefile:81) followed by the R > 0, S > 0 checks:
//   * parseTagAndLength: high-tag-number form, no indefinite length, long-form
//     lengths minimal (no leading 0x00, value >= 0x80), "length too large" at
//     >= 2^23 before each shift;
//   * the SEQUENCE must be universal/constructed/tag 16 (0x30), each INTEGER
//     universal/primitive/tag 2 (0x02), non-empty and minimally encoded
//     (checkInteger);
//   * extra elements after S inside the SEQUENCE and trailing bytes after the
//     SEQUENCE are ACCEPTED (asn1 parseField / Unmarshal returns `rest`).
// Pinned by the reference's fixed vectors bccsp/sw/impl_test.go:924-961 and
// bccsp/utils/ecdsa_test.go:19-62 (tests/golden/p256_vectors.jsonl).
//
// Compiled for the device (each lane parses its own signature out of HBM) and
// for the host (bh_parse_der_sig in the C-ABI).
#pragma once
#include "bh_common.h"

namespace bh {

struct DerSig {
  uint32_t r[8], s[8];  // magnitudes (little-endian limbs) when <= 256 bits
  uint32_t r_big, s_big;  // 1 if the magnitude exceeds 32 bytes
};

// Returns 0 on success.
BH_HD int der_tag_len(const uint8_t* b, uint32_t n, uint32_t* off, uint32_t* cls,
                      uint32_t* cmp, uint32_t* tag, uint32_t* len) {
  if (*off >= n) return -1;
  uint32_t t = b[(*off)++];
  *cls = t >> 6;
  *cmp = (t >> 5) & 1u;
  *tag = t & 0x1fu;
  if (*tag == 0x1fu) {  // parseBase128Int
    uint64_t v = 0;
    uint32_t shifted = 0;
    for (;;) {
      if (*off >= n) return -1;
      if (shifted == 5) return -1;
      uint32_t x = b[*off];
      if (shifted == 0 && x == 0x80u) return -1;
      v = (v << 7) | (x & 0x7fu);
      (*off)++;
      shifted++;
      if (!(x & 0x80u)) break;
    }
    if (v > 0x7fffffffull || v < 0x1full) return -1;
    *tag = (uint32_t)v;
  }
  if (*off >= n) return -1;
  uint32_t lb = b[(*off)++];
  if (!(lb & 0x80u)) {
    *len = lb & 0x7fu;
    return 0;
  }
  uint32_t nb = lb & 0x7fu;
  if (nb == 0) return -1;  // indefinite length
  uint32_t L = 0;
  for (uint32_t i = 0; i < nb; i++) {
    if (*off >= n) return -1;
    uint32_t x = b[(*off)++];
    if (L >= (1u << 23)) return -1;  // length too large
    L = (L << 8) | x;
    if (L == 0) return -1;  // superfluous leading zeros
  }
  if (L < 0x80u) return -1;  // non-minimal length
  *len = L;
  return 0;
}

// parseField for a *big.Int. sign: -1/0/+1. For positive values fills the
// magnitude limbs (or *big = 1).
BH_HD int der_int(const uint8_t* b, uint32_t n, uint32_t* off, int* sign, uint32_t mag[8],
                  uint32_t* big) {
  if (*off == n) return -1;  // sequence truncated
  uint32_t cls, cmp, tag, len;
  if (der_tag_len(b, n, off, &cls, &cmp, &tag, &len)) return -1;
  if (cls != 0 || tag != 2 || cmp) return -1;
  if ((uint64_t)*off + len > n) return -1;  // data truncated
  const uint32_t start = *off;
  *off += len;
  if (len == 0) return -1;  // empty integer
  const uint32_t b0 = b[start];
  if (len > 1) {
    const uint32_t b1 = b[start + 1];
    if ((b0 == 0 && !(b1 & 0x80u)) || (b0 == 0xffu && (b1 & 0x80u))) return -1;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) mag[i] = 0;
  *big = 0;
  if (b0 & 0x80u) {
    *sign = -1;
    return 0;
  }
  if (len == 1 && b0 == 0) {
    *sign = 0;
    return 0;
  }
  *sign = 1;
  uint32_t s0 = start + (b0 == 0 ? 1u : 0u);
  uint32_t L = start + len - s0;
  if (L > 32) {
    *big = 1;
    return 0;
  }
  // right-align the L magnitude bytes into 32 big-endian byte slots
  const uint32_t end = start + len;  // one past the last byte
#pragma unroll
  for (int j = 0; j < 32; j++) {  // j = byte index from the least significant end
    uint32_t v = 0;
    if ((uint32_t)j < L) v = b[end - 1 - j];
    mag[j >> 2] |= v << (8 * (j & 3));
  }
  return 0;
}

// Returns R_OK, R_DER, R_R_NONPOS or R_S_NONPOS (bccsp/utils/ecdsa.go:41-65).
BH_HD uint8_t der_parse_sig(const uint8_t* b, uint32_t n, DerSig* o) {
  uint32_t off = 0, cls, cmp, tag, len;
  if (n == 0) return R_DER;
  if (der_tag_len(b, n, &off, &cls, &cmp, &tag, &len)) return R_DER;
  if (cls != 0 || tag != 16 || !cmp) return R_DER;
  if ((uint64_t)off + len > n) return R_DER;
  const uint8_t* in = b + off;
  uint32_t io = 0;
  int rs = 0, ss = 0;
  if (der_int(in, len, &io, &rs, o->r, &o->r_big)) return R_DER;
  if (der_int(in, len, &io, &ss, o->s, &o->s_big)) return R_DER;
  if (rs <= 0) return R_R_NONPOS;
  if (ss <= 0) return R_S_NONPOS;
  return R_OK;
}

}  // namespace bh
