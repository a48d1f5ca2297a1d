// Per-record stages of the batched ECDSA verify pipeline (P-256 / secp256k1).
//
//   stage_prep   : CSP.Verify arg checks, Go-exact DER parse, low-S, key and r
//                  range / on-curve checks, digest (fused SHA-256 or given),
//                  e = hashToNat, Montgomery conversions.        (1 lane/record)
//   stage_inv    : w = s^-1 mod n by Montgomery's batch trick over a set of
//                  records, u1 = e w, u2 = r w.               (1 lane/chunk)
//   stage_ladder : Q table, signed-window (Booth w=5) ladder for u2 Q, fixed-base
//                  comb (kGW-bit signed windows) for u1 G, final add, projective
//                  x == r (or r + n) check.                   (1 lane/record)
//
// Reference semantics restated (see DESIGN.md for the full contract):
//   bccsp/sw/impl.go:247-270, bccsp/sw/ecdsa.go:41-57, bccsp/utils/ecdsa.go:41-89,
//   Go 1.21.4 crypto/ecdsa verifyNISTEC/hashToNat/pointFromAffine.
// All intermediate records live in HBM as structure-of-arrays (8 u32 limbs per
// value, limb-major with stride `ns`), so every per-limb access by a wave is one
// coalesced 256-byte transaction.
#pragma once
#include <type_traits>

#include "blake2b.h"
#include "der.h"
#include "fe.h"
#include "ec30.h"
#include "sha256.h"
#include "sha3.h"

namespace bh {

enum : uint32_t {
  BHF_HASH_SHA256 = 1u,    // msg is a message: digest = SHA-256(msg) (identity.Verify)
  BHF_NO_LOW_S = 2u,       // skip Fabric's low-S rule (plain Go ecdsa.Verify semantics)
  BHF_HASH_SHA3_256 = 8u,  // msg is a message: digest = SHA3-256(msg) (SHA3 hash family)
};

// Digest source of a verify record (compile-time, one k_prep instantiation each).
enum : int { HK_GIVEN_OR_SHA256 = 0, HK_SHA3_256 = 1 };

// Status byte kept per record between stages: low 7 bits = reason, bit 7 = r+n < p.
enum : uint8_t { ST_R2OK = 0x80u };

struct BatchIn {  // device pointers (see include/bdls_hip.h bh_batch)
  const uint8_t* pub;
  const uint8_t* sig;
  const uint64_t* sig_off;
  const uint32_t* sig_len;
  const uint8_t* msg;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  uint32_t flags;
  // optional second message span (bh_verify_2seg): message i is
  // msg[msg_off, +msg_len) || msg[msg2_off, +msg2_len); nullptr = one span
  const uint64_t* msg2_off = nullptr;
  const uint32_t* msg2_len = nullptr;
};

// BDLS consensus messages: vendor/github.com/BDLS-bft/bdls/message.go SignedProto
// fields (device pointers; see include/bdls_hip.h bh_bdls_batch).
struct BdlsIn {
  const uint8_t* xy;  // n * 64: X || Y (PubKeyAxis, 32 B each)
  const uint8_t* r;
  const uint64_t* r_off;
  const uint32_t* r_len;
  const uint8_t* s;
  const uint64_t* s_off;
  const uint32_t* s_len;
  const uint32_t* version;
  const uint8_t* msg;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  uint32_t flags;
};

struct Work {
  uint32_t ns;      // SoA stride in records (multiple of 64)
  uint32_t* e;      // [8][ns]  e, then u1
  uint32_t* r;      // [8][ns]  r, then u2
  uint32_t* sm;     // [8][ns]  s * R mod n
  uint32_t* pre;    // [8][ns]  batch-inversion prefix products
  uint32_t* qx;     // [9][ns]  Q.x * 2^270 mod p (radix 2^30, canonical)
  uint32_t* qy;     // [9][ns]
  uint32_t* rm;     // [9][ns]  r * 2^270 mod p (canonical)
  uint32_t* r2m;    // [9][ns]  (r + n) * 2^270 mod p   (valid iff ST_R2OK)
  uint8_t* st;      // [ns]
  uint32_t* qtab;   // [ns/64][64 lanes][16][28]  per-lane Q multiples 1..16 (Jacobian, radix 2^30)
  uint32_t* gpart;  // [28][ns]  u1 G of key-comb list position j (X, Y, Z, infinity flag)
};

// Per-batch key plan (device): open-addressed fingerprint table for key
// dedup, per-record slot, work lists and per-key comb tables.
struct Plan {
  uint32_t hc;          // fingerprint table capacity (power of two >= 2 n)
  uint32_t max_tables;  // key tables available
  uint64_t* slot_hash;  // [hc] 0 = empty
  uint32_t* slot_rep;   // [hc] smallest record index with this fingerprint
  uint32_t* slot_cnt;   // [hc] records verified equal to the representative key
  uint32_t* slot_tab;   // [hc] key-table index or kNone
  uint32_t* rec_slot;   // [ns] slot or kNone
  uint32_t* comb_list;  // [ns] records on the key-comb path (k_split order)
  uint32_t* comb_order; // the comb list k_keycomb reads: comb_list, or its
                        // key-sorted copy (comb_sort; stored in rec_slot's
                        // buffer, which is dead from then on)
  uint32_t* ladder_list;  // [ns] records on the variable-base ladder path
  uint32_t* counters;   // [0] n_comb, [1] n_ladder, [2] table builds
  uint32_t* rec_tab;    // [ns] table id of the record's key (kNone: ladder)
  uint32_t* tab_rec;    // [max_tables] record whose Q builds the table
  uint32_t* tab_dst;    // [max_tables] table id the build writes
  uint32_t* tables;     // [max_tables][kKWin][kKEnt][kQPt]  per-batch tables
};
constexpr uint32_t kNone = 0xffffffffu;

// Per-launch choices made on the host (bdls_hip.cpp run_dev).
struct LaunchOpts {
  uint32_t inv_chunk;  // records per batch-inversion lane
  uint32_t min_uses;   // key-table threshold (uses of one key in the batch)
  uint32_t min_batch;  // no per-batch tables below this batch size
  bool keep;           // BH_F_KEEP_KEYS: new tables go to the key registry
  int wide;            // lanes per record on the key-table path (1, 4, 16)
  uint32_t wide_block = 256;  // threads per workgroup of the multi-lane kernels
  // BDLS batches: the BLAKE2b digests run on a second stream (hipStream_t)
  // beside prep / inverse / plan / the u2 Q halves; fork and join are
  // hipEvent_t. Opaque here so the host harness compiles this header.
  void* aux = nullptr;
  void* ev_fork = nullptr;
  void* ev_join = nullptr;
  // Two compute lanes (bdls_hip.cpp Lane1): the table-build kernel waits for
  // the other lane's last build (build_wait) and marks its own end
  // (build_done), so the two lanes' chain-bound builds alternate and each runs
  // beside the other lane's key comb instead of beside its build.
  void* ev_build_wait = nullptr;
  void* ev_build_done = nullptr;
  // per-batch key tables of one-lane-per-record batches as Lim-Lee combs
  // (verify.h lltab_build; BH_LL=0 keeps the 4-bit windows everywhere)
  bool ll_tables = true;
  // Host batches (round 5): the keys arrive before the signatures and
  // messages. With this hipEvent_t set, the pass runs its key half (key
  // import, plan, table builds) first and waits for the event -- the rest of
  // the batch uploaded -- only before prep; otherwise it waits up front.
  void* records_ready = nullptr;
};

// Lanes per record on the key-table path by batch size (records far below
// chip size are spread over 16 or 4 lanes; the secp256k1 ladder then runs on
// 2 lanes per record).
constexpr uint32_t kWide16Max = 8192, kWide4Max = 32768;
BH_HD int wide_for(size_t m) { return m <= kWide16Max ? 16 : m <= kWide4Max ? 4 : 1; }
// Partial-sum slots of w.gpart: one per record (stage_gpart), or for wide
// batches the split kernels' ladder pairs [0, 2 ns) + key-comb groups
// [2 ns, (2 + wide) ns).
BH_HD size_t gpart_slots(size_t ns) {
  const int wide = wide_for(ns);
  return wide > 1 ? (2 + (size_t)wide) * ns : ns;
}

// G comb table: kGW-bit signed windows. Window w in [0, kCombWindows), entry
// j in [0, kCombEntries): (j+1) * 2^(kGW w) * G, affine, canonical radix-2^30
// Montgomery x (limbs 0..8) and y (limbs 9..17), padded to kGEntry words.
// kGW = 13 (round 4): 20 windows x 4,096 entries x 72 B = 5.9 MB per curve
// (L2 + MALL); same-box A/B at config 2 (profiles/r04/v4): HBM-resident
// 140.0-142.5 M verifies/s at 10 bits (26 windows, 958 KB), 144.2-146.5 at 12,
// 146.8-148.3 at 13, 147.2-148.2 at 14 (19 windows, 11.2 MB).
#ifndef BH_GCOMB_BITS
#define BH_GCOMB_BITS 13
#endif
constexpr int kGW = BH_GCOMB_BITS;
static_assert(kGW >= 8 && kGW <= 14, "G comb window width");
// digits of k + M (M = sum 2^(kGW-1) 2^(kGW w)) minus 2^(kGW-1) are k's signed
// digits in [-2^(kGW-1), 2^(kGW-1)); k < 2^256 needs kGW * windows >= 257.
constexpr int kCombWindows = (257 + kGW - 1) / kGW;
constexpr int kCombEntries = 1 << (kGW - 1);
static_assert(kCombWindows * kGW <= 288, "recoded scalar fits 9 limbs");
constexpr int kGEntry = 18;
constexpr int kQTab = 16;
constexpr int kQPt = 28;  // words per Jacobian point in the Q table (27 + pad)

struct alignas(16) W4 {
  uint32_t x, y, z, w;
};

// Per-record scalars / field elements (e, r, s, prefixes: 8 words; Q, r R,
// (r + n) R: 9 words). BH_AOS (default): record-major, a record's limbs
// contiguous -- consecutive lanes still write consecutive bytes (prep, the
// inverse), and the key-grouped and ladder kernels, whose lanes take records
// in list order (scattered indices), read each record from one or two cache
// lines instead of one line per limb. Otherwise limb-major (stride ns).
#ifndef BH_AOS
#define BH_AOS 1
#endif
BH_HD void ld8(uint32_t v[8], const uint32_t* base, uint32_t i, uint32_t ns) {
#if BH_AOS
  const W4* p = reinterpret_cast<const W4*>(base + (size_t)i * 8);
  const W4 a = p[0], b = p[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#else
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = base[(size_t)k * ns + i];
#endif
}
BH_HD void st8(uint32_t* base, uint32_t i, uint32_t ns, const uint32_t v[8]) {
#if BH_AOS
  W4* p = reinterpret_cast<W4*>(base + (size_t)i * 8);
  p[0] = W4{v[0], v[1], v[2], v[3]};
  p[1] = W4{v[4], v[5], v[6], v[7]};
#else
#pragma unroll
  for (int k = 0; k < 8; k++) base[(size_t)k * ns + i] = v[k];
#endif
}
BH_HD void ld9(uint32_t v[9], const uint32_t* base, uint32_t i, uint32_t ns) {
#pragma unroll
  for (int k = 0; k < 9; k++) v[k] = BH_AOS ? base[(size_t)i * 9 + k] : base[(size_t)k * ns + i];
}
BH_HD void st9(uint32_t* base, uint32_t i, uint32_t ns, const uint32_t v[9]) {
#pragma unroll
  for (int k = 0; k < 9; k++) (BH_AOS ? base[(size_t)i * 9 + k] : base[(size_t)k * ns + i]) = v[k];
}

// ------------------------------------------------------------------ prep
// Public key bytes X || Y (32 B big-endian each) -> canonical radix-2^30
// Montgomery coordinates; false unless 0 <= X, Y < p and Y^2 = X^3 + aX + b
// (Go pointFromAffine, crypto/ecdsa verifyNISTEC).
template <class P, class C>
BH_HD bool key_import(const uint8_t* q, uint32_t qx30[9], uint32_t qy30[9]) {
  uint32_t qx[8], qy[8], pp[8];
  load_const8(pp, C::p);
  be32_to_limbs(qx, q);
  be32_to_limbs(qy, q + 32);
  if (geq8(qx, pp) || geq8(qy, pp)) return false;
  f_from_u256(qx30, qx);
  f_from_u256(qy30, qy);
  f_to_mont<P>(qx30, qx30);
  f_to_mont<P>(qy30, qy30);
  f_canon<P>(qx30, qx30);
  f_canon<P>(qy30, qy30);
  return j_on_curve<P>(qx30, qy30);
}

// The key half of prep for a pass that plans and builds before its
// signatures / messages arrive (LaunchOpts::records_ready): Q imported as in
// stage_prep, st = R_OK or R_BAD_KEY (stage_prep rewrites both later; a record
// whose signature then fails keeps its key's place in the plan, which only
// decides which tables are built).
template <class P, class C>
BH_HD void stage_prep_key(const BatchIn& in, const Work& w, uint32_t i) {
  uint32_t qx30[9], qy30[9];
  const bool ok = key_import<P, C>(in.pub + (size_t)i * 64, qx30, qy30);
  if (!ok) {
    f_const(qx30, P::gx_m);
    f_const(qy30, P::gy_m);
  }
  st9(w.qx, i, w.ns, qx30);
  st9(w.qy, i, w.ns, qy30);
  w.st[i] = ok ? (uint8_t)R_OK : (uint8_t)R_BAD_KEY;
}

// e = hashToNat(digest) mod n for record i: the given digest, or the fused
// SHA-256 / SHA3-256 of its (one- or two-span) message.
template <class C, int HK>
BH_HD void digest_e(const BatchIn& in, uint32_t i, uint32_t e[8]) {
  const uint32_t mlen = in.msg_len[i];
  const bool fused = HK == HK_SHA3_256 || (in.flags & BHF_HASH_SHA256) != 0;
  const uint8_t* m = in.msg + in.msg_off[i];
  const uint32_t mlen2 = in.msg2_len ? in.msg2_len[i] : 0u;  // fused modes only
  if constexpr (HK == HK_SHA3_256) {
    uint8_t hb[32];
    if (mlen2) sha3_256_msg2(hb, m, mlen, in.msg + in.msg2_off[i], mlen2);
    else sha3_256_msg(hb, m, mlen);
    be32_to_limbs(e, hb);  // hashToNat: the 32-byte digest, big-endian
  } else if (fused) {
    uint32_t h[8];
    if (mlen2) sha256_msg2(h, m, mlen, in.msg + in.msg2_off[i], mlen2);
    else sha256_msg(h, m, mlen);
#pragma unroll
    for (int k = 0; k < 8; k++) e[k] = h[7 - k];
  } else {
    const uint32_t L = mlen < 32 ? mlen : 32;
#pragma unroll
    for (int k = 0; k < 8; k++) e[k] = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {  // j = byte index from the least significant end
      uint32_t v = 0;
      if ((uint32_t)j < L) v = m[L - 1 - j];
      e[j >> 2] |= v << (8 * (j & 3));
    }
  }
  uint32_t nn[8], t[8];
  load_const8(nn, C::n);
  const uint32_t bo = sub8(t, e, nn);
  if (!bo) copy8(e, t);  // e < 2^256 < 2n: one conditional subtraction
}

// HK: HK_GIVEN_OR_SHA256 (msg is the digest, or with BHF_HASH_SHA256 the
// message) or HK_SHA3_256 (msg is the message, SHA3-256 digest). DEFER: e is
// left to k_digest (w.e untouched; a rejected record's e is any scalar < n).
template <class P, class N, class C, int HK = HK_GIVEN_OR_SHA256, bool DEFER = false>
BH_HD void stage_prep(const BatchIn& in, const Work& w, uint32_t i) {
  uint8_t reason = R_OK;
  uint32_t r[8], s[8], e[8];
  uint32_t qx30[9], qy30[9];
  const uint32_t slen = in.sig_len[i];
  const uint32_t mlen = in.msg_len[i];
  const bool fused = HK == HK_SHA3_256 || (in.flags & BHF_HASH_SHA256) != 0;
  // impl.go:249-257: empty signature, then empty digest (a fused message always
  // has a 32-byte digest).
  if (slen == 0) reason = R_EMPTY_SIG;
  else if (!fused && mlen == 0) reason = R_EMPTY_DIGEST;
  DerSig ds;
  if (reason == R_OK) reason = der_parse_sig(in.sig + in.sig_off[i], slen, &ds);
  uint32_t half[8], nn[8];
  load_const8(half, C::half_n);
  load_const8(nn, C::n);
  if (reason == R_OK) {
    copy8(r, ds.r);
    copy8(s, ds.s);
    // sw/ecdsa.go:48-54 IsLowS: S <= floor(n/2)
    if (!(in.flags & BHF_NO_LOW_S) && (ds.s_big || !geq8(half, s))) reason = R_HIGH_S;
  }
  // ---- inside crypto/ecdsa.Verify (verifyNISTEC): Q first, then r, s ranges
  if (reason == R_OK && !key_import<P, C>(in.pub + (size_t)i * 64, qx30, qy30))
    reason = R_BAD_KEY;
  if (reason == R_OK && (ds.r_big || geq8(r, nn))) reason = R_R_RANGE;
  if (reason == R_OK && (ds.s_big || geq8(s, nn))) reason = R_S_RANGE;
  // ---- digest -> e (hashToNat: left-most 32 bytes, reduced mod n); DEFER:
  // k_digest computes it on the second stream (small fused batches)
  if (reason == R_OK && !DEFER) digest_e<C, HK>(in, i, e);
  uint8_t st = reason;
  if (reason == R_OK) {
    // r*R mod p and, when r + n < p, (r + n)*R mod p for the x-mod-n check
    uint32_t pmn[8], rn[8], rm[9], r2m[9];
    load_const8(pmn, C::p_minus_n);
    f_from_u256(rm, r);
    f_to_mont<P>(rm, rm);
    f_canon<P>(rm, rm);
    if (!geq8(r, pmn)) {
      st |= ST_R2OK;
      add8(rn, r, nn);
      f_from_u256(r2m, rn);
      f_to_mont<P>(r2m, r2m);
      f_canon<P>(r2m, r2m);
    } else {
      f_copy(r2m, rm);
    }
    st9(w.rm, i, w.ns, rm);
    st9(w.r2m, i, w.ns, r2m);
    to_mont<N>(s, s);
  } else {
    // keep the arithmetic of failed lanes well defined: e = r = 1, s = 1 (Mont),
    // Q = G
    for (int k = 0; k < 8; k++) { e[k] = r[k] = 0; }
    e[0] = r[0] = 1;
    load_const8(s, N::r1);
    f_const(qx30, P::gx_m);
    f_const(qy30, P::gy_m);
  }
  if (!DEFER) st8(w.e, i, w.ns, e);
  st8(w.r, i, w.ns, r);
  st8(w.sm, i, w.ns, s);
  st9(w.qx, i, w.ns, qx30);
  st9(w.qy, i, w.ns, qy30);
  w.st[i] = st;
}

// big.Int.SetBytes on a big-endian byte string of any length: value (if it
// fits 256 bits), *big if it does not, *zero if it is 0.
BH_HD void setbytes_u256(const uint8_t* b, uint32_t len, uint32_t v[8], bool* big, bool* zero) {
  uint32_t lo = 0;
  while (lo < len && b[lo] == 0) lo++;
  const uint32_t L = len - lo;
  *zero = (L == 0);
  *big = (L > 32);
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = 0;
  if (L > 32) return;
#pragma unroll
  for (int j = 0; j < 32; j++) {
    uint32_t x = 0;
    if ((uint32_t)j < L) x = b[len - 1 - j];
    v[j >> 2] |= x << (8 * (j & 3));
  }
}

// e = SignedProto.Hash() (message.go:97-138) as hashToInt: 32 bytes, then mod n,
// stored to w.e for stage_prep. One lane per record; the device runs the
// 4-lanes-per-record k_bdls_hash (verify_kernels.hip) with the same result.
template <class C>
BH_HD void stage_bdls_hash(const BdlsIn& in, const Work& w, uint32_t i) {
  uint8_t hsh[32];
  uint32_t e[8], nn[8], t[8];
  const uint8_t* q = in.xy + (size_t)i * 64;
  bdls_signed_proto_hash(hsh, in.version[i], q, q + 32, in.msg + in.msg_off[i], in.msg_len[i]);
  be32_to_limbs(e, hsh);
  load_const8(nn, C::n);
  if (!sub8(t, e, nn)) copy8(e, t);
  st8(w.e, i, w.ns, e);
}

// SignedProto.Verify (message.go:170-184): hash = SignedProto.Hash(), then Go
// crypto/ecdsa.Verify(pub{curve, X, Y}, hash, R, S) with R, S from SetBytes.
// secp256k1 takes verifyLegacy; P-256 takes verifyNISTEC. No low-S rule.
// Off-curve / out-of-range keys are rejected (BH_R_BAD_KEY) on both curves:
// for secp256k1 Go would compute on them, but consensus.go:456-466 admits only
// registered participants' keys, so such inputs never reach Verify in BDLS.
template <class P, class N, class C>
BH_HD void stage_prep(const BdlsIn& in, const Work& w, uint32_t i) {
  uint8_t reason = R_OK;
  uint32_t r[8], s[8], nn[8];
  uint32_t qx30[9], qy30[9];
  load_const8(nn, C::n);
  bool rbig, rzero, sbig, szero;
  setbytes_u256(in.r + in.r_off[i], in.r_len[i], r, &rbig, &rzero);
  setbytes_u256(in.s + in.s_off[i], in.s_len[i], s, &sbig, &szero);
  if (rzero) reason = R_R_NONPOS;       // ecdsa.Verify: r.Sign() <= 0
  else if (szero) reason = R_S_NONPOS;
  const uint8_t* q = in.xy + (size_t)i * 64;
  if (reason == R_OK && !key_import<P, C>(q, qx30, qy30)) reason = R_BAD_KEY;
  if (reason == R_OK && (rbig || geq8(r, nn))) reason = R_R_RANGE;
  if (reason == R_OK && (sbig || geq8(s, nn))) reason = R_S_RANGE;
  // e (w.e) is written by stage_bdls_hash / k_bdls_hash, possibly concurrently:
  // prep never touches it (a rejected record's e is any scalar < n)
  uint8_t st = reason;
  if (reason == R_OK) {
    uint32_t pmn[8], rn[8], rm[9], r2m[9];
    load_const8(pmn, C::p_minus_n);
    f_from_u256(rm, r);
    f_to_mont<P>(rm, rm);
    f_canon<P>(rm, rm);
    if (!geq8(r, pmn)) {
      st |= ST_R2OK;
      add8(rn, r, nn);
      f_from_u256(r2m, rn);
      f_to_mont<P>(r2m, r2m);
      f_canon<P>(r2m, r2m);
    } else {
      f_copy(r2m, rm);
    }
    st9(w.rm, i, w.ns, rm);
    st9(w.r2m, i, w.ns, r2m);
    to_mont<N>(s, s);
  } else {
    for (int k = 0; k < 8; k++) r[k] = 0;
    r[0] = 1;
    load_const8(s, N::r1);
    f_const(qx30, P::gx_m);
    f_const(qy30, P::gy_m);
  }
  st8(w.r, i, w.ns, r);
  st8(w.sm, i, w.ns, s);
  st9(w.qx, i, w.ns, qx30);
  st9(w.qy, i, w.ns, qy30);
  w.st[i] = st;
}

// ------------------------------------------------------------ batch inverse
// One lane's records (strided). Montgomery's trick: one safegcd inversion per
// lane, 3 multiplications per record. U1 = false (BDLS batches whose digests
// are still being hashed): w = s^-1 R goes to w.sm for stage_u1, u1 later.
template <class N, bool U1 = true, bool VAR = false>
BH_HD void stage_inv(const Work& w, uint32_t c, uint32_t stride, uint32_t n) {
  // lane c owns records c, c + stride, c + 2 stride, ... (< n): consecutive
  // lanes touch consecutive records, so every limb access is coalesced
  uint32_t acc[8], x[8];
  load_const8(acc, N::r1);
  uint32_t last = c;
  for (uint32_t i = c; i < n; i += stride) {
    st8(w.pre, i, w.ns, acc);  // prefix of this lane's earlier records
    ld8(x, w.sm, i, w.ns);
    mont_mul<N>(acc, acc, x);
    last = i;
  }
  if (c >= n) return;
  uint32_t inv[8];
  mont_inv_sg<N, VAR>(inv, acc);  // (prod s_i)^-1 * R
  for (uint32_t i = last;; i -= stride) {
    uint32_t pre[8], wi[8], t[8];
    ld8(pre, w.pre, i, w.ns);
    mont_mul<N>(wi, inv, pre);  // s_i^-1 * R
    ld8(x, w.sm, i, w.ns);
    mont_mul<N>(inv, inv, x);
    if constexpr (U1) {
      ld8(t, w.e, i, w.ns);
      mont_mul<N>(t, t, wi);    // u1 = e * w (plain)
      st8(w.e, i, w.ns, t);
    } else {
      st8(w.sm, i, w.ns, wi);
    }
    ld8(t, w.r, i, w.ns);
    mont_mul<N>(t, t, wi);      // u2 = r * w (plain)
    st8(w.r, i, w.ns, t);
    if (i < c + stride) break;
  }
}

// u1 = e w for the U1 = false inverse (after the digests are in w.e).
template <class N>
BH_HD void calc_u1(uint32_t u1[8], const Work& w, uint32_t i) {
  uint32_t wi[8];
  ld8(u1, w.e, i, w.ns);
  ld8(wi, w.sm, i, w.ns);
  mont_mul<N>(u1, u1, wi);
}

// ------------------------------------------------------------------ ladder
BH_HD void booth5(uint32_t in6, uint32_t* mag, bool* neg) {
  uint32_t sgn = 0u - (in6 >> 5);  // all ones if the top bit is set
  uint32_t d = (63u - in6) & sgn;
  d |= in6 & ~sgn;
  *mag = (d >> 1) + (d & 1u);
  *neg = sgn != 0;
}

// Q table: each lane owns a contiguous run of 16 entries x 28 words (27 used:
// X, Y, Z radix 2^30; padded to 112 B = 7 x 16 B) at
// ((wave * 64 + lane) * 16 + entry) * 28. A lookup is seven 16-byte loads that
// touch ~2 cache lines per lane; the earlier lane-interleaved layout touched
// one line per distinct digit per word (measured ~16x L2-miss traffic).

BH_HD uint32_t* qtab_entry(uint32_t* tab, uint32_t wave, uint32_t entry, uint32_t lane) {
  return tab + (((size_t)wave * 64 + lane) * kQTab + entry) * kQPt;
}

BH_HD void qtab_store(uint32_t* tab, uint32_t wave, uint32_t entry, uint32_t lane, const J30& P) {
  uint32_t v[28];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    v[k] = P.X[k];
    v[9 + k] = P.Y[k];
    v[18 + k] = P.Z[k];
  }
  v[27] = 0;
  W4* d = reinterpret_cast<W4*>(qtab_entry(tab, wave, entry, lane));
#pragma unroll
  for (int q = 0; q < 7; q++) d[q] = W4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}

BH_HD void qtab_load(J30& P, const uint32_t* tab, uint32_t wave, uint32_t entry, uint32_t lane) {
  const W4* s = reinterpret_cast<const W4*>(qtab_entry(const_cast<uint32_t*>(tab), wave, entry, lane));
  uint32_t v[28];
#pragma unroll
  for (int q = 0; q < 7; q++) {
    const W4 t = s[q];
    v[4 * q] = t.x;
    v[4 * q + 1] = t.y;
    v[4 * q + 2] = t.z;
    v[4 * q + 3] = t.w;
  }
#pragma unroll
  for (int k = 0; k < 9; k++) {
    P.X[k] = v[k];
    P.Y[k] = v[9 + k];
    P.Z[k] = v[18 + k];
  }
}

// One G comb-table entry t = w * kCombEntries + j: (j+1) 2^(8w) G, affine,
// canonical Montgomery radix 2^30 (out[0..8] = x, out[9..17] = y). Used by the
// init kernel (and the test-only host harness).
template <class P>
BH_HD void gtab_entry(uint32_t t, uint32_t* out) {
  const uint32_t win = t / kCombEntries, j = t % kCombEntries;
  J30 B;
  f_const(B.X, P::gx_m);
  f_const(B.Y, P::gy_m);
  f_const(B.Z, P::r1);
  for (uint32_t d = 0; d < (uint32_t)kGW * win; d++) j_dbl<P>(B, B);
  // (j+1) B by left-to-right double-and-add over the bits of j+1 (<= kCombEntries)
  const uint32_t k = j + 1;
  int top = 31;
  while (!((k >> top) & 1u)) top--;
  J30 A;
  j_copy(A, B);
  for (int b = top - 1; b >= 0; b--) {
    j_dbl<P>(A, A);
    if ((k >> b) & 1u) {
      bool same;
      J30 R;
      j_add<P>(R, A, B, &same);  // A = m B with 2 <= m < kCombEntries: never degenerate
      j_copy(A, R);
    }
  }
  uint32_t zi[9], zi2[9], x[9], y[9], z[9];
  f_reduce<P>(z, A.Z);
  f_inv<P>(zi, z);
  f_sqr<P>(zi2, zi);
  f_mul<P>(x, A.X, zi2);
  f_mul<P>(zi2, zi2, zi);
  f_mul<P>(y, A.Y, zi2);
  f_reduce<P>(x, x);
  f_reduce<P>(y, y);
  for (int q = 0; q < 9; q++) {
    out[q] = x[q];
    out[9 + q] = y[q];
  }
}

// v >>= B (288-bit, compile-time B < 288)
template <int B>
BH_HD void shr_const(uint32_t v[9]) {
  constexpr int ws = B / 32, bs = B % 32;
#pragma unroll
  for (int q = 0; q < 9; q++) {
    const uint32_t lo = (q + ws < 9) ? v[q + ws] : 0u;
    const uint32_t hi = (q + ws + 1 < 9) ? v[q + ws + 1] : 0u;
    if constexpr (bs != 0) v[q] = (lo >> bs) | (hi << (32 - bs));
    else v[q] = lo;
  }
}

struct GOff {
  uint32_t v[9];
};
constexpr GOff make_goff() {
  GOff o{};
  for (int w = 0; w < kCombWindows; w++) {
    const int b = w * kGW + kGW - 1;
    o.v[b / 32] |= 1u << (b % 32);
  }
  return o;
}
constexpr GOff kGOff = make_goff();

// v (288-bit) = k + M for the G comb's signed-digit recoding (see kGW)
BH_HD void recode_goff(uint32_t v[9], const uint32_t k[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    c += (uint64_t)k[q] + kGOff.v[q];
    v[q] = (uint32_t)c;
    c >>= 32;
  }
  v[8] = (uint32_t)c + kGOff.v[8];
}

// ---- shared tail: u1 G by the fixed-base comb, then A + B and the x check
// u1 G: kGW-bit signed windows over the affine table (kCombWindows mixed
// adds). The common step is one in-place mixed addition; a zero digit (odd
// 2^-kGW per window), B still at infinity, and the degenerate additions of
// crafted scalars take a side branch that the lanes skip together.
// Software-pipelined (BH_GCOMB_PREFETCH, default 1): window win + 1's entry is
// loaded before window win's addition, so its L2 / MALL latency (the 5.9 MB
// table does not fit one XCD's 4 MB L2) runs under a mixed addition instead
// of stalling the wave -- there is no doubling here to hide it behind, unlike
// the key comb's Horner step.
#ifndef BH_GCOMB_PREFETCH
#define BH_GCOMB_PREFETCH 1
#endif
// the digit of the window v now starts at (v shifted past it) and its entry
BH_HD void g_window(uint32_t v[9], int win, const uint32_t* gtab, uint32_t tx[9], uint32_t ty[9],
                    uint32_t& mag, bool& neg) {
  const int d = (int)(v[0] & (2u * kCombEntries - 1u)) - kCombEntries;
  shr_const<kGW>(v);
  mag = (uint32_t)(d < 0 ? -d : d);
  neg = d < 0;
  const uint32_t* te = gtab + ((size_t)win * kCombEntries + (mag ? mag - 1 : 0)) * kGEntry;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    tx[k] = te[k];
    ty[k] = te[9 + k];
  }
}

// One window of g_comb: B += T (T = the signed entry, mag 0: B unchanged).
template <class P>
BH_HD void g_step(J30& B, bool& b_inf, const uint32_t tx[9], const uint32_t ty[9], uint32_t mag,
                  const uint32_t one[9]) {
  if (mag == 0u || b_inf) {  // zero digit: B unchanged; B at infinity: B = T
    if (mag != 0u) {
      f_copy(B.X, tx);
      f_copy(B.Y, ty);
      f_copy(B.Z, one);
      b_inf = false;
    }
  } else {
    bool same;
    if (j_madd<P>(B, B, tx, ty, &same)) {  // rare: x(B) == x(T)
      if (same) {
        J30 Tj;
        f_copy(Tj.X, tx);
        f_copy(Tj.Y, ty);
        f_copy(Tj.Z, one);
        j_dbl<P>(B, Tj);
      } else {
        b_inf = true;
      }
    }
  }
}

template <class P>
BH_HD void g_comb(J30& B, bool& b_inf, const uint32_t* gtab, const uint32_t u1[8]) {
  uint32_t one[9];
  f_const(one, P::r1);
  b_inf = true;
  f_copy(B.X, one);
  f_copy(B.Y, one);
  f_copy(B.Z, one);
  uint32_t v[9];
  recode_goff(v, u1);
  uint32_t tx[9], ty[9], mag;
  bool neg;
  if (BH_GCOMB_PREFETCH) g_window(v, 0, gtab, tx, ty, mag, neg);
#pragma unroll 1
  for (int win = 0; win < kCombWindows; win++) {
    if (BH_GCOMB_PREFETCH) {
      // next window's entry (past the last window: a valid entry, unused)
      uint32_t nx[9], ny[9], nmag;
      bool nneg;
      const int nw = win + 1 < kCombWindows ? win + 1 : win;
      g_window(v, nw, gtab, nx, ny, nmag, nneg);
      if (neg) f_neg<P, 64>(ty, ty);
      g_step<P>(B, b_inf, tx, ty, mag, one);
      f_copy(tx, nx);
      f_copy(ty, ny);
      mag = nmag;
      neg = nneg;
    } else {
      g_window(v, win, gtab, tx, ty, mag, neg);
      if (neg) f_neg<P, 64>(ty, ty);
      g_step<P>(B, b_inf, tx, ty, mag, one);
    }
  }
}

// Pt = A + B (explicit doubling / infinity), then x(Pt) mod n == r  <=>
// X == r Z^2  or  (r + n < p and) X == (r + n) Z^2.
template <class P>
BH_HD bool finish_check(const Work& w, uint32_t i, const J30& A, bool a_inf, const J30& B,
                        bool b_inf) {
  J30 Pt;
  bool p_inf;
  if (b_inf) {
    j_copy(Pt, A);
    p_inf = a_inf;
  } else if (a_inf) {
    j_copy(Pt, B);
    p_inf = false;
  } else {
    bool same;
    const bool deg = j_add<P>(Pt, A, B, &same);
    p_inf = false;
    if (deg) {
      if (same) j_dbl<P>(Pt, A);
      else p_inf = true;
    }
  }
  uint32_t z2[9], t[9], x[9], rm[9];
  f_sqr<P>(z2, Pt.Z);                  // [b2]
  const bool z_zero = f_is_zero2<P>(z2);
  f_reduce<P>(x, Pt.X);                // canonical X
  ld9(rm, w.rm, i, w.ns);
  f_mul<P>(t, rm, z2);
  f_canon<P>(t, t);
  bool ok = f_eq(t, x);
  if (w.st[i] & ST_R2OK) {
    ld9(rm, w.r2m, i, w.ns);
    f_mul<P>(t, rm, z2);
    f_canon<P>(t, t);
    ok = ok || f_eq(t, x);
  }
  return ok && !p_inf && !z_zero;
}

// Variable-base path: Q multiples 1..16 in the lane's scratch slab (slot =
// (wave, lane)), Booth w=5 windows over u2, most significant first.
template <class P>
BH_HD void q_ladder(J30& A, bool& a_inf, const Work& w, uint32_t i, uint32_t wave,
                    uint32_t lane) {
  uint32_t u2[8], qx[9], qy[9], one[9];
  ld8(u2, w.r, i, w.ns);
  ld9(qx, w.qx, i, w.ns);
  ld9(qy, w.qy, i, w.ns);
  f_const(one, P::r1);
  J30 T;
  f_copy(T.X, qx);
  f_copy(T.Y, qy);
  f_copy(T.Z, one);
  qtab_store(w.qtab, wave, 0, lane, T);
  j_dbl<P>(T, T);
  qtab_store(w.qtab, wave, 1, lane, T);
  for (uint32_t k = 2; k < kQTab; k++) {
    bool same;
    j_madd<P>(T, T, qx, qy, &same);  // (k+1) Q = k Q + Q, never degenerate for 2 <= k < 16
    qtab_store(w.qtab, wave, k, lane, T);
  }
  // K = u2 << 28 (288 bits): window i's 6 Booth bits sit at the top after 51-i shifts
  uint32_t K[9];
  K[0] = u2[0] << 28;
#pragma unroll
  for (int k = 1; k < 8; k++) K[k] = (u2[k] << 28) | (u2[k - 1] >> 4);
  K[8] = u2[7] >> 4;
  {
    uint32_t mag;
    bool neg;
    booth5(K[8] >> 26, &mag, &neg);
#pragma unroll
    for (int k = 8; k > 0; k--) K[k] = (K[k] << 5) | (K[k - 1] >> 27);
    K[0] <<= 5;
    qtab_load(A, w.qtab, wave, mag ? mag - 1 : 0, lane);
    if (neg) f_neg<P, 64>(A.Y, A.Y);
    a_inf = (mag == 0);
  }
  for (int win = 50; win >= 0; win--) {
    uint32_t mag;
    bool neg;
    booth5(K[8] >> 26, &mag, &neg);
#pragma unroll
    for (int k = 8; k > 0; k--) K[k] = (K[k] << 5) | (K[k - 1] >> 27);
    K[0] <<= 5;
    J30 T2;
    qtab_load(T2, w.qtab, wave, mag ? mag - 1 : 0, lane);  // issued before the doublings
    for (int d = 0; d < 5; d++) j_dbl<P>(A, A);
    if (neg) f_neg<P, 64>(T2.Y, T2.Y);
    J30 R;
    bool same;
    const bool deg = j_add<P>(R, A, T2, &same);
    const bool take = mag != 0;
    const bool use_t = take && a_inf;
    const bool use_r = take && !a_inf && !deg;
    const bool rare = take && !a_inf && deg;
    j_sel(A, use_r, R, A);
    j_sel(A, use_t, T2, A);
    if (rare) {  // A == +-T: only reachable at the last window for crafted u2
      if (same) j_dbl<P>(A, T2);
      else a_inf = true;
    }
    if (use_t) a_inf = false;
  }
}

// ---- secp256k1: GLV endomorphism (the split btcec uses to halve the
// doublings, vendor/github.com/BDLS-bft/bdls/crypto/btcec/btcec.go:765-865
// splitK). phi(x, y) = (beta x, y) = lambda (x, y); u2 = k1 + k2 lambda (mod n)
// with |k1|, |k2| < 2^128, so u2 Q = k1 Q + k2 phi(Q): 125 doublings instead
// of 255. The split is libsecp256k1's secp256k1_scalar_split_lambda (c_i =
// round(u2 g_i / 2^384), k2 = c1 (-b1) + c2 (-b2), k1 = u2 - k2 lambda); any
// valid split gives the same point, hence the same verdict, as btcec's.
struct GlvK1 {
  static constexpr uint32_t g1[8] = {0x45dbb031u, 0xe893209au, 0x71e8ca7fu, 0x3daa8a14u,
                                     0x9284eb15u, 0xe86c90e4u, 0xa7d46bcdu, 0x3086d221u};
  static constexpr uint32_t g2[8] = {0x8ac47f71u, 0x1571b4aeu, 0x9df506c6u, 0x221208acu,
                                     0x0abfe4c4u, 0x6f547fa9u, 0x010e8828u, 0xe4437ed6u};
  // -b1, -b2, -lambda times 2^256 mod n (a Montgomery product with them is a
  // plain product mod n)
  static constexpr uint32_t mb1R[8] = {0x0ad9263cu, 0xc50468d0u, 0xfaa6ed42u, 0x1b1c8205u,
                                       0x8ac47f71u, 0x1571b4aeu, 0x9df506c6u, 0x221208acu};
  static constexpr uint32_t mb2R[8] = {0x6a144696u, 0x0cac5e50u, 0xf3ba5939u, 0x1e8a8dc5u,
                                       0xba244fceu, 0x176cdf65u, 0x8e173580u, 0xc25575ebu};
  static constexpr uint32_t mlamR[8] = {0x06a3d4a3u, 0xcf54734fu, 0x2b820beeu, 0x8e1af539u,
                                        0xad96826du, 0x8c5699f9u, 0x7aa729c6u, 0xacd7bfe8u};
  // beta 2^270 mod p, radix 2^30 (canonical)
  static constexpr uint32_t beta_m[9] = {0x22c82b32u, 0x361d08c9u, 0x02bd6290u,
                                         0x1631c4b8u, 0x0140ff78u, 0x38d02e39u,
                                         0x0fe3a625u, 0x2bcbb3d5u, 0x00008dabu};
};

// (k g) >> 384 rounded to nearest (bit 383 added); k, g < 2^256, result < 2^129
BH_HD void mul_shift384(uint32_t out[8], const uint32_t k[8], const uint32_t g[8]) {
  uint32_t t[16];
#pragma unroll
  for (int q = 0; q < 16; q++) t[q] = 0;
#pragma unroll
  for (int a = 0; a < 8; a++) {
    uint64_t c = 0;
#pragma unroll
    for (int b = 0; b < 8; b++) {
      c += (uint64_t)k[a] * g[b] + t[a + b];
      t[a + b] = (uint32_t)c;
      c >>= 32;
    }
    t[a + 8] = (uint32_t)c;
  }
  uint64_t c = t[11] >> 31;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    c += t[12 + q];
    out[q] = (uint32_t)c;
    c >>= 32;
  }
  out[4] = (uint32_t)c;
  out[5] = out[6] = out[7] = 0;
}

// bits [b, b + 6) of a 160-bit value (5 limbs); b compile-time after unrolling
BH_HD uint32_t bits6(const uint32_t v[5], uint32_t b) {
  const uint32_t q = b >> 5, sh = b & 31u;
  uint32_t x = v[q] >> sh;
  if (sh > 26 && q + 1 < 5) x |= v[q + 1] << (32 - sh);
  return x & 63u;
}

template <class P>
BH_HD void j_acc(J30& A, bool& a_inf, const J30& T, bool t_inf);  // below
template <class P>
BH_HD void j_acc_aff(J30& A, bool& a_inf, const uint32_t tx[9], const uint32_t ty[9],
                     const uint32_t one[9], bool t_inf);  // below

// parts: bit 0 = the k1 Q half, bit 1 = the k2 phi(Q) half (3 = all of u2 Q;
// the 2-lane ladder runs one half per lane and adds the two results).
template <class P>
BH_HD void q_ladder_glv(J30& A, bool& a_inf, const Work& w, uint32_t i, uint32_t wave,
                        uint32_t lane, uint32_t parts = 3) {
  uint32_t u2[8], qx[9], qy[9], one[9];
  ld8(u2, w.r, i, w.ns);
  ld9(qx, w.qx, i, w.ns);
  ld9(qy, w.qy, i, w.ns);
  f_const(one, P::r1);
  J30 T;
  f_copy(T.X, qx);
  f_copy(T.Y, qy);
  f_copy(T.Z, one);
  qtab_store(w.qtab, wave, 0, lane, T);
  j_dbl<P>(T, T);
  qtab_store(w.qtab, wave, 1, lane, T);
  for (uint32_t k = 2; k < kQTab; k++) {
    bool same;
    j_madd<P>(T, T, qx, qy, &same);  // (k+1) Q = k Q + Q, never degenerate for 2 <= k < 16
    qtab_store(w.qtab, wave, k, lane, T);
  }
  // u2 = k1 + k2 lambda (mod n), then |k1|, |k2| with their signs
  uint32_t c1[8], c2[8], k1[8], k2[8], t[8], cst[8];
  mul_shift384(c1, u2, GlvK1::g1);
  mul_shift384(c2, u2, GlvK1::g2);
  load_const8(cst, GlvK1::mb1R);
  mont_mul<Fn_k1>(k2, c1, cst);
  load_const8(cst, GlvK1::mb2R);
  mont_mul<Fn_k1>(t, c2, cst);
  mod_add<Fn_k1>(k2, k2, t);
  load_const8(cst, GlvK1::mlamR);
  mont_mul<Fn_k1>(k1, k2, cst);
  mod_add<Fn_k1>(k1, k1, u2);
  load_const8(cst, Cv_k1::half_n);
  const bool s1 = !geq8(cst, k1), s2 = !geq8(cst, k2);  // "negative": > n/2
  if (s1) mod_neg<Fn_k1>(k1, k1);
  if (s2) mod_neg<Fn_k1>(k2, k2);
  // Booth windows read bits [5 win - 1, 5 win + 4]: K = k << 1 (k < 2^128,
  // so windows 0..25 suffice and the top digit is non-negative)
  uint32_t K1[5], K2[5];
  K1[0] = k1[0] << 1;
  K2[0] = k2[0] << 1;
#pragma unroll
  for (int q = 1; q < 5; q++) {
    K1[q] = (k1[q] << 1) | (k1[q - 1] >> 31);
    K2[q] = (k2[q] << 1) | (k2[q - 1] >> 31);
  }
  uint32_t beta[9];
  f_const(beta, GlvK1::beta_m);
  f_copy(A.X, one);
  f_copy(A.Y, one);
  f_copy(A.Z, one);
  a_inf = true;
  for (int win = 25; win >= 0; win--) {
    if (win != 25)
      for (int d = 0; d < 5; d++) j_dbl<P>(A, A);
    uint32_t mag;
    bool neg;
    if (parts & 1u) {
      booth5(bits6(K1, 5u * (uint32_t)win), &mag, &neg);
      J30 T1;
      qtab_load(T1, w.qtab, wave, mag ? mag - 1 : 0, lane);
      if (neg != s1) f_neg<P, 64>(T1.Y, T1.Y);
      j_acc<P>(A, a_inf, T1, mag == 0);
    }
    if (parts & 2u) {
      booth5(bits6(K2, 5u * (uint32_t)win), &mag, &neg);
      J30 T2;
      qtab_load(T2, w.qtab, wave, mag ? mag - 1 : 0, lane);
      f_mul<P>(T2.X, T2.X, beta);  // phi: (beta X, Y, Z)
      if (neg != s2) f_neg<P, 64>(T2.Y, T2.Y);
      j_acc<P>(A, a_inf, T2, mag == 0);
    }
  }
}

// Returns true iff the signature equation holds (valid). Lanes whose prep
// failed run on placeholder inputs (Q = G, u1 = u2 = 1) and are masked by the
// caller.
template <class P>
BH_HD bool stage_ladder(const Work& w, const uint32_t* gtab, uint32_t i, uint32_t wave,
                        uint32_t lane) {
  J30 A, B;
  bool a_inf, b_inf;
  if constexpr (P::a_is_minus3) q_ladder<P>(A, a_inf, w, i, wave, lane);
  else q_ladder_glv<P>(A, a_inf, w, i, wave, lane);
  uint32_t u1[8];
  ld8(u1, w.e, i, w.ns);
  g_comb<P>(B, b_inf, gtab, u1);
  return finish_check<P>(w, i, A, a_inf, B, b_inf);
}

// ---------------------------------------------------------------- per-key comb
// Records whose public key occurs >= kMinUses times in the batch share one
// fixed-base table for their key, built inside the same step:
//   entry (win, j) = (j+1) 2^(4 win) Q,  win in [0, 65), j in [0, 8)
// (Jacobian, 28 words). u2 Q is then 65 table additions with 4-bit signed
// digits in [-7, 8] and no doublings.
constexpr int kKW = 4;                           // signed-window width (bits)
constexpr int kKWin = (257 + kKW - 1) / kKW;     // 65 windows at 4 bits
constexpr int kKEnt = 1 << (kKW - 1);            // 8 entries per window at 4 bits
constexpr uint32_t kKTabWords = (uint32_t)kKWin * kKEnt * kQPt;
constexpr uint32_t kMinUses = 4;
// Below this batch size the step is latency-bound (one table build is a
// serial 1.07M-instruction lane, more than one ladder), so key tables are off.
constexpr uint32_t kKeyTableMinBatch = 8192;

// Signed kKW-bit digits of a scalar by one addition: with M = sum over the
// windows of 2^(kKW w + kKW - 1), window w of k + M minus kKEnt is digit w of
// k in [-kKEnt, kKEnt - 1] (the G comb's recode_goff for the key tables).
struct KOff {
  uint32_t v[9];
};
constexpr KOff make_koff() {
  KOff o{};
  for (int w = 0; w < kKWin; w++) {
    const int b = w * kKW + kKW - 1;
    o.v[b / 32] |= 1u << (b % 32);
  }
  return o;
}
constexpr KOff kKOff = make_koff();

BH_HD void recode_koff(uint32_t v[9], const uint32_t k[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    c += (uint64_t)k[q] + kKOff.v[q];
    v[q] = (uint32_t)c;
    c >>= 32;
  }
  v[8] = (uint32_t)c + kKOff.v[8];
}

BH_HD void ktab_store(uint32_t* tab, uint32_t win, uint32_t j, const J30& P) {
  uint32_t v[28];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    v[k] = P.X[k];
    v[9 + k] = P.Y[k];
    v[18 + k] = P.Z[k];
  }
  v[27] = 0;
  W4* d = reinterpret_cast<W4*>(tab + ((size_t)win * kKEnt + j) * kQPt);
#pragma unroll
  for (int q = 0; q < 7; q++) d[q] = W4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}

BH_HD void ktab_load(J30& P, const uint32_t* tab, uint32_t win, uint32_t j) {
  const W4* s = reinterpret_cast<const W4*>(tab + ((size_t)win * kKEnt + j) * kQPt);
  uint32_t v[28];
#pragma unroll
  for (int q = 0; q < 7; q++) {
    const W4 t = s[q];
    v[4 * q] = t.x;
    v[4 * q + 1] = t.y;
    v[4 * q + 2] = t.z;
    v[4 * q + 3] = t.w;
  }
#pragma unroll
  for (int k = 0; k < 9; k++) {
    P.X[k] = v[k];
    P.Y[k] = v[9 + k];
    P.Z[k] = v[18 + k];
  }
}

// One lane per table: entry j of window w = (j+1) 16^w Q. Per window a co-Z
// chain (ec30.h j_dblu / j_zaddu): DBLU gives 2B and B on 2B's Z, then six
// ZADDUs give 3B..8B, each re-basing B onto the new sum's Z, and one doubling
// of 8B gives the next window's base 16B:
//   8 + 6 x 7 + 8 = 58 F_p mul/sqr per window (the plain Jacobian sequence,
//   5 doublings + 3 full additions, is 88).
// The entries are ordinary Jacobian points (each with its own Z), so the key
// comb is unchanged. ZADDU cannot degenerate here: k B = +-B would need n to
// divide (k -+ 1) 16^w with k - 1 <= 7, and n is a prime of 256 bits.
template <class P>
BH_HD void ktab_build(uint32_t* tab, const Work& w, uint32_t rec) {
  J30 B, Bz, S;
  ld9(B.X, w.qx, rec, w.ns);
  ld9(B.Y, w.qy, rec, w.ns);
  f_const(B.Z, P::r1);
  for (uint32_t win = 0; win < (uint32_t)kKWin; win++) {
    ktab_store(tab, win, 0, B);               // 1 B
    j_dblu<P>(S, Bz, B);                      // S = 2B, Bz = B on S's Z
    ktab_store(tab, win, 1, S);               // 2 B
#pragma unroll 1  // one ZADDU body (~10 KB of code; unrolled: same speed, 5x the code)
    for (uint32_t j = 2; j < (uint32_t)kKEnt; j++) {
      J30 T;
      j_zaddu<P>(T, Bz, S);                   // T = (j+1) B; Bz onto T's Z
      ktab_store(tab, win, j, T);
      j_copy(S, T);
    }
    j_dbl<P>(B, S);                           // 16 B: the next window's base
  }
}

// Registry slots (round 5) also hold the 4-bit windows AFFINE at kRegWin
// (built below, after the comb layout); aff selects that form.
BH_HD uint32_t reg_win_offset();
BH_HD void llaff_load(uint32_t x[9], uint32_t y[9], const uint32_t* tab, uint32_t b);
template <class P>
BH_HD void win_entry(J30& T, const uint32_t* tab, uint32_t win, uint32_t j, bool aff,
                     const uint32_t one[9]) {
  if (aff) {
    llaff_load(T.X, T.Y, tab + reg_win_offset(), win * (uint32_t)kKEnt + j);
    f_copy(T.Z, one);
  } else {
    ktab_load(T, tab, win, j);
  }
}

// u2 Q from a key table: kKW-bit signed windows (least significant first).
template <class P>
BH_HD void q_keycomb(J30& A, bool& a_inf, const Work& w, uint32_t i, const uint32_t* tab,
                     bool aff = false) {
  uint32_t one[9];
  f_const(one, P::r1);
  uint32_t k2[8];
  ld8(k2, w.r, i, w.ns);
  a_inf = true;
  f_const(A.X, P::r1);
  f_const(A.Y, P::r1);
  f_const(A.Z, P::r1);
  uint32_t carry = 0;
  for (int win = 0; win < kKWin; win++) {
    // carry-scan digits in [-7, 8] (the wide path's recode_koff gives offset
    // digits in [-8, 7]: the same scalar, another digit string)
    const uint32_t t = (k2[0] & 0xfu) + carry;
#pragma unroll
    for (int k = 0; k < 7; k++) k2[k] = (k2[k] >> 4) | (k2[k + 1] << 28);
    k2[7] >>= 4;
    const bool neg = t > 8u;
    const uint32_t mag = neg ? 16u - t : t;
    carry = neg ? 1u : 0u;
    J30 T;
    win_entry<P>(T, tab, win, mag ? mag - 1 : 0, aff, one);
    if (neg) f_neg<P, 64>(T.Y, T.Y);
    J30 R;
    bool same;
    // (affine entries: a mixed addition, 11 F_p ops instead of 16)
    const bool deg = aff ? j_madd<P>(R, A, T.X, T.Y, &same) : j_add<P>(R, A, T, &same);
    const bool take = mag != 0;
    const bool use_t = take && a_inf;
    const bool use_r = take && !a_inf && !deg;
    const bool rare = take && !a_inf && deg;  // only via the mod-n wrap of the top window
    j_sel(A, use_r, R, A);
    j_sel(A, use_t, T, A);
    if (rare) {
      if (same) j_dbl<P>(A, T);
      else a_inf = true;
    }
    if (use_t) a_inf = false;
  }
}

// ---------------------------------------------------------------- per-key signed Lim-Lee comb
// Per-batch key tables of LARGE batches (one lane per record, o.wide == 1).
// A SIGNED Lim-Lee comb (round 4; round 3 had the unsigned 6 x 43 comb): t =
// BH_LL_T teeth spaced s = ceil(257 / t) bits. For odd k < 2^257 put
//   c = (k >> 1) | 2^(t s - 1),   d_(i,j) = 2 c_(s i + j) - 1 in {-1, +1};
// then k = sum_(j < s) 2^j V_j with V_j = sum_(i < t) d_(i,j) 2^(s i): every
// column is a nonzero signed sum (sum 2^(s i + j) (2 c - 1) = 2 c - 2^(t s) + 1
// = k). With B_i = 2^(s i) Q the table holds the 2^(t-1) points
//   E[m] = B_(t-1) + sum_(i < t-1) (2 m_i - 1) B_i,
// and V_j Q = +E[m_j] when column j's top tooth is set, else -E[~m_j] (m_j =
// the column's lower t - 1 bits). u2 Q = k Q with k = u2 (u2 odd) or u2 + n
// (u2 even; n Q = 0), by Horner from the top column, whose top bit is the set
// bit t s - 1 (so it is +E): s - 1 doublings + s - 1 mixed additions per record
// and no empty columns -- at t = 7 (s = 37) 36 + 36 instead of the unsigned
// 6 x 43 comb's 42 + 43 with a zero-column select, for a table of the same 64
// entries.
// Build, one lane per table (round 5): (t - 1) s doublings give D_i = 2 B_i and
// B_(i+1) = 2^(s-1) D_i; those 2 (t - 1) chain points are made affine with one
// inversion (Montgomery's trick). The 2^(t-1) entries are then SUMS of two
// small affine tables over a split of the lower t - 1 digits into a low group
// (a digits) and a high group (the other t - 1 - a, plus the top tooth):
//   E[m] = H[m >> a] + L[m & (2^a - 1)],
//   L[x] = sum_(i < a) (2 x_i - 1) B_i,
//   H[y] = B_(t-1) + sum_(a <= i < t-1) (2 y_(i-a) - 1) B_i.
// L and H (2^a + 2^(t-1-a) points) come from two Gray-code walks of mixed
// additions of +-D_i (flipping digit i from -1 to +1 adds 2 B_i), made affine
// with a second inversion; each entry is one affine addition H + L whose
// denominators x_H - x_L are inverted together (a third inversion): 6 F_p ops
// per entry instead of the full Gray walk over all entries (11 + 1) and its
// backward affine pass (6), and no raw Jacobian entry written and read back.
// No build step can degenerate: every scalar involved lies in (0, n / 2), the
// walks' partial sums exceed every d_i they add with e + d < n, and H's scalar
// (~2^(s (t-1))) never equals +-L's (< 2^(s a + 1)). The Horner additions keep
// explicit degenerate handling (A = +-V_j only for crafted scalars), as a
// branch the lanes skip together.
#ifndef BH_LL_T
#define BH_LL_T 7  // teeth: 7 x 37 bits, 64 entries (signed)
#endif
constexpr int kLLTeeth = BH_LL_T, kLLSpace = (257 + kLLTeeth - 1) / kLLTeeth;
constexpr int kLLTS = kLLTeeth * kLLSpace;        // >= 257: c < 2^(t s)
constexpr uint32_t kLLEnt = 1u << (kLLTeeth - 1);  // entries E[0 .. 2^(t-1))
constexpr uint32_t kLLAff = 20;                    // words per affine point
// the build's split: L over the a low digits, H over the others + the top tooth
constexpr int kLLA = (kLLTeeth - 1) / 2;
constexpr uint32_t kLLNL = 1u << kLLA, kLLNH = 1u << (kLLTeeth - 1 - kLLA);
constexpr uint32_t kLLWalk = kLLNL + kLLNH;         // L and H points (two walks)
constexpr uint32_t kLLChain = 2u * (kLLTeeth - 1);  // Jacobian D_i / B_(i+1) of the chain
// Table region (words): entries [0, kLLEnt) x kLLAff (all the comb reads), then
// build scratch: affine B_0..B_(t-1), D_0..D_(t-2) (aux), affine L and H, raw
// Jacobian points (the chain's, then the walks'), running Z / denominator
// products (12 words each).
constexpr uint32_t kLLAux = kLLEnt;
constexpr uint32_t kLLLH = kLLAux + 2u * kLLTeeth - 1u;
constexpr uint32_t kLLRaw = ((kLLLH + kLLWalk) * kLLAff + 3u) & ~3u;
constexpr uint32_t kLLRawN = kLLChain > kLLWalk ? kLLChain : kLLWalk;
constexpr uint32_t kLLPre = kLLRaw + 28u * kLLRawN;
static_assert(kLLTS >= 257 && kLLTS <= 288 && kLLSpace < 64 && kLLTeeth >= 3 &&
                  kLLPre + 12u * kLLEnt <= kKTabWords && kLLChain <= kLLEnt &&
                  kLLWalk <= kLLEnt,
              "comb table layout");

BH_HD void llraw_store(uint32_t* tab, uint32_t b, const J30& P) { ktab_store(tab + kLLRaw, 0, b, P); }
BH_HD void llraw_load(J30& P, const uint32_t* tab, uint32_t b) { ktab_load(P, tab + kLLRaw, 0, b); }

BH_HD void llpre_store(uint32_t* tab, uint32_t m, const uint32_t z[9]) {
  W4* d = reinterpret_cast<W4*>(tab + kLLPre + 12u * m);
  d[0] = W4{z[0], z[1], z[2], z[3]};
  d[1] = W4{z[4], z[5], z[6], z[7]};
  d[2] = W4{z[8], 0u, 0u, 0u};
}

BH_HD void llpre_load(uint32_t z[9], const uint32_t* tab, uint32_t m) {
  const W4* s = reinterpret_cast<const W4*>(tab + kLLPre + 12u * m);
  const W4 a = s[0], b = s[1], c = s[2];
  z[0] = a.x; z[1] = a.y; z[2] = a.z; z[3] = a.w;
  z[4] = b.x; z[5] = b.y; z[6] = b.z; z[7] = b.w;
  z[8] = c.x;
}

// affine point slot b (entries E[b], b < kLLEnt; then the aux points)
BH_HD void llaff_store(uint32_t* tab, uint32_t b, const uint32_t x[9], const uint32_t y[9]) {
  W4* d = reinterpret_cast<W4*>(tab + (size_t)b * kLLAff);
  d[0] = W4{x[0], x[1], x[2], x[3]};
  d[1] = W4{x[4], x[5], x[6], x[7]};
  d[2] = W4{x[8], y[0], y[1], y[2]};
  d[3] = W4{y[3], y[4], y[5], y[6]};
  d[4] = W4{y[7], y[8], 0u, 0u};
}

BH_HD void llaff_load(uint32_t x[9], uint32_t y[9], const uint32_t* tab, uint32_t b) {
  const W4* s = reinterpret_cast<const W4*>(tab + (size_t)b * kLLAff);
  const W4 a = s[0], c = s[1], d = s[2], e = s[3], f = s[4];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = c.x; x[5] = c.y; x[6] = c.z; x[7] = c.w;
  x[8] = d.x; y[0] = d.y; y[1] = d.z; y[2] = d.w;
  y[3] = e.x; y[4] = e.y; y[5] = e.z; y[6] = e.w;
  y[7] = f.x; y[8] = f.y;
}

// The same 18 words (x then y) through 8-byte loads at any 8-byte-aligned
// slot: k_keycomb's LDS copies of a workgroup's tables pack entries at 72
// bytes (kLLLds words), the per-batch tables at 80 (kLLAff); the pointer may
// be either (a flat load).
constexpr uint32_t kLLLds = 18;
struct alignas(8) W2 {
  uint32_t x, y;
};
BH_HD void llent_load(uint32_t x[9], uint32_t y[9], const uint32_t* p) {
  const W2* s = reinterpret_cast<const W2*>(p);
  W2 v[9];
#pragma unroll
  for (int k = 0; k < 9; k++) v[k] = s[k];
  x[0] = v[0].x; x[1] = v[0].y; x[2] = v[1].x; x[3] = v[1].y;
  x[4] = v[2].x; x[5] = v[2].y; x[6] = v[3].x; x[7] = v[3].y;
  x[8] = v[4].x; y[0] = v[4].y; y[1] = v[5].x; y[2] = v[5].y;
  y[3] = v[6].x; y[4] = v[6].y; y[5] = v[7].x; y[6] = v[7].y;
  y[7] = v[8].x; y[8] = v[8].y;
}

// Field inverse by safegcd (fe.h mod_inv_sg, constant iteration so the lanes
// of a wave stay together): a R -> a^-1 R for the radix-2^30 field (any beta
// f_reduce accepts, a != 0 mod p). The divsteps run on the canonical value
// (a R)^-1, and one product with R^3 returns to the Montgomery domain. About a
// third of the Fermat chain's instructions (255 squarings + 12 products).
template <class P>
BH_HD void f_inv_sg(uint32_t r[9], const uint32_t a[9]) {
  uint32_t c[9], c8[8], i8[8], r3[9];
  f_reduce<P>(c, a);
  f_to_u256(c8, c);
  mod_inv_sg<typename P::M32>(i8, c8);
  f_from_u256(c, i8);
  f_const(r3, P::r3);
  f_mul<P>(r, c, r3);
}

// (X, Y, Z) -> affine (X / Z^2, Y / Z^3) given zi = Z^-1
template <class P>
BH_HD void ll_to_affine(uint32_t x[9], uint32_t y[9], const J30& E, const uint32_t zi[9]) {
  uint32_t z2[9], z3[9];
  f_sqr<P>(z2, zi);
  f_mul<P>(z3, z2, zi);
  f_mul<P>(x, E.X, z2);
  f_mul<P>(y, E.Y, z3);
}

// Walk position m (0..2^(t-1) - 1) -> entry gray(m); step m flips digit ctz(m).
BH_HD uint32_t ll_gray(uint32_t m) { return m ^ (m >> 1); }

// One Gray-code walk of the build (L or H): the 2^nd points
//   P[g] = top + sum_(k < nd) (2 g_k - 1) B_(i0 + k)   (top = B_(t-1) for H, none for L),
// as raw Jacobian points at raw slots [r0, r0 + 2^nd) in walk order with the
// running product z of their Z (the whole build's walks share one product
// chain: pre slot r0 + m holds z after point m). Start: top - sum B_(i0 + k)
// (mixed additions of -B, never degenerate); step m flips digit ctz(m) of
// gray(m), adding +-D_(i0 + ctz(m)).
template <class P>
BH_HD void ll_walk(uint32_t* tab, uint32_t i0, int nd, bool top, uint32_t r0, uint32_t z[9],
                   const uint32_t one[9]) {
  J30 A;
  bool same;
  int k = nd - 1;
  if (top) {
    llaff_load(A.X, A.Y, tab, kLLAux + kLLTeeth - 1u);  // B_(t-1)
  } else {  // -B_(i0 + nd - 1)
    llaff_load(A.X, A.Y, tab, kLLAux + i0 + (uint32_t)k);
    f_neg<P, 64>(A.Y, A.Y);
    k--;
  }
  f_copy(A.Z, one);
#pragma unroll 1
  for (; k >= 0; k--) {
    uint32_t bx[9], by[9];
    llaff_load(bx, by, tab, kLLAux + i0 + (uint32_t)k);
    f_neg<P, 64>(by, by);
    (void)j_madd<P>(A, A, bx, by, &same);  // never degenerate (see above)
  }
  llraw_store(tab, r0, A);
  if (r0 == 0) f_copy(z, A.Z);
  else f_mul<P>(z, z, A.Z);
  llpre_store(tab, r0, z);
  const uint32_t npts = 1u << nd;
  uint32_t nx[9], ny[9];
  llaff_load(nx, ny, tab, kLLAux + kLLTeeth + i0);  // D_i0 for m = 1
#pragma unroll 1
  for (uint32_t m = 1; m < npts; m++) {
    uint32_t dx[9], dy[9];
    f_copy(dx, nx);
    f_copy(dy, ny);
    if (m + 1u < npts)
      llaff_load(nx, ny, tab, kLLAux + kLLTeeth + i0 + (uint32_t)__builtin_ctz(m + 1u));
    const uint32_t g = ll_gray(m);
    if (!((g >> __builtin_ctz(m)) & 1u)) f_neg<P, 64>(dy, dy);  // digit back to -1
    (void)j_madd<P>(A, A, dx, dy, &same);                        // never degenerate
    llraw_store(tab, r0 + m, A);
    f_mul<P>(z, z, A.Z);
    llpre_store(tab, r0 + m, z);
  }
}

// Montgomery's trick backwards over raw slots [0, cnt) with pre[k] = prod of
// the Z of slots 0..k: each raw point made affine into the affine slot
// dst(k). inv = (pre[cnt - 1])^-1 on entry.
template <class P, class Dst>
BH_HD void ll_affine_back(uint32_t* tab, uint32_t cnt, uint32_t inv[9], Dst dst) {
#pragma unroll 1
  for (uint32_t c = cnt; c-- > 0;) {
    J30 E;
    llraw_load(E, tab, c);
    uint32_t zi[9], x[9], y[9];
    if (c > 0) {
      uint32_t pre[9];
      llpre_load(pre, tab, c - 1u);
      f_mul<P>(zi, inv, pre);
      f_mul<P>(inv, inv, E.Z);
    } else {
      f_copy(zi, inv);
    }
    ll_to_affine<P>(x, y, E, zi);
    llaff_store(tab, dst(c), x, y);
  }
}

template <class P>
BH_HD void lltab_build(uint32_t* tab, const Work& w, uint32_t rec, uint32_t* scr = nullptr) {
  // scr: the build scratch (aux / L / H / raw points / prefix products at the
  // slot's own offsets); the slot itself unless the caller has LDS for it
  // (k_reg_win: one table per workgroup)
  if (!scr) scr = tab;
  uint32_t one[9];
  f_const(one, P::r1);
  // 1. The doubling chain: chain point 2i = D_i = 2 B_i, 2i + 1 = B_(i+1);
  //    raw Jacobian copies and the running product of their Z, then all made
  //    affine with one inversion. B_0 = Q is affine already.
  J30 B;
  ld9(B.X, w.qx, rec, w.ns);
  ld9(B.Y, w.qy, rec, w.ns);
  llaff_store(scr, kLLAux, B.X, B.Y);
  f_copy(B.Z, one);
  uint32_t z[9];
#pragma unroll 1
  for (uint32_t i = 0; i + 1 < (uint32_t)kLLTeeth; i++) {
    j_dbl<P>(B, B);
    llraw_store(scr, 2u * i, B);
    if (i == 0) f_copy(z, B.Z);
    else f_mul<P>(z, z, B.Z);
    llpre_store(scr, 2u * i, z);
#pragma unroll 1
    for (int d = 1; d < kLLSpace; d++) j_dbl<P>(B, B);
    llraw_store(scr, 2u * i + 1u, B);
    f_mul<P>(z, z, B.Z);
    llpre_store(scr, 2u * i + 1u, z);
  }
  uint32_t inv[9];
  f_inv_sg<P>(inv, z);
  // D_i -> aux slot t + i; B_(i+1) -> aux slot i + 1
  ll_affine_back<P>(scr, kLLChain, inv, [](uint32_t c) {
    return (c & 1u) ? kLLAux + (c >> 1) + 1u : kLLAux + kLLTeeth + (c >> 1);
  });
  // 2. L (digits 0 .. a-1) and H (digits a .. t-2 + the top tooth) by two
  //    Gray walks into raw slots [0, NL) and [NL, NL + NH), one product chain,
  //    made affine with one inversion into L / H slots (by Gray index).
  ll_walk<P>(scr, 0u, kLLA, false, 0u, z, one);
  ll_walk<P>(scr, (uint32_t)kLLA, kLLTeeth - 1 - kLLA, true, kLLNL, z, one);
  f_inv_sg<P>(inv, z);
  ll_affine_back<P>(scr, kLLWalk, inv, [](uint32_t c) {
    return kLLLH + (c < kLLNL ? ll_gray(c) : kLLNL + ll_gray(c - kLLNL));
  });
  // 3. E[m] = H[m >> a] + L[m & (NL - 1)]: affine additions, the denominators
  //    x_H - x_L inverted together. Forward: their running products (pre);
  //    backward: lambda = (y_H - y_L) / (x_H - x_L), x = lambda^2 - x_H - x_L,
  //    y = lambda (x_L - x) - y_L (beta 34 each: the comb's mixed additions
  //    take beta <= 64).
  uint32_t hx[9], hy[9], lx[9], ly[9], d[9];
#pragma unroll 1
  for (uint32_t m = 0; m < kLLEnt; m++) {
    if ((m & (kLLNL - 1u)) == 0u) llaff_load(hx, hy, scr, kLLLH + kLLNL + (m >> kLLA));
    llaff_load(lx, ly, scr, kLLLH + (m & (kLLNL - 1u)));
    f_sub<P, 32>(d, hx, lx);                 // [b34], nonzero (H != +-L)
    if (m == 0) f_copy(z, d);
    else f_mul<P>(z, z, d);
    if (m + 1u < kLLEnt) llpre_store(scr, m, z);
  }
  f_inv_sg<P>(inv, z);
#pragma unroll 1
  for (uint32_t m = kLLEnt; m-- > 0;) {
    if (m == kLLEnt - 1u || (m & (kLLNL - 1u)) == kLLNL - 1u)
      llaff_load(hx, hy, scr, kLLLH + kLLNL + (m >> kLLA));
    llaff_load(lx, ly, scr, kLLLH + (m & (kLLNL - 1u)));
    f_sub<P, 32>(d, hx, lx);
    uint32_t di[9], lam[9], t[9], x[9], y[9];
    if (m > 0u) {
      uint32_t pre[9];
      llpre_load(pre, scr, m - 1u);
      f_mul<P>(di, inv, pre);                // (x_H - x_L)^-1
      f_mul<P>(inv, inv, d);
    } else {
      f_copy(di, inv);
    }
    f_sub<P, 32>(t, hy, ly);                 // [b34]
    f_mul<P>(lam, t, di);                    // [b2]
    f_sqr<P>(x, lam);                        // [b2]
    f_add(t, hx, lx);                        // [b4]
    f_sub<P, 32>(x, x, t);                   // [b34]
    f_sub<P, 64>(t, lx, x);                  // [b66]
    f_mul<P>(y, lam, t);                     // [b2]
    f_sub<P, 32>(y, y, ly);                  // [b34]
    llaff_store(tab, m, x, y);
  }
}

// ---- registry slots (round 5) ---------------------------------------------------
// A key kept in the device registry (bh_keys_register, BH_F_KEEP_KEYS) pays
// one build and is used for as long as it lives, so its slot holds BOTH forms
// a batch may need: the signed comb of one-lane batches (lltab_build's layout
// at offset 0: k_keycomb's folded Horner, 798 F_p ops per use instead of the
// windows' 1,040 + the 13-bit G comb's 220 + a final addition) and the 4-bit
// windows made AFFINE (kRegWin: 65 x 8 entries in the 80-byte llaff layout)
// for the multi-lane kernels of small batches, which split the windows over
// their lanes (a comb's doubling chain cannot be split): mixed additions, 11
// F_p ops per window instead of 16. Per-batch tables keep one form each.
constexpr uint32_t kRegWin = (kLLPre + 12u * kLLEnt + 3u) & ~3u;
constexpr uint32_t kRegWinRaw = kRegWin + (uint32_t)kKWin * kKEnt * kLLAff;
constexpr uint32_t kRegWinPre = kRegWinRaw + 28u * kKEnt;
static_assert(kRegWinPre + 12u * kKEnt <= kKTabWords && kRegWin % 4 == 0, "registry slot layout");
BH_HD uint32_t reg_win_offset() { return kRegWin; }

BH_HD void z_store(uint32_t* p, const uint32_t z[9]) {
  W4* d = reinterpret_cast<W4*>(p);
  d[0] = W4{z[0], z[1], z[2], z[3]};
  d[1] = W4{z[4], z[5], z[6], z[7]};
  d[2] = W4{z[8], 0u, 0u, 0u};
}
BH_HD void z_load(uint32_t z[9], const uint32_t* p) {
  const W4* s = reinterpret_cast<const W4*>(p);
  const W4 a = s[0], b = s[1], c = s[2];
  z[0] = a.x; z[1] = a.y; z[2] = a.z; z[3] = a.w;
  z[4] = b.x; z[5] = b.y; z[6] = b.z; z[7] = b.w;
  z[8] = c.x;
}

// The affine 4-bit windows of a registry slot. Window win from its base
// B = 16^win Q: the multiples B .. 8B (a co-Z doubling, then co-Z additions,
// as ktab_build; never degenerate), made affine with one inversion
// (Montgomery's trick over the 8 Z) -- ~140 F_p ops per window on top of the
// chain's 58. The raw points and the Z
// prefix products go through `raw` (store / load / store_z / load_z): the
// slot's own scratch when one lane builds every window (reg_build, the host
// harness), a column of LDS when each window has its own lane (k_reg_win).
template <class P, class Raw>
BH_HD void reg_window(uint32_t* tab, uint32_t win, const J30& B, Raw& raw) {
  J30 Bz, S;
  uint32_t z[9];
  raw.store(0u, B);
  f_copy(z, B.Z);
  raw.store_z(0u, z);
  j_dblu<P>(S, Bz, B);  // S = 2B, Bz = B on S's Z
  raw.store(1u, S);
  f_mul<P>(z, z, S.Z);
  raw.store_z(1u, z);
#pragma unroll 1
  for (uint32_t j = 2; j < (uint32_t)kKEnt; j++) {
    J30 T;
    j_zaddu<P>(T, Bz, S);  // T = (j+1) B; Bz onto T's Z
    raw.store(j, T);
    f_mul<P>(z, z, T.Z);
    raw.store_z(j, z);
    j_copy(S, T);
  }
  uint32_t inv[9];
  f_inv_sg<P>(inv, z);
#pragma unroll 1
  for (uint32_t j = (uint32_t)kKEnt; j-- > 0;) {
    J30 E;
    raw.load(E, j);
    uint32_t zi[9], x[9], y[9];
    if (j > 0) {
      uint32_t pz[9];
      raw.load_z(pz, j - 1u);
      f_mul<P>(zi, inv, pz);
      f_mul<P>(inv, inv, E.Z);
    } else {
      f_copy(zi, inv);
    }
    ll_to_affine<P>(x, y, E, zi);
    llaff_store(tab + kRegWin, win * (uint32_t)kKEnt + j, x, y);
  }
}

// reg_window's scratch in the slot itself (kRegWinRaw / kRegWinPre).
struct RegSlotRaw {
  uint32_t* tab;
  BH_HDM void store(uint32_t j, const J30& P) { ktab_store(tab + kRegWinRaw, 0, j, P); }
  BH_HDM void load(J30& P, uint32_t j) const { ktab_load(P, tab + kRegWinRaw, 0, j); }
  BH_HDM void store_z(uint32_t j, const uint32_t z[9]) { z_store(tab + kRegWinPre + 12u * j, z); }
  BH_HDM void load_z(uint32_t z[9], uint32_t j) const { z_load(z, tab + kRegWinPre + 12u * j); }
};

// The bases 16^win Q by four doublings each; the windows one after another.
template <class P>
BH_HD void ktab_build_aff(uint32_t* tab, const Work& w, uint32_t rec) {
  J30 B;
  ld9(B.X, w.qx, rec, w.ns);
  ld9(B.Y, w.qy, rec, w.ns);
  f_const(B.Z, P::r1);
  RegSlotRaw raw{tab};
#pragma unroll 1
  for (uint32_t win = 0; win < (uint32_t)kKWin; win++) {
    reg_window<P>(tab, win, B, raw);
    if (win + 1u < (uint32_t)kKWin) {
#pragma unroll 1
      for (int d = 0; d < kKW; d++) j_dbl<P>(B, B);
    }
  }
}

// A registry slot: the comb, then the affine windows (one lane, ~16.8k F_p
// ops once per key; the device splits it: reg_build_comb in the build kernel,
// the windows one lane each in k_reg_win).
template <class P>
BH_HD void reg_build(uint32_t* tab, const Work& w, uint32_t rec) {
  lltab_build<P>(tab, w, rec);
  ktab_build_aff<P>(tab, w, rec);
}
template <class P>
BH_HD void reg_build_comb(uint32_t* tab, const Work& w, uint32_t rec, uint32_t* scr = nullptr) {
  lltab_build<P>(tab, w, rec, scr);
}

// Curve constants of a base-field class (the order n for u2 + n).
template <class P>
using CvOf = typename std::conditional<P::a_is_minus3 != 0, Cv_p256, Cv_k1>::type;

// Column j of the signed comb: entry index and sign (V_j = +-E[idx]).
BH_HD void ll_column(const uint64_t sl[kLLTeeth], int j, uint32_t& idx, bool& neg) {
  uint32_t m = 0;
#pragma unroll
  for (int t = 0; t + 1 < kLLTeeth; t++) m |= (uint32_t)((sl[t] >> j) & 1ull) << t;
  neg = ((sl[kLLTeeth - 1] >> j) & 1ull) == 0ull;
  idx = neg ? (~m & (kLLEnt - 1u)) : m;
}

// The comb's tooth slices of u2: bits [s i, s i + s) of c = (k >> 1) | 2^(t s - 1).
template <class P>
BH_HD void ll_slices(uint64_t sl[kLLTeeth], const uint32_t u2[8]) {
  using Cv = CvOf<P>;
  const uint32_t add = (u2[0] & 1u) ? 0u : ~0u;  // even u2: k = u2 + n
  uint32_t k[9], c[9];
  uint64_t cy = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    cy += (uint64_t)u2[q] + (Cv::n[q] & add);
    k[q] = (uint32_t)cy;
    cy >>= 32;
  }
  k[8] = (uint32_t)cy;  // k < 2^257
#pragma unroll
  for (int q = 0; q < 8; q++) c[q] = (k[q] >> 1) | (k[q + 1] << 31);
  c[8] = 0u;
  c[(kLLTS - 1) >> 5] |= 1u << ((kLLTS - 1) & 31);
#pragma unroll
  for (int t = 0; t < kLLTeeth; t++) {
    const int lo = kLLSpace * t, wd = lo >> 5, sh = lo & 31;
    uint64_t x = (uint64_t)c[wd] >> sh;
    if (wd + 1 < 9) x |= (uint64_t)c[wd + 1] << (32 - sh);
    if (wd + 2 < 9 && sh + kLLSpace > 64) x |= (uint64_t)c[wd + 2] << (64 - sh);
    sl[t] = x & ((1ull << kLLSpace) - 1ull);
  }
}

// u2 Q from an affine signed comb table (Horner over the s columns, top first).
// stride 0: the per-batch table in global memory (16-byte loads of its 80-byte
// slots); else entries `stride` words apart read by llent_load (k_keycomb's
// LDS copy, or the global table when the workgroup's copy is full).
template <class P>
BH_HD void q_llcomb(J30& A, bool& a_inf, const Work& w, uint32_t i, const uint32_t* tab,
                    uint32_t stride = 0) {
  uint32_t u2[8], one[9];
  ld8(u2, w.r, i, w.ns);
  f_const(one, P::r1);
  uint64_t sl[kLLTeeth];
  ll_slices<P>(sl, u2);
  uint32_t idx;
  bool neg;
  ll_column(sl, kLLSpace - 1, idx, neg);  // top column: top bit set, +E[idx]
  if (stride) llent_load(A.X, A.Y, tab + idx * stride);
  else llaff_load(A.X, A.Y, tab, idx);
  f_copy(A.Z, one);
  a_inf = false;
#pragma unroll 1
  for (int j = kLLSpace - 2; j >= 0; j--) {
    j_dbl<P>(A, A);  // (while a_inf, A is a placeholder the next point replaces)
    ll_column(sl, j, idx, neg);
    uint32_t tx[9], ty[9], nty[9];
    if (stride) llent_load(tx, ty, tab + idx * stride);
    else llaff_load(tx, ty, tab, idx);
    f_neg<P, 64>(nty, ty);
    f_sel(ty, neg, nty, ty);
    bool same;
    const bool deg = j_madd<P>(A, A, tx, ty, &same);
    if (a_inf || deg) {  // rare (crafted scalars): lanes skip this together
      if (a_inf || same) {  // A was infinity: V; A == V: 2 V
        J30 T;
        f_copy(T.X, tx);
        f_copy(T.Y, ty);
        f_copy(T.Z, one);
        if (a_inf) j_copy(A, T);
        else j_dbl<P>(A, T);
        a_inf = false;
      } else {  // A == -V
        a_inf = true;
      }
    }
  }
}

// ---- u1 G folded into the key comb's Horner (round 5) ---------------------------
// The G half shares the key comb's s - 1 = 36 doublings. u1 is recoded like u2
// (ll_slices: k = u1 or u1 + n, t = 7 teeth x s = 37 columns, digits +-1), so
// u1 G = sum_j 2^j W_j G with W_j = sum_i d_(i,j) 2^(s i). The Horner adds the
// columns in groups of kGF (BH_GFOLD, default 3): the group of columns
// j, .., j + kGF - 1 (j = 1, 1 + kGF, ..., s - kGF) as ONE point
//   (sum_c 2^c W_(j+c)) G
// at column j (adding W_(j+c) c columns late, doubled c times, is the same
// sum), and column 0 alone. The group table holds the sign patterns whose top
// digit (tooth t - 1 of column j + kGF - 1) is +1 -- every entry a positive
// multiple of G below 2^(225 + kGF), never infinity; the other half are their
// negatives -- and the single-column table the 2^(t-1) patterns of one column
// with its top digit +1. kGF = 2: 8,192 + 64 affine points, 660 KB per curve
// (L2-resident), 18 + 1 = 19 mixed additions per record; kGF = 3: 2^20 + 64
// points, 84 MB (MALL), 12 + 1 = 13. Built at bh_init. Against the separate
// 13-bit G comb (20 mixed additions) the fold also drops the u1 G partial sum
// the build kernel stored and k_keycomb reloaded, and the final addition A + B.
#ifndef BH_GFOLD
#define BH_GFOLD 3  // same box (profiles/r05/v6): 2 columns 179.8 / 180.6, 3 columns 188.5 / 189.2 M/s
#endif
constexpr int kGF = BH_GFOLD;
static_assert(kGF >= 1 && kGF <= 4 && (kLLSpace - 1) % kGF == 0,
              "column groups of the folded G tables tile columns 1 .. s - 1");
constexpr int kGFBits = (kLLTeeth - 1) + (kGF - 1) * kLLTeeth;  // group entry index bits
constexpr uint32_t kG2Ent = 1u << kGFBits;                        // group entries
constexpr uint32_t kG1Ent = kLLEnt;                               // single-column entries
constexpr int kGAdds = (kLLSpace - 1) / kGF + 1;                  // G additions per record
// base points of the tables' construction: (2 m + 1) 2^(s i) G, i < t, m < 2^(kGF-1)
constexpr uint32_t kGOdd = 1u << (kGF - 1);
constexpr uint32_t kGBase = (uint32_t)kLLTeeth * kGOdd;
constexpr size_t kG2Words = (size_t)(kG2Ent + kG1Ent + kGBase) * kLLAff;
// Per curve, one device buffer holds the 13-bit G comb (ladder records,
// registry-table records, small batches) and, after it, the folded tables
// (group entries, single-column entries, base points).
constexpr size_t kGCombWords = (size_t)kCombWindows * kCombEntries * kGEntry;
constexpr size_t kGTabAllWords = kGCombWords + kG2Words;
static_assert(kGCombWords % 4 == 0, "folded tables 16-byte aligned");
BH_HD const uint32_t* g2_of(const uint32_t* gtab) { return gtab + kGCombWords; }

// v G for v < 2^288 (v != 0) by left-to-right double-and-add from the affine
// G, made affine (Fermat inverse). A = m G with 2 <= m < v before every
// addition, never +-G, for v < n. Init-time only.
template <class P>
BH_HD void scalar_g_affine(const uint32_t v[9], uint32_t x[9], uint32_t y[9]) {
  uint32_t gx[9], gy[9];
  f_const(gx, P::gx_m);
  f_const(gy, P::gy_m);
  int topbit = 287;
  while (topbit > 0 && !((v[topbit >> 5] >> (topbit & 31)) & 1u)) topbit--;
  J30 A;
  f_copy(A.X, gx);
  f_copy(A.Y, gy);
  f_const(A.Z, P::r1);
  for (int b = topbit - 1; b >= 0; b--) {
    j_dbl<P>(A, A);
    if ((v[b >> 5] >> (b & 31)) & 1u) {
      bool same;
      (void)j_madd<P>(A, A, gx, gy, &same);
    }
  }
  uint32_t z[9], zi[9], zi2[9];
  f_reduce<P>(z, A.Z);
  f_inv<P>(zi, z);
  f_sqr<P>(zi2, zi);
  f_mul<P>(x, A.X, zi2);
  f_mul<P>(zi2, zi2, zi);
  f_mul<P>(y, A.Y, zi2);
  f_reduce<P>(x, x);
  f_reduce<P>(y, y);
}

// Base point k = i * kGOdd + m of the folded tables: (2 m + 1) 2^(s i) G,
// affine, at slot kG2Ent + kG1Ent + k. One lane per point (init kernel 1).
template <class P>
BH_HD void gtab2_base(uint32_t k, uint32_t* g2) {
  const uint32_t i = k / kGOdd, m = k % kGOdd;
  uint32_t v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const int b = kLLSpace * (int)i;
  const uint64_t mag = (uint64_t)(2u * m + 1u) << (b & 31);
  v[b >> 5] = (uint32_t)mag;
  if ((b >> 5) + 1 < 9) v[(b >> 5) + 1] = (uint32_t)(mag >> 32);
  uint32_t x[9], y[9];
  scalar_g_affine<P>(v, x, y);
  llaff_store(g2, kG2Ent + kG1Ent + k, x, y);
}

// Entry t of the folded tables (init kernel 2, after the base points): t <
// kG2Ent a group pattern -- index bits, most significant first: the top
// column's lower t - 1 teeth (its top tooth is +1), then the other kGF - 1
// columns' t teeth each, highest column first; else the single column
// (1 << (t - 1)) | (t - kG2Ent). The point sum_i c_i 2^(s i) G with odd c_i,
// |c_i| < 2^kGF, c_(t-1) > 0, from the top term down by mixed additions of
// +-base points (a partial sum above 2^(s (i+1)) - ... never meets +-|c_i|
// 2^(s i) G), made affine by safegcd. Affine radix-2^30 Montgomery in the
// 80-byte llaff layout.
template <class P>
BH_HD void gtab2_entry(uint32_t t, uint32_t* g2) {
  constexpr uint32_t top = 1u << (kLLTeeth - 1), all = (1u << kLLTeeth) - 1u;
  int c[kLLTeeth];
  for (int i = 0; i < kLLTeeth; i++) c[i] = 0;
  if (t < kG2Ent) {
    for (int cc = 0; cc < kGF; cc++) {  // column cc of the group (0 = lowest)
      const uint32_t bits = cc == kGF - 1 ? (top | (t >> ((kGF - 1) * kLLTeeth)))
                                          : (t >> (cc * kLLTeeth)) & all;
      for (int i = 0; i < kLLTeeth; i++) c[i] += (2 * (int)((bits >> i) & 1u) - 1) << cc;
    }
  } else {
    const uint32_t b = top | (t - kG2Ent);
    for (int i = 0; i < kLLTeeth; i++) c[i] = 2 * (int)((b >> i) & 1u) - 1;
  }
  J30 A;
  llaff_load(A.X, A.Y, g2, kG2Ent + kG1Ent + (uint32_t)(kLLTeeth - 1) * kGOdd +
                               (uint32_t)((c[kLLTeeth - 1] - 1) / 2));
  f_const(A.Z, P::r1);
  for (int i = kLLTeeth - 2; i >= 0; i--) {
    const int a = c[i] < 0 ? -c[i] : c[i];
    uint32_t bx[9], by[9];
    llaff_load(bx, by, g2, kG2Ent + kG1Ent + (uint32_t)i * kGOdd + (uint32_t)((a - 1) / 2));
    if (c[i] < 0) f_neg<P, 64>(by, by);
    bool same;
    (void)j_madd<P>(A, A, bx, by, &same);  // never degenerate (see above)
  }
  uint32_t zi[9], x[9], y[9];
  f_inv_sg<P>(zi, A.Z);
  ll_to_affine<P>(x, y, A, zi);
  llaff_store(g2, t, x, y);
}

// The folded G entry added at column j of u1's slices: the group of columns
// j .. j + kGF - 1 (j >= 1), the single column for j = 0 (index past the
// group table). neg: the entry's negative (all digits flipped).
BH_HD void g2_column(const uint64_t gl[kLLTeeth], int j, uint32_t& idx, bool& neg) {
  if (j == 0) {
    ll_column(gl, 0, idx, neg);
    idx += kG2Ent;
    return;
  }
  constexpr uint32_t all = (1u << kLLTeeth) - 1u;
  uint32_t col[kGF];
#pragma unroll
  for (int cc = 0; cc < kGF; cc++) {
    uint32_t b = 0;
#pragma unroll
    for (int t = 0; t < kLLTeeth; t++) b |= (uint32_t)((gl[t] >> (j + cc)) & 1ull) << t;
    col[cc] = b;
  }
  neg = ((col[kGF - 1] >> (kLLTeeth - 1)) & 1u) == 0u;
  uint32_t x = col[kGF - 1] & (all >> 1);
  if (neg) x = ~col[kGF - 1] & (all >> 1);
#pragma unroll
  for (int cc = kGF - 2; cc >= 0; cc--) x = (x << kLLTeeth) | ((neg ? ~col[cc] : col[cc]) & all);
  idx = x;
}

// A += +-(tx, ty) with the explicit degenerate cases (A at infinity: A = T;
// A == T: 2 T; A == -T: infinity), as a branch the lanes skip together.
template <class P>
BH_HD void ll_madd(J30& A, bool& a_inf, const uint32_t tx[9], uint32_t ty[9], bool neg,
                   const uint32_t one[9]) {
  bool same;
  const bool deg = j_madd<P>(A, A, tx, ty, &same, neg);  // the sign in its r pass
  if (a_inf || deg) {  // rare (crafted scalars)
    if (neg) f_neg<P, 64>(ty, ty);
    if (a_inf || same) {
      J30 T;
      f_copy(T.X, tx);
      f_copy(T.Y, ty);
      f_copy(T.Z, one);
      if (a_inf) j_copy(A, T);
      else j_dbl<P>(A, T);
      a_inf = false;
    } else {
      a_inf = true;
    }
  }
}

// A = 2 A + T (T = +-(tx, ty)) as (A + T) + A: a mixed addition that also
// rescales A onto the sum's Z (j_madd_co), then a co-Z addition (j_zaddu):
// 8M + 3S + 5M + 2S = 18 F_p ops against a doubling + a mixed addition's 19
// (round 5). Degenerate cases, as branches the lanes skip together: A at
// infinity -> T; A == T -> 3 T = 2 T + T; A == -T -> A; A + T == -A (the
// co-Z sum's x difference is 0; A + T == A would need T = 0) -> infinity.
// Round 6: the sign of T is folded into the mixed addition's r pass (f_csub);
// ty is negated in place only on the rare branches that use T itself.
template <class P>
BH_HD void ll_dbladd(J30& A, bool& a_inf, const uint32_t tx[9], uint32_t ty[9], bool neg,
                     const uint32_t one[9]) {
  if (a_inf) {  // rare: 2 inf + T
    if (neg) f_neg<P, 64>(ty, ty);
    f_copy(A.X, tx);
    f_copy(A.Y, ty);
    f_copy(A.Z, one);
    a_inf = false;
    return;
  }
  J30 R, Az;
  bool same;
  if (j_madd_co<P>(R, Az, A, tx, ty, &same, neg)) {  // rare: A == +-T
    if (neg) f_neg<P, 64>(ty, ty);
    J30 T;
    f_copy(T.X, tx);
    f_copy(T.Y, ty);
    f_copy(T.Z, one);
    if (same) {
      j_dbl<P>(A, T);
      (void)j_madd<P>(A, A, tx, ty, &same);  // 2 T + T: 2 T != +-T (prime order)
    }  // else A == -T: 2 A + T = A, unchanged
    return;
  }
  j_zaddu<P>(A, R, Az);
  if (f_is_zero2<P>(A.Z)) a_inf = true;  // rare: A + T == -A
}

// u1 G + u2 Q from the key's signed comb table (stride as q_llcomb) and the
// folded G tables g2: Horner from the top column; at column j A = 2 A + V_j Q
// (ll_dbladd), and at the lowest column of each G group and at j = 0 the
// folded G entry (loaded one group ahead).
template <class P>
BH_HD void q_llcomb_g(J30& A, bool& a_inf, const Work& w, uint32_t i, const uint32_t* tab,
                      uint32_t stride, const uint32_t* g2) {
  uint32_t u2[8], u1[8], one[9];
  ld8(u2, w.r, i, w.ns);
  ld8(u1, w.e, i, w.ns);
  f_const(one, P::r1);
  uint64_t sl[kLLTeeth], gl[kLLTeeth];
  ll_slices<P>(sl, u2);
  ll_slices<P>(gl, u1);
  uint32_t idx;
  bool neg;
  ll_column(sl, kLLSpace - 1, idx, neg);  // top column: top bit set, +E[idx]
  if (stride) llent_load(A.X, A.Y, tab + idx * stride);
  else llaff_load(A.X, A.Y, tab, idx);
  f_copy(A.Z, one);
  a_inf = false;
  uint32_t gx[9], gy[9], gidx;
  bool gneg;
  g2_column(gl, kLLSpace - kGF, gidx, gneg);
  llaff_load(gx, gy, g2, gidx);
#pragma unroll 1
  for (int j = kLLSpace - 2; j >= 0; j--) {
    {
      uint32_t tx[9], ty[9];
      ll_column(sl, j, idx, neg);
      if (stride) llent_load(tx, ty, tab + idx * stride);
      else llaff_load(tx, ty, tab, idx);
      ll_dbladd<P>(A, a_inf, tx, ty, neg, one);  // A = 2 A + V_j Q
    }
    if (j == 0 || (j - 1) % kGF == 0) {
      ll_madd<P>(A, a_inf, gx, gy, gneg, one);
      if (j > 0) {  // the next folded G entry: the group at j - kGF, or column 0
        g2_column(gl, j > kGF ? j - kGF : 0, gidx, gneg);
        llaff_load(gx, gy, g2, gidx);
      }
    }
  }
}

template <class P>
BH_HD bool stage_keycomb_fold(const Work& w, uint32_t i, const uint32_t* tab, uint32_t stride,
                              const uint32_t* g2) {
  J30 A;
  bool a_inf;
  q_llcomb_g<P>(A, a_inf, w, i, tab, stride, g2);
  return finish_check<P>(w, i, A, a_inf, A, true);
}

// ---- variable-base ladder with u1 G folded in (round 5; P-256) ---------------
// u2 Q by odd signed 5-bit windows -- the regular recoding: k = u2, or u2 + n
// when u2 is even, is odd; digit i = 2 b_i - 31 with b_i = bits [5i+1, 5i+5]
// of k (odd, nonzero, in [-31, 31]), the top digit (i = 51) 2 bit_256 + 1 > 0
// -- so every window is A = 32 A + d_i Q = 2 (16 A) + d_i Q: 4 doublings and
// the composite (A + T) + A (j_dbladd: j_add_co + j_zaddu, 16 + 7 F_p ops
// against a doubling's 8 + an addition's 16) with no zero digit to skip. The
// table holds the odd multiples Q, 3 Q, ..., 31 Q from a co-Z chain (DBLU + 15
// ZADDU: 114 F_p ops against 162 for 1..16 Q). u1 G is folded into the same
// doubling chain: the folded G groups of k_keycomb (g2_column: kGF columns of
// u1's 7 x 37 comb, weight 2^j at j = 0, 1, 1 + kGF, ..., 37 - kGF) are mixed
// additions at the doubling positions with that weight (the last 7 windows):
// 13 of them against the 13-bit G comb's 20 plus the final A + B. Per verify
// ~3,070 F_p ops against ~3,280 (3,200).
//
// A = 2 A + (+-T) for a Jacobian T (neg: -T, the sign folded into the
// addition's r pass; T.Y is negated in place only on the rare branches that
// use T itself), degenerate cases as ll_dbladd: A at infinity -> T; A == T -> 3 T; A == -T -> A (unchanged);
// A + T == -A -> infinity.
#ifndef BH_LADDER_CSUB
#define BH_LADDER_CSUB 1
#endif
template <class P>
BH_HD void j_dbladd(J30& A, bool& a_inf, J30& T, bool neg) {
  if (a_inf) {  // rare: 2 inf + T
    if (neg) f_neg<P, 64>(T.Y, T.Y);
    j_copy(A, T);
    a_inf = false;
    return;
  }
  J30 R, Az;
  bool same;
  if (j_add_co<P>(R, Az, A, T, &same, neg)) {  // rare: A == +-T (the sign in its r pass)
    if (neg) f_neg<P, 64>(T.Y, T.Y);
    if (same) {
      J30 D;
      j_dbl<P>(D, T);
      (void)j_add<P>(A, D, T, &same);  // 2 T + T: 2 T != +-T (prime order)
    }  // else A == -T: 2 A + T = A, unchanged
    return;
  }
  j_zaddu<P>(A, R, Az);
  if (f_is_zero2<P>(A.Z)) a_inf = true;  // rare: A + T == -A
}

// the doubling positions (remaining doublings = weight exponent) that take a
// folded G entry: 0 (column 0) and the groups' lowest columns 1, 1 + kGF, ...
BH_HD bool g_fold_pos(int p) { return p == 0 || (p >= 1 && p <= kLLSpace - kGF && (p - 1) % kGF == 0); }

template <class P>
BH_HD void q_ladder_odd_g(J30& A, bool& a_inf, const Work& w, uint32_t i, uint32_t wave,
                          uint32_t lane, const uint32_t* g2) {
  using Cv = CvOf<P>;
  uint32_t u2[8], u1[8], qx[9], qy[9], one[9];
  ld8(u2, w.r, i, w.ns);
  ld8(u1, w.e, i, w.ns);
  ld9(qx, w.qx, i, w.ns);
  ld9(qy, w.qy, i, w.ns);
  f_const(one, P::r1);
  // odd multiples (2m + 1) Q, m = 0..15: DBLU, then S += D by ZADDU (D rescaled)
  {
    J30 Qa, D, S;
    f_copy(Qa.X, qx);
    f_copy(Qa.Y, qy);
    f_copy(Qa.Z, one);
    j_dblu<P>(D, S, Qa);  // D = 2 Q, S = Q on D's Z
    qtab_store(w.qtab, wave, 0, lane, S);
#pragma unroll 1
    for (uint32_t m = 1; m < (uint32_t)kQTab; m++) {
      J30 Sn;
      j_zaddu<P>(Sn, D, S);  // Sn = (2m + 1) Q; D onto Sn's Z (never degenerate)
      qtab_store(w.qtab, wave, m, lane, Sn);
      j_copy(S, Sn);
    }
  }
  // k = u2 (odd) or u2 + n, shifted so bit b sits at 288-bit position b + 30:
  // window i's bits [5i+1, 5i+5] reach K[8] bits 25..29 after 50 - i shifts
  uint32_t K[9];
  {
    const uint32_t add = (u2[0] & 1u) ? 0u : ~0u;
    uint32_t k[9];
    uint64_t cy = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      cy += (uint64_t)u2[q] + (Cv::n[q] & add);
      k[q] = (uint32_t)cy;
      cy >>= 32;
    }
    k[8] = (uint32_t)cy;
    K[0] = k[0] << 30;
#pragma unroll
    for (int q = 1; q < 9; q++) K[q] = (k[q] << 30) | (k[q - 1] >> 2);
  }
  uint64_t gl[kLLTeeth];
  ll_slices<P>(gl, u1);
  uint32_t gx[9], gy[9], gidx;
  bool gneg;
  int gp = kLLSpace - kGF;  // the next folded G position (descending)
  g2_column(gl, gp, gidx, gneg);
  llaff_load(gx, gy, g2, gidx);
  auto g_add = [&]() {
    ll_madd<P>(A, a_inf, gx, gy, gneg, one);
    if (gp > 0) {
      gp = gp > kGF ? gp - kGF : 0;
      g2_column(gl, gp, gidx, gneg);
      llaff_load(gx, gy, g2, gidx);
    }
  };
  qtab_load(A, w.qtab, wave, (K[8] >> 30) & 1u, lane);  // top digit 2 bit_256 + 1: Q or 3 Q
  a_inf = false;
#pragma unroll 1
  for (int win = 50; win >= 0; win--) {
    const uint32_t b = (K[8] >> 25) & 31u;
#pragma unroll
    for (int q = 8; q > 0; q--) K[q] = (K[q] << 5) | (K[q - 1] >> 27);
    K[0] <<= 5;
    const bool neg = b < 16u;
    const uint32_t mag = neg ? 31u - 2u * b : 2u * b - 31u;
    J30 T;
    qtab_load(T, w.qtab, wave, (mag - 1u) >> 1, lane);  // issued before the doublings
#pragma unroll 1
    for (int d = 1; d <= 4; d++) {
      j_dbl<P>(A, A);  // (while a_inf, A is a placeholder the next point replaces)
      if (g_fold_pos(5 * win + 5 - d)) g_add();
    }
#if BH_LADDER_CSUB
    j_dbladd<P>(A, a_inf, T, neg);
#else
    if (neg) f_neg<P, 64>(T.Y, T.Y);
    j_dbladd<P>(A, a_inf, T, false);
#endif
    if (g_fold_pos(5 * win)) g_add();
  }
}

// One-lane ladder records: P-256 through the odd-window ladder with u1 G
// folded in; secp256k1 through the GLV ladder + the 13-bit G comb.
template <class P>
BH_HD bool stage_ladder_fold(const Work& w, const uint32_t* gtab, uint32_t i, uint32_t wave,
                             uint32_t lane) {
  if constexpr (P::a_is_minus3) {
    J30 A;
    bool a_inf;
    q_ladder_odd_g<P>(A, a_inf, w, i, wave, lane, g2_of(gtab));
    return finish_check<P>(w, i, A, a_inf, A, true);
  } else {
    return stage_ladder<P>(w, gtab, i, wave, lane);
  }
}

template <class P>
BH_HD bool stage_keycomb(const Work& w, const uint32_t* gtab, uint32_t i, const uint32_t* tab,
                         bool aff = false) {
  J30 A, B;
  bool a_inf, b_inf;
  q_keycomb<P>(A, a_inf, w, i, tab, aff);
  uint32_t u1[8];
  ld8(u1, w.e, i, w.ns);
  g_comb<P>(B, b_inf, gtab, u1);
  return finish_check<P>(w, i, A, a_inf, B, b_inf);
}

// Split key comb (large batches). The u1 G half does not need the key tables,
// so k_ktab_ladder computes it for every key-comb record WHILE the tables are
// built (the build runs one wave per SIMD and leaves issue slots free), and
// k_keycomb then only adds the 65 table points and the stored u1 G. Stored by
// list position j, SoA, so both sides are coalesced.
constexpr uint32_t kGPartWords = 28;
template <class P>
BH_HD void stage_gpart(const Work& w, const uint32_t* gtab, uint32_t i, uint32_t j) {
  J30 B;
  bool b_inf;
  uint32_t u1[8];
  ld8(u1, w.e, i, w.ns);
  g_comb<P>(B, b_inf, gtab, u1);
  uint32_t* o = w.gpart + j;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    o[(size_t)k * w.ns] = B.X[k];
    o[(size_t)(9 + k) * w.ns] = B.Y[k];
    o[(size_t)(18 + k) * w.ns] = B.Z[k];
  }
  o[(size_t)27 * w.ns] = b_inf ? 1u : 0u;
}

template <class P>
BH_HD bool stage_keycomb_q(const Work& w, uint32_t i, uint32_t j, const uint32_t* tab,
                           bool ll = false, uint32_t stride = 0, bool aff = false) {
  J30 A, B;
  bool a_inf;
  if (ll) q_llcomb<P>(A, a_inf, w, i, tab, stride);  // a per-batch Lim-Lee comb table
  else q_keycomb<P>(A, a_inf, w, i, tab, aff);
  const uint32_t* o = w.gpart + j;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    B.X[k] = o[(size_t)k * w.ns];
    B.Y[k] = o[(size_t)(9 + k) * w.ns];
    B.Z[k] = o[(size_t)(18 + k) * w.ns];
  }
  const bool b_inf = o[(size_t)27 * w.ns] != 0;
  return finish_check<P>(w, i, A, a_inf, B, b_inf);
}

// 64-bit key fingerprint of the canonical Montgomery Q (never 0).
BH_HD uint64_t key_hash(const Work& w, uint32_t i) {
  uint32_t qx[9], qy[9];
  ld9(qx, w.qx, i, w.ns);
  ld9(qy, w.qy, i, w.ns);
  uint64_t h = 0x9e3779b97f4a7c15ull;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    h ^= qx[k];
    h *= 0xff51afd7ed558ccdull;
    h ^= (uint64_t)qy[k] << 32;
    h ^= h >> 29;
  }
  return h ? h : 1;
}

BH_HD bool same_key(const Work& w, uint32_t a, uint32_t b) {
  uint32_t xa[9], ya[9], xb[9], yb[9];
  ld9(xa, w.qx, a, w.ns);
  ld9(ya, w.qy, a, w.ns);
  ld9(xb, w.qx, b, w.ns);
  ld9(yb, w.qy, b, w.ns);
  uint32_t d = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) d |= (xa[k] ^ xb[k]) | (ya[k] ^ yb[k]);
  return d == 0;
}


// ------------------------------------------------------------ key registry
// Persistent per-device, per-curve store of key tables (include/bdls_hip.h
// bh_keys_register / BH_F_KEEP_KEYS): an open-addressed fingerprint table ->
// table index, the canonical Montgomery key per table (full compare on every
// hit) and the tables themselves (kKTabWords words each, same layout as the
// per-batch tables). Entries are only added (bh_keys_clear resets), and a
// fingerprint slot is published only after its table is complete.
struct KeyReg {
  uint32_t cap;         // tables (0 = registry not allocated)
  uint32_t hc;          // fingerprint slots (power of two >= 2 cap)
  uint64_t* slot_hash;  // [hc] 0 = empty
  uint32_t* slot_tab;   // [hc]
  uint32_t* keys;       // [cap][18] qx || qy (canonical radix-2^30 Montgomery)
  uint32_t* tables;     // [cap][kKTabWords]
  uint32_t* count;      // [1] tables handed out (may exceed cap; clamp on read)
};

// Table ids: registry index, or kLocal | per-batch plan index.
constexpr uint32_t kLocal = 0x80000000u;

BH_HD const uint32_t* tab_ptr(const Plan& pl, const KeyReg& g, uint32_t id) {
  return (id & kLocal) ? pl.tables + (size_t)(id & ~kLocal) * kKTabWords
                       : g.tables + (size_t)id * kKTabWords;
}

BH_HD bool reg_key_eq(const KeyReg& g, uint32_t t, const Work& w, uint32_t i) {
  const uint32_t* k = g.keys + (size_t)t * 18;
  uint32_t qx[9], qy[9];
  ld9(qx, w.qx, i, w.ns);
  ld9(qy, w.qy, i, w.ns);
  uint32_t d = 0;
#pragma unroll
  for (int q = 0; q < 9; q++) d |= (k[q] ^ qx[q]) | (k[9 + q] ^ qy[q]);
  return d == 0;
}

BH_HD void reg_key_store(const KeyReg& g, uint32_t t, const Work& w, uint32_t i) {
  uint32_t* k = g.keys + (size_t)t * 18;
  uint32_t qx[9], qy[9];
  ld9(qx, w.qx, i, w.ns);
  ld9(qy, w.qy, i, w.ns);
#pragma unroll
  for (int q = 0; q < 9; q++) {
    k[q] = qx[q];
    k[9 + q] = qy[q];
  }
}

// Registry table for record i's key, or kNone.
BH_HD uint32_t reg_lookup(const KeyReg& g, const Work& w, uint32_t i, uint64_t h) {
  if (g.cap == 0) return kNone;
  const uint32_t mask = g.hc - 1;
  uint32_t p = (uint32_t)h & mask;
  for (uint32_t probe = 0; probe < g.hc; probe++) {
    const uint64_t cur = g.slot_hash[p];
    if (cur == 0) return kNone;
    if (cur == h) {
      const uint32_t t = g.slot_tab[p];
      if (t < g.cap && reg_key_eq(g, t, w, i)) return t;
    }
    p = (p + 1) & mask;
  }
  return kNone;
}

// ------------------------------------------------------- wide key comb
// For batches far smaller than the chip (block validation, one BDLS round),
// L lanes share one record: lane l of the group adds the key-table windows
// win = l, l + L, ... and the G-comb windows likewise, then the L partial
// sums are combined by a butterfly over the group. The signed digits come
// from one offset addition instead of a carry scan (recode_koff for the key
// tables, recode_goff for the G comb), so every lane reads its windows
// directly. These digits (in [-8, 7]) differ from q_keycomb's carry-scan
// digits (in [-7, 8]) but represent the same scalar, so the sums are the same
// point; the two paths may meet the rare degenerate addition (A = +-T) on
// different inputs, and both resolve it exactly (tests/test_hostsim.py and
// tests/test_bdls.py run crafted scalars through both).

// o = v >> sh (288-bit), 0 <= sh < 192
BH_HD void shr288(uint32_t o[9], const uint32_t v[9], uint32_t sh) {
  const uint32_t ws = sh >> 5, bs = sh & 31u;
  uint32_t t[9];
#pragma unroll
  for (int q = 0; q < 9; q++) {
    uint32_t x = 0;
#pragma unroll
    for (uint32_t d = 0; d < 9; d++)  // every word shift of a 288-bit value
      if (ws == d) x = (q + (int)d < 9) ? v[q + d] : 0u;
    t[q] = x;
  }
#pragma unroll
  for (int q = 0; q < 9; q++) {
    const uint32_t hi = (q + 1 < 9) ? t[q + 1] : 0u;
    o[q] = bs ? ((t[q] >> bs) | (hi << (32 - bs))) : t[q];
  }
}

// Acc += T (Jacobian), with infinity flags and the explicit degenerate cases.
template <class P>
BH_HD void j_acc(J30& A, bool& a_inf, const J30& T, bool t_inf) {
  J30 R;
  bool same;
  const bool deg = j_add<P>(R, A, T, &same);
  const bool take = !t_inf;
  const bool use_t = take && a_inf;
  const bool use_r = take && !a_inf && !deg;
  const bool rare = take && !a_inf && deg;
  j_sel(A, use_r, R, A);
  j_sel(A, use_t, T, A);
  if (rare) {
    if (same) j_dbl<P>(A, T);
    else a_inf = true;
  }
  if (use_t) a_inf = false;
}

// Acc += (tx, ty) affine (mixed addition).
template <class P>
BH_HD void j_acc_aff(J30& A, bool& a_inf, const uint32_t tx[9], const uint32_t ty[9],
                     const uint32_t one[9], bool t_inf) {
  J30 R;
  bool same;
  const bool deg = j_madd<P>(R, A, tx, ty, &same);
  const bool take = !t_inf;
  const bool use_t = take && a_inf;
  const bool use_r = take && !a_inf && !deg;
  const bool rare = take && !a_inf && deg;
  j_sel(A, use_r, R, A);
  if (use_t) {
    f_copy(A.X, tx);
    f_copy(A.Y, ty);
    f_copy(A.Z, one);
  }
  if (rare) {
    if (same) {
      J30 T;
      f_copy(T.X, tx);
      f_copy(T.Y, ty);
      f_copy(T.Z, one);
      j_dbl<P>(A, T);
    } else {
      a_inf = true;
    }
  }
  if (use_t) a_inf = false;
}

template <class P, int L>
BH_HD void g_comb_part(J30& C, bool& c_inf, const uint32_t* gtab, const uint32_t u1[8],
                       uint32_t l);  // below

// Lane l's u2 Q windows (win = l, l + L, ...) of the key table.
template <class P, int L>
BH_HD void keycomb_q_part(J30& C, bool& c_inf, const Work& w, uint32_t i, const uint32_t* tab,
                          uint32_t l, bool aff = false) {
  uint32_t k[8], v[9], sv[9], one[9];
  f_const(one, P::r1);
  f_const(C.X, P::r1);
  f_const(C.Y, P::r1);
  f_const(C.Z, P::r1);
  c_inf = true;
  ld8(k, w.r, i, w.ns);
  recode_koff(v, k);
  shr288(sv, v, (uint32_t)kKW * l);
  for (int m = 0; m * L < kKWin; m++) {
    const uint32_t win = l + (uint32_t)(m * L);
    const int d = (int)(sv[0] & (2u * kKEnt - 1u)) - kKEnt;
    shr_const<kKW * L>(sv);
    if (win < (uint32_t)kKWin) {
      const uint32_t mag = (uint32_t)(d < 0 ? -d : d);
      J30 T;
      win_entry<P>(T, tab, win, mag ? mag - 1 : 0, aff, one);
      if (d < 0) f_neg<P, 64>(T.Y, T.Y);
      if (aff) j_acc_aff<P>(C, c_inf, T.X, T.Y, one, mag == 0);  // mixed: 11 F_p ops
      else j_acc<P>(C, c_inf, T, mag == 0);
    }
  }
}

// Lane l's partial sum C = sum over its windows of (key-table digit points
// + G-comb digit points).
template <class P, int L>
BH_HD void keycomb_part(J30& C, bool& c_inf, const Work& w, const uint32_t* gtab, uint32_t i,
                        const uint32_t* tab, uint32_t l, bool aff = false) {
  keycomb_q_part<P, L>(C, c_inf, w, i, tab, l, aff);  // u2 Q: 4-bit windows win = l + m L
  uint32_t k[8];
  ld8(k, w.e, i, w.ns);
  g_comb_part<P, L>(C, c_inf, gtab, k, l);        // u1 G: kGW-bit windows win = l + m L
}

// C += the G-comb windows win = l, l + L, ... of u1 G (kGW-bit signed digits
// from one offset addition, recode_goff).
template <class P, int L>
BH_HD void g_comb_part(J30& C, bool& c_inf, const uint32_t* gtab, const uint32_t u1[8],
                       uint32_t l) {
  uint32_t v[9], sv[9];
  recode_goff(v, u1);
  shr288(sv, v, (uint32_t)kGW * l);
  uint32_t one[9];
  f_const(one, P::r1);
  for (int m = 0; m * L < kCombWindows; m++) {
    const uint32_t win = l + (uint32_t)(m * L);
    const int d = (int)(sv[0] & (2u * kCombEntries - 1u)) - kCombEntries;
    shr_const<kGW * L>(sv);
    if (win < (uint32_t)kCombWindows) {
      const uint32_t mag = (uint32_t)(d < 0 ? -d : d);
      const uint32_t* te = gtab + ((size_t)win * kCombEntries + (mag ? mag - 1 : 0)) * kGEntry;
      uint32_t tx[9], ty[9];
#pragma unroll
      for (int q = 0; q < 9; q++) {
        tx[q] = te[q];
        ty[q] = te[9 + q];
      }
      if (d < 0) f_neg<P, 64>(ty, ty);
      j_acc_aff<P>(C, c_inf, tx, ty, one, mag == 0);
    }
  }
}

// One lane's half of the 2-lane secp256k1 ladder (small, latency-bound
// batches): lane `part` computes k1 Q (part 0) or k2 phi(Q) (part 1) and every
// other G-comb window; the caller adds the two halves and runs finish_check.
template <class P>
BH_HD void ladder2_part(J30& C, bool& c_inf, const Work& w, const uint32_t* gtab, uint32_t i,
                        uint32_t wave, uint32_t lane, uint32_t part) {
  q_ladder_glv<P>(C, c_inf, w, i, wave, lane, 1u << part);
  uint32_t u1[8];
  ld8(u1, w.e, i, w.ns);
  g_comb_part<P, 2>(C, c_inf, gtab, u1, part);
}

// Partial-sum scratch for the split wide kernels (BDLS batches: the u2 Q
// halves run while the digests are hashed, the u1 G halves after): slot g of
// a lane, SoA with stride `stride` (>= lanes), 28 words (X, Y, Z, infinity).
BH_HD void part_store(const Work& w, uint32_t g, uint32_t stride, const J30& C, bool c_inf) {
  uint32_t* o = w.gpart + g;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    o[(size_t)k * stride] = C.X[k];
    o[(size_t)(9 + k) * stride] = C.Y[k];
    o[(size_t)(18 + k) * stride] = C.Z[k];
  }
  o[(size_t)27 * stride] = c_inf ? 1u : 0u;
}

BH_HD void part_load(const Work& w, uint32_t g, uint32_t stride, J30& C, bool& c_inf) {
  const uint32_t* o = w.gpart + g;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    C.X[k] = o[(size_t)k * stride];
    C.Y[k] = o[(size_t)(9 + k) * stride];
    C.Z[k] = o[(size_t)(18 + k) * stride];
  }
  c_inf = o[(size_t)27 * stride] != 0;
}

}  // namespace bh
