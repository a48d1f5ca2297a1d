// TEST-ONLY host harness: runs the exact per-record stage functions of
// bdls_amd/csrc/verify.h (the code the HIP kernels execute) sequentially on the
// CPU, so the arithmetic can be checked against the oracle in a container with
// no GPU. Never linked into libbdlship.so; the product path has no CPU fallback.
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../bdls_amd/csrc/verify.h"
#include "../../bdls_amd/csrc/shard.h"
#include "../../bdls_amd/csrc/pack.h"

using namespace bh;

static std::vector<uint32_t> g_gtab, g_gtab_k1;

template <class P>
static const uint32_t* gtab_for() {
  std::vector<uint32_t>& g = P::sparse_p256 ? g_gtab : g_gtab_k1;
  if (g.empty()) {  // the device buffer's layout: 13-bit comb, then the folded tables
    g.assign(kGTabAllWords, 0);
    for (uint32_t t = 0; t < (uint32_t)(kCombWindows * kCombEntries); t++)
      gtab_entry<P>(t, g.data() + (size_t)t * kGEntry);
    for (uint32_t k = 0; k < kGBase; k++) gtab2_base<P>(k, g.data() + kGCombWords);
    for (uint32_t t = 0; t < kG2Ent + kG1Ent; t++) gtab2_entry<P>(t, g.data() + kGCombWords);
  }
  return g.data();
}

// Lanes per record on the key-table path (verify_kernels.hip k_keycomb_wide);
// 1 = k_keycomb.
static int g_wide = 1;
extern "C" void hs_set_wide(int L) { g_wide = L; }
// 1: per-batch tables of the one-lane comb (g_wide == 1) are Lim-Lee combs
// (verify.h lltab_build / q_llcomb), as the device builds them for large
// batches; 0: the 4-bit windowed tables.
static int g_ll = 0;
extern "C" void hs_set_ll(int on) { g_ll = on; }
// 1: every key table is built as a registry slot (verify.h reg_build: the comb +
// affine 4-bit windows) and read as one: the one-lane route walks the comb with
// u1 G folded in, the multi-lane route the affine windows (mixed additions)
static int g_reg = 0;
extern "C" void hs_set_reg(int on) { g_reg = on; }
// the comb's shape as built (teeth << 8 | spacing), for the crafted-scalar tests
extern "C" uint32_t hs_ll_shape() { return ((uint32_t)kLLTeeth << 8) | (uint32_t)kLLSpace; }
// u1 columns per folded G entry as built (BH_GFOLD)
extern "C" uint32_t hs_gfold() { return (uint32_t)kGF; }
// the G comb's window width as built (BH_GCOMB_BITS)
extern "C" uint32_t hs_gcomb_bits() { return (uint32_t)kGW; }

template <class P, int L>
static bool wide_keycomb(const Work& w, const uint32_t* gtab, uint32_t i, const uint32_t* tab) {
  J30 C[L];
  bool inf[L];
  for (int l = 0; l < L; l++)
    keycomb_part<P, L>(C[l], inf[l], w, gtab, i, tab, (uint32_t)l, g_reg != 0);
  for (int off = 1; off < L; off <<= 1) {  // the kernel's __shfl_xor butterfly
    J30 D[L];
    bool dinf[L];
    for (int l = 0; l < L; l++) {
      j_copy(D[l], C[l]);
      dinf[l] = inf[l];
      j_acc<P>(D[l], dinf[l], C[l ^ off], inf[l ^ off]);
    }
    for (int l = 0; l < L; l++) {
      j_copy(C[l], D[l]);
      inf[l] = dinf[l];
    }
  }
  return finish_check<P>(w, i, C[0], inf[0], C[0], true);
}

template <class P>
static bool keycomb_any(const Work& w, const uint32_t* gtab, uint32_t i, const uint32_t* tab) {
  switch (g_wide) {
    case 2: return wide_keycomb<P, 2>(w, gtab, i, tab);
    case 4: return wide_keycomb<P, 4>(w, gtab, i, tab);
    case 8: return wide_keycomb<P, 8>(w, gtab, i, tab);
    case 16: return wide_keycomb<P, 16>(w, gtab, i, tab);
    case 32: return wide_keycomb<P, 32>(w, gtab, i, tab);  // k_small's group
    case 0: return stage_keycomb<P>(w, gtab, i, tab, g_reg != 0);
    default:
      if (!g_ll && !g_reg) {  // windowed tables: u1 G stored by list position, then the table half
        stage_gpart<P>(w, gtab, i, i);
        return stage_keycomb_q<P>(w, i, i, tab, false);
      }
      // comb tables: u1 G folded into the Horner (k_keycomb). Its three ways
      // to read a comb table, taken in turn: 16-byte loads of the per-batch
      // table (stride 0), the workgroup's packed LDS copy (kLLLds words per
      // entry), and the per-batch table through the same 8-byte loads (a run
      // past the LDS slots)
      switch (i % 3) {
        case 0: return stage_keycomb_fold<P>(w, i, tab, 0, g2_of(gtab));
        case 1: {
          std::vector<uint32_t> lds((size_t)kLLEnt * kLLLds);
          for (uint32_t e = 0; e < kLLEnt; e++)
            for (uint32_t k = 0; k < kLLLds; k++) lds[e * kLLLds + k] = tab[e * kLLAff + k];
          return stage_keycomb_fold<P>(w, i, lds.data(), kLLLds, g2_of(gtab));
        }
        default: return stage_keycomb_fold<P>(w, i, tab, kLLAff, g2_of(gtab));
      }
  }
}

// Sequential restatement of the device launch sequence (verify_kernels.hip
// seq()): prep, inv, key dedup / plan / split, key tables, both verify paths.
// min_uses overrides kMinUses (and the batch-size gate) so tests can force
// either path.
template <class P, class N, class C, class IN>
static int run_seq(const IN& in, uint32_t n, uint32_t chunk, uint32_t min_uses, uint8_t* reason,
                   uint32_t* n_comb) {
  const uint32_t* gtab = gtab_for<P>();
  const uint32_t ns = (n + 63) & ~63u;
  std::vector<uint32_t> buf((size_t)9 * 9 * ns + (size_t)2 * ns * kQTab * kQPt +
                            (size_t)kGPartWords * ns);
  std::vector<uint8_t> st(ns);
  Work w;
  w.ns = ns;
  uint32_t* p = buf.data();
  w.e = p; p += 8 * ns;
  w.r = p; p += 8 * ns;
  w.sm = p; p += 8 * ns;
  w.pre = p; p += 8 * ns;
  w.qx = p; p += 9 * ns;
  w.qy = p; p += 9 * ns;
  w.rm = p; p += 9 * ns;
  w.r2m = p; p += 9 * ns;
  p += 9 * ns;
  w.qtab = p;
  p += (size_t)2 * ns * kQTab * kQPt;
  w.gpart = p;
  w.st = st.data();
  for (uint32_t i = 0; i < n; i++) {
    if constexpr (std::is_same_v<IN, BatchIn>) {
      if (in.flags & BHF_HASH_SHA3_256) stage_prep<P, N, C, HK_SHA3_256>(in, w, i);
      else stage_prep<P, N, C>(in, w, i);
    } else {
      stage_bdls_hash<C>(in, w, i);
      stage_prep<P, N, C>(in, w, i);
    }
  }
  const uint32_t lanes = (n + chunk - 1) / chunk;
  for (uint32_t c = 0; c < lanes; c++) stage_inv<N>(w, c, lanes, n);
  // dedup: representative = first record with an equal key
  std::vector<uint32_t> rep(n, kNone), cnt(n, 0);
  std::unordered_map<uint64_t, std::vector<uint32_t>> by_hash;
  for (uint32_t i = 0; i < n; i++) {
    if ((w.st[i] & 0x7f) != R_OK) continue;
    auto& v = by_hash[key_hash(w, i)];
    uint32_t r = kNone;
    if (!v.empty() && same_key(w, i, v[0])) r = v[0];
    if (v.empty()) {
      v.push_back(i);
      r = i;
    }
    rep[i] = r;
    if (r != kNone) cnt[r]++;
  }
  std::vector<uint32_t> tab_of(n, kNone);
  std::vector<std::vector<uint32_t>> tables;
  uint32_t combs = 0;
  for (uint32_t i = 0; i < n; i++) {
    if ((w.st[i] & 0x7f) != R_OK) {
      reason[i] = w.st[i] & 0x7f;
      continue;
    }
    const uint32_t r = rep[i];
    bool ok;
    if (r != kNone && cnt[r] >= min_uses) {
      if (tab_of[r] == kNone) {
        tab_of[r] = (uint32_t)tables.size();
        tables.emplace_back(kKTabWords);
        if (g_reg) {  // a registry slot: the comb + affine windows
          reg_build<P>(tables.back().data(), w, r);
        } else if (g_ll && g_wide == 1) {  // comb: the device's two build lanes, one after the other
          lltab_build<P>(tables.back().data(), w, r);
        } else {
          ktab_build<P>(tables.back().data(), w, r);  // the device's co-Z chain
        }
      }
      ok = keycomb_any<P>(w, gtab, i, tables[tab_of[r]].data());
      combs++;
    } else if (!P::a_is_minus3 && g_wide > 1) {
      // the 2-lane secp256k1 ladder (verify_kernels.hip k_ladder2_q / _g): the two
      // GLV halves in two Q-table slots, added as the kernel's lane 0 does
      J30 C0, C1;
      bool i0, i1;
      ladder2_part<P>(C0, i0, w, gtab, i, (2 * i) / 64, (2 * i) % 64, 0);
      ladder2_part<P>(C1, i1, w, gtab, i, (2 * i + 1) / 64, (2 * i + 1) % 64, 1);
      j_acc<P>(C0, i0, C1, i1);
      ok = finish_check<P>(w, i, C0, i0, C0, true);
    } else {
      ok = stage_ladder_fold<P>(w, gtab, i, i / 64, i % 64);
    }
    reason[i] = ok ? R_OK : R_MATH;
  }
  if (n_comb) *n_comb = combs;
  return 0;
}

extern "C" int hs_verify2(const uint8_t* pub, const uint8_t* sig, const uint64_t* soff,
                          const uint32_t* slen, const uint8_t* msg, const uint64_t* moff,
                          const uint32_t* mlen, uint32_t n, uint32_t flags, uint32_t chunk,
                          uint32_t min_uses, uint8_t* reason, uint32_t* n_comb) {
  BatchIn in{pub, sig, soff, slen, msg, moff, mlen, flags};
  return run_seq<F30_p256, Fn_p256, Cv_p256>(in, n, chunk, min_uses, reason, n_comb);
}

// secp256k1 with the Fabric record layout but BHF_NO_LOW_S and a caller-chosen
// digest: reaches the curve-level edge cases (x wrap, infinity, u1 G == u2 Q)
// that BLAKE2b-hashed BDLS messages cannot be steered into.
// bh_verify_2seg's two-span messages: msg[moff, +mlen) || msg[m2off, +m2len)
extern "C" int hs_verify_2seg(const uint8_t* pub, const uint8_t* sig, const uint64_t* soff,
                              const uint32_t* slen, const uint8_t* msg, const uint64_t* moff,
                              const uint32_t* mlen, const uint64_t* m2off, const uint32_t* m2len,
                              uint32_t n, uint32_t flags, uint8_t* reason) {
  BatchIn in{pub, sig, soff, slen, msg, moff, mlen, flags};
  in.msg2_off = m2off;
  in.msg2_len = m2len;
  return run_seq<F30_p256, Fn_p256, Cv_p256>(in, n, 4, kMinUses, reason, nullptr);
}

extern "C" int hs_verify_k1_digest(const uint8_t* pub, const uint8_t* sig, const uint64_t* soff,
                                   const uint32_t* slen, const uint8_t* dg, const uint64_t* doff,
                                   const uint32_t* dlen, uint32_t n, uint32_t min_uses,
                                   uint8_t* reason) {
  BatchIn in{pub, sig, soff, slen, dg, doff, dlen, BHF_NO_LOW_S};
  return run_seq<F30_k1, Fn_k1, Cv_k1>(in, n, 4, min_uses, reason, nullptr);
}

extern "C" int hs_verify_bdls(int curve, const uint8_t* xy, const uint8_t* r, const uint64_t* roff,
                              const uint32_t* rlen, const uint8_t* s, const uint64_t* soff,
                              const uint32_t* slen, const uint32_t* ver, const uint8_t* msg,
                              const uint64_t* moff, const uint32_t* mlen, uint32_t n,
                              uint32_t min_uses, uint8_t* reason) {
  BdlsIn in{xy, r, roff, rlen, s, soff, slen, ver, msg, moff, mlen, 0};
  if (curve == 0) return run_seq<F30_p256, Fn_p256, Cv_p256>(in, n, 4, min_uses, reason, nullptr);
  return run_seq<F30_k1, Fn_k1, Cv_k1>(in, n, 4, min_uses, reason, nullptr);
}

extern "C" int hs_verify(const uint8_t* pub, const uint8_t* sig, const uint64_t* soff,
                         const uint32_t* slen, const uint8_t* msg, const uint64_t* moff,
                         const uint32_t* mlen, uint32_t n, uint32_t flags, uint32_t chunk,
                         uint8_t* reason) {
  return hs_verify2(pub, sig, soff, slen, msg, moff, mlen, n, flags, chunk, kMinUses, reason,
                    nullptr);
}

// ---- field-op probes for tests/test_field30.py (bound stress) ----
extern "C" void hs_f_mul(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  f_mul<F30_p256>(r, a, b);
}
extern "C" void hs_f_sub32(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  f_sub<F30_p256, 32>(r, a, b);
}
extern "C" void hs_f_sub64(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  f_sub<F30_p256, 64>(r, a, b);
}
extern "C" void hs_f_add(const uint32_t* a, const uint32_t* b, uint32_t* r) { f_add(r, a, b); }
extern "C" void hs_f_reduce(const uint32_t* a, uint32_t* r) { f_reduce<F30_p256>(r, a); }
extern "C" void hs_f_sqr(const uint32_t* a, uint32_t* r) { f_sqr<F30_p256>(r, a); }
// round 6's fused passes, both curves (curve 0 = P-256, 1 = secp256k1), K = 32 / 64
template <class F, int K>
static void fused(int op, const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t* r) {
  switch (op) {
    case 0: f_add2x(r, a, b); break;
    case 1: f_addsub<F, K>(r, a, b, c); break;
    case 2: f_sub2<F, K>(r, a, b, c); break;
    case 3: f_csub<F, K>(r, false, a, b); break;
    case 4: f_csub<F, K>(r, true, a, b); break;
  }
}
extern "C" void hs_f_fused(int curve, int K, int op, const uint32_t* a, const uint32_t* b,
                           const uint32_t* c, uint32_t* r) {
  if (K == 96) {  // the mixed addition's sign pass (f_csub only)
    if (op == 3 || op == 4) {
      if (curve == 0) f_csub<F30_p256, 96>(r, op == 4, a, b);
      else f_csub<F30_k1, 96>(r, op == 4, a, b);
    }
    return;
  }
  if (curve == 0) (K == 32 ? fused<F30_p256, 32> : fused<F30_p256, 64>)(op, a, b, c, r);
  else (K == 32 ? fused<F30_k1, 32> : fused<F30_k1, 64>)(op, a, b, c, r);
}
extern "C" void hs_bdls_hash(uint32_t version, const uint8_t* x32, const uint8_t* y32,
                             const uint8_t* msg, uint32_t mlen, uint8_t* out) {
  bdls_signed_proto_hash(out, version, x32, y32, msg, mlen);
}

// ---- scalar-field inversion probes (tests/test_field30.py) ----
extern "C" void hs_n_inv(int curve, const uint32_t* a, uint32_t* r) {
  if (curve == 0) mod_inv_sg<Fn_p256>(r, a);
  else mod_inv_sg<Fn_k1>(r, a);
}
extern "C" void hs_n_inv_var(int curve, const uint32_t* a, uint32_t* r) {
  if (curve == 0) mod_inv_sg<Fn_p256, true>(r, a);
  else mod_inv_sg<Fn_k1, true>(r, a);
}
extern "C" void hs_n_mont_inv(int curve, const uint32_t* a, uint32_t* r) {
  if (curve == 0) mont_inv_sg<Fn_p256>(r, a);
  else mont_inv_sg<Fn_k1>(r, a);
}
extern "C" void hs_sha256(const uint8_t* msg, uint32_t len, uint32_t* out) {
  sha256_msg(out, msg, len);
}
// k_digest_grp's split compression (sha256.h): every block loaded with
// sha256_load_block, expanded by sha256_sched_wk, compressed by
// sha256_rounds_wk; two spans m1 || m2 (l2 = 0: one span).
extern "C" void hs_sha256_split(const uint8_t* m1, uint32_t l1, const uint8_t* m2, uint32_t l2,
                                uint32_t* out) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t len = (uint64_t)l1 + l2, total = ((len + 9 + 63) / 64) * 64;
  for (uint64_t blk = 0; blk < total; blk += 64) {
    uint32_t w[16], wk[64];
    sha256_load_block(w, m1, l2 ? l1 : len, l2 ? m2 : m1, len, total, blk);
    sha256_sched_wk(wk, w);
    sha256_rounds_wk(h, wk);
  }
  for (int i = 0; i < 8; i++) out[i] = h[i];
}
extern "C" void hs_sha3_256(const uint8_t* msg, uint32_t len, uint8_t* out) {
  sha3_256_msg(out, msg, len);
}

// bh_verify's multi-device split (bdls_amd/csrc/shard.h, used by bdls_hip.cpp
// submit_job / finish_part) for n records over ndev devices: returns 0 when
// the shards are contiguous, 64-aligned, non-empty, cover [0, n) and their
// bitmaps merge into exactly the single-device bitmap of `valid` (n bytes,
// 0/1); otherwise a code naming the first broken property.
extern "C" int hs_shard_check(size_t n, size_t ndev, const uint8_t* valid, size_t* nshards) {
  const size_t nd = bh::shard_devices(n, ndev);
  std::vector<uint8_t> want((n + 7) / 8 + 1, 0), got((n + 7) / 8 + 1, 0);
  for (size_t i = 0; i < n; i++)
    if (valid[i]) want[i >> 3] |= (uint8_t)(1u << (i & 7));
  size_t next = 0, used = 0;
  for (size_t k = 0; k < nd; k++) {
    const bh::Shard s = bh::shard_of(n, nd, k);
    if (!s.len) break;
    if (s.lo != next) return 1;           // not contiguous
    if (s.lo % 64) return 2;              // bitmap offset not byte / word aligned
    if (k + 1 < nd && bh::shard_of(n, nd, k + 1).len && s.len % 64) return 3;  // ragged before the end
    // the device's result words for this shard: bit i = record lo + i
    std::vector<uint64_t> words((s.len + 63) / 64, 0);
    for (size_t i = 0; i < s.len; i++)
      if (valid[s.lo + i]) words[i >> 6] |= 1ull << (i & 63);
    bh::shard_bitmap_merge(got.data(), s, words.data());
    next = s.lo + s.len;
    used++;
  }
  if (next != n) return 4;                // records left out
  if (n && used != nd) return 5;          // a device got no work
  if (memcmp(want.data(), got.data(), want.size())) return 6;  // merged bitmap differs
  *nshards = used;
  return 0;
}

// ---- staged BatchVerify packing (bdls_amd/csrc/pack.h) ------------------------
// Packs records [lo, lo + m) of a SoA batch exactly as bdls_hip.cpp
// enqueue_staged does (plan, then fill with the per-chunk callback).
// force: -1 the sample decides, 0 / 1 de-duplication off / on. info[0..7] =
// nkeys, dedup, fixed_msg, msg_stride, sig_bytes, msg_bytes, nchunks, rebuilds,
// [8..9] plan / fill microseconds;
// bounds: the chunk byte bounds (sig then msg, nchunks + 1 each) in the order
// the callback saw them complete. Returns -1 when a chunk was reported before
// its bytes were all written or out of order.
struct HsSrc {
  const uint8_t *pub, *sig, *msg;
  const uint64_t *sig_off, *msg_off;
  const uint32_t *sig_len, *msg_len;
  const uint8_t* key(size_t i) const { return pub + i * 64; }
  const uint8_t* sig_(size_t i) const { return sig + sig_off[i]; }
};
struct HsSrcA {
  const HsSrc* s;
  const uint8_t* key(size_t i) const { return s->key(i); }
  const uint8_t* sig(size_t i) const { return s->sig_(i); }
  uint32_t sig_len(size_t i) const { return s->sig_len[i]; }
  const uint8_t* msg(size_t i) const { return s->msg + s->msg_off[i]; }
  uint32_t msg_len(size_t i) const { return s->msg_len[i]; }
};
extern "C" int hs_pack(const uint8_t* pub, const uint8_t* sig, const uint64_t* sig_off,
                       const uint32_t* sig_len, const uint8_t* msg, const uint64_t* msg_off,
                       const uint32_t* msg_len, size_t lo, size_t m, int threads, int force,
                       uint8_t* keys, uint32_t* key_idx, uint32_t* slen, uint32_t* mlen,
                       uint8_t* sig_out, uint8_t* msg_out, uint64_t* info, uint64_t* bounds) {
  static bh::pack::Packer* P[65] = {nullptr};
  threads = std::max(1, std::min(64, threads));
  if (!P[threads]) P[threads] = new bh::pack::Packer(threads);
  HsSrc src{pub, sig, msg, sig_off, msg_off, sig_len, msg_len};
  HsSrcA a{&src};
  bh::pack::Out out{keys, key_idx, slen, mlen};
  bh::pack::Result r;
  P[threads]->plan(a, lo, m, &r, force);
  int next = 0, bad = 0;
  static const bool nocheck = getenv("HS_PACK_NOCHECK") != nullptr;  // tools/pack_bench.py
  P[threads]->fill(a, out, sig_out, msg_out, &r, [&](int c) {
    if (c != next++) bad = 1;
    if (nocheck) return;
    // every record of chunk c is in place when its callback runs
    const size_t K = (size_t)r.nchunks, ca = (m * c) / K, cb = (m * (c + 1)) / K;
    uint64_t so = r.sig_chunk[c], mo = r.msg_chunk[c];
    for (size_t i = ca; i < cb; i++) {
      if (sig_len[lo + i] && memcmp(sig_out + so, sig + sig_off[lo + i], sig_len[lo + i])) bad = 1;
      if (msg_len[lo + i] && memcmp(msg_out + mo, msg + msg_off[lo + i], msg_len[lo + i])) bad = 1;
      so += sig_len[lo + i];
      mo += msg_len[lo + i];
    }
    if (so != r.sig_chunk[c + 1] || mo != r.msg_chunk[c + 1]) bad = 1;
  });
  const uint64_t v[10] = {r.nkeys, (uint64_t)r.dedup, (uint64_t)r.fixed_msg, r.msg_stride,
                          r.sig_bytes, r.msg_bytes, (uint64_t)r.nchunks, (uint64_t)r.rebuilds,
                          (uint64_t)(r.plan_ms * 1e3), (uint64_t)(r.fill_ms * 1e3)};
  memcpy(info, v, sizeof(v));
  for (int c = 0; c <= r.nchunks; c++) {
    bounds[c] = r.sig_chunk[c];
    bounds[r.nchunks + 1 + c] = r.msg_chunk[c];
  }
  return bad ? -1 : 0;
}

extern "C" double hs_estimate_distinct(size_t s, size_t ds) {
  return bh::pack::estimate_distinct(s, ds);
}
