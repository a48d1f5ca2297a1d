/*
 * Synthetic workload generator for bench.py and the large parity tests.
 * Produces BASELINE.json configs as verify records:
 *   config 2: n records, `nkeys` distinct P-256 keys, `msg_len`-byte random
 *             messages (fused SHA-256), 1/`corrupt_den` of the records
 *             corrupted over the eleven classes below, seeded.
 *   config 5: nkeys >= n: record i signs with key i (one distinct key per
 *             record, no reuse anywhere in the batch).
 * Signing follows bccsp/sw/ecdsa.go:27-39 (signECDSA: ecdsa.Sign, ToLowS, DER)
 * with a seeded nonce so every batch is reproducible. OpenSSL libcrypto
 * provides k*G / d*G on the host; this is data preparation, outside every
 * timed region, and is not the oracle (that is oracle/orc.c).
 * The expected reason per record follows by construction from the corruption
 * class; tests/ confirm it against oracle/orc.c on samples.
 */
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/obj_mac.h>
#include <openssl/evp.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { C_NONE = 0, C_MSG_FLIP, C_HIGH_S, C_R_ZERO, C_R_GE_N, C_S_GE_N, C_Q_OFFCURVE, C_Q_GE_P,
       C_DER_TRAILING, C_DER_EXTRA, C_DER_NONMIN, C_DER_LONGLEN, C_NUM };
/* expected reason per class (include/bdls_hip.h BH_R_*) */
static const uint8_t kExpect[C_NUM] = {0, 9, 6, 4, 8, 6, 7, 7, 0, 0, 3, 3};

#define SIG_STRIDE 80 /* bytes reserved per record in the sig buffer */

static uint64_t splitmix(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static void rand_bytes(uint64_t *s, uint8_t *out, size_t n) {
  for (size_t i = 0; i < n; i += 8) {
    uint64_t v = splitmix(s);
    for (size_t k = 0; k < 8 && i + k < n; k++) out[i + k] = (uint8_t)(v >> (8 * k));
  }
}

/* scalar in [1, n-1] from the stream */
static void rand_scalar(uint64_t *s, BIGNUM *out, const BIGNUM *n, BN_CTX *ctx) {
  uint8_t b[40];
  do {
    rand_bytes(s, b, 40);
    BN_bin2bn(b, 40, out);
    BN_nnmod(out, out, n, ctx);
  } while (BN_is_zero(out));
}

/* DER INTEGER from a non-negative BIGNUM (minimal) */
static size_t der_int(uint8_t *o, const BIGNUM *v, int nonmin, int longlen) {
  uint8_t mag[40];
  int L = BN_bn2bin(v, mag);
  size_t k = 0;
  int pad = (L == 0) || (mag[0] & 0x80);
  size_t clen = (size_t)L + (pad ? 1 : 0) + (nonmin ? 1 : 0);
  if (L == 0) clen = 1 + (nonmin ? 1 : 0);
  o[k++] = 0x02;
  if (longlen) {
    o[k++] = 0x81;
  }
  o[k++] = (uint8_t)clen;
  if (nonmin) o[k++] = 0x00;
  if (L == 0) {
    o[k++] = 0x00;
    return k;
  }
  if (pad) o[k++] = 0x00;
  memcpy(o + k, mag, L);
  return k + L;
}

typedef struct {
  size_t lo, hi, n; /* global record range [lo, hi) of a batch of n records */
  size_t base;      /* global index of output slot 0 (shard start) */
  uint64_t seed;
  int nkeys, msg_len, corrupt_den;
  const uint8_t *keypub; /* nkeys * 64 */
  const uint8_t *keypriv; /* nkeys * 32 */
  uint8_t *pub, *msg, *sig, *reason, *cls;
  uint64_t *moff, *soff;
  uint32_t *mlen, *slen;
  int family; /* 0 SHA2 (SHA-256), 1 SHA3 (SHA3-256): msp/identities.go:219-227 */
} gjob;

static void *gen_worker(void *arg) {
  gjob *j = (gjob *)arg;
  EC_GROUP *g = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
  BN_CTX *ctx = BN_CTX_new();
  BIGNUM *n = BN_new(), *p = BN_new(), *half = BN_new(), *k = BN_new(), *kinv = BN_new(),
         *r = BN_new(), *s = BN_new(), *e = BN_new(), *d = BN_new(), *t = BN_new(),
         *x = BN_new();
  EC_GROUP_get_order(g, n, ctx);
  EC_GROUP_get_curve(g, p, NULL, NULL, ctx);
  BN_rshift1(half, n);
  EC_POINT *R = EC_POINT_new(g), *Q = EC_POINT_new(g);
  const int unique = (size_t)j->nkeys >= j->n;  /* record i signs with key i */
  uint8_t dg[32], b32[32], upub[64], upriv[32];
  for (size_t gi = j->lo; gi < j->hi; gi++) {
    const size_t i = gi - j->base; /* output slot */
    uint64_t st = j->seed * 0x100000001b3ull + gi * 0x9e3779b97f4a7c15ull + 17;
    splitmix(&st);
    const uint64_t kr = splitmix(&st);
    const uint8_t *kpub, *kpriv;
    if (unique) {
      /* key gi, derived exactly as key_worker would (no n-sized key table) */
      uint64_t ks = j->seed * 0xff51afd7ed558ccdull + (uint64_t)gi * 0xc4ceb9fe1a85ec53ull + 99;
      rand_scalar(&ks, d, n, ctx);
      EC_POINT_mul(g, Q, d, NULL, NULL, ctx);
      EC_POINT_get_affine_coordinates(g, Q, x, t, ctx);
      BN_bn2binpad(d, upriv, 32);
      BN_bn2binpad(x, upub, 32);
      BN_bn2binpad(t, upub + 32, 32);
      kpub = upub;
      kpriv = upriv;
    } else {
      const size_t key = (size_t)(kr % (uint64_t)j->nkeys);
      kpub = j->keypub + 64 * key;
      kpriv = j->keypriv + 32 * key;
    }
    int cls = C_NONE;
    if (j->corrupt_den > 0 && splitmix(&st) % (uint64_t)j->corrupt_den == 0)
      cls = 1 + (int)(splitmix(&st) % (C_NUM - 1));
    uint8_t *m = j->msg + (size_t)i * j->msg_len;
    rand_bytes(&st, m, j->msg_len);
    j->moff[i] = (uint64_t)i * j->msg_len;
    j->mlen[i] = (uint32_t)j->msg_len;
    if (j->family == 1) EVP_Digest(m, j->msg_len, dg, NULL, EVP_sha3_256(), NULL);
    else SHA256(m, j->msg_len, dg);
    /* sign: r = x(kG) mod n, s = k^-1 (e + r d) mod n, low-S */
    BN_bin2bn(kpriv, 32, d);
    BN_bin2bn(dg, 32, e);
    BN_nnmod(e, e, n, ctx);
    do {
      rand_scalar(&st, k, n, ctx);
      EC_POINT_mul(g, R, k, NULL, NULL, ctx);
      EC_POINT_get_affine_coordinates(g, R, x, NULL, ctx);
      BN_nnmod(r, x, n, ctx);
      BN_mod_inverse(kinv, k, n, ctx);
      BN_mod_mul(t, r, d, n, ctx);
      BN_mod_add(t, t, e, n, ctx);
      BN_mod_mul(s, kinv, t, n, ctx);
    } while (BN_is_zero(r) || BN_is_zero(s));
    if (BN_cmp(s, half) > 0) BN_sub(s, n, s);
    uint8_t *q = j->pub + (size_t)i * 64;
    memcpy(q, kpub, 64);
    /* corruptions */
    switch (cls) {
      case C_MSG_FLIP: m[splitmix(&st) % j->msg_len] ^= (uint8_t)(1u << (splitmix(&st) % 8)); break;
      case C_HIGH_S: BN_sub(s, n, s); break;
      case C_R_ZERO: BN_zero(r); break;
      case C_R_GE_N: BN_add(r, r, n); if (BN_num_bits(r) > 256) BN_copy(r, n); break;
      case C_S_GE_N: BN_add(s, s, n); if (BN_num_bits(s) > 256) BN_copy(s, n); break;
      case C_Q_OFFCURVE: q[63] ^= 1; break;
      case C_Q_GE_P: {
        BN_bin2bn(q, 32, t);
        BN_add(t, t, p);
        if (BN_num_bits(t) > 256) BN_copy(t, p);
        BN_bn2binpad(t, b32, 32);
        memcpy(q, b32, 32);
        break;
      }
      default: break;
    }
    /* DER */
    uint8_t body[SIG_STRIDE], *o = j->sig + (size_t)i * SIG_STRIDE;
    size_t bl = der_int(body, r, cls == C_DER_NONMIN, cls == C_DER_LONGLEN);
    bl += der_int(body + bl, s, 0, 0);
    if (cls == C_DER_EXTRA) {
      body[bl++] = 0x02; body[bl++] = 0x01; body[bl++] = 0x07;
    }
    size_t L = 0;
    o[L++] = 0x30;
    o[L++] = (uint8_t)bl;
    memcpy(o + L, body, bl);
    L += bl;
    if (cls == C_DER_TRAILING) {
      o[L++] = 0xde; o[L++] = 0xad;
    }
    j->soff[i] = (uint64_t)i * SIG_STRIDE;
    j->slen[i] = (uint32_t)L;
    j->reason[i] = kExpect[cls];
    j->cls[i] = (uint8_t)cls;
  }
  EC_POINT_free(R);
  EC_POINT_free(Q);
  BIGNUM *v[] = {n, p, half, k, kinv, r, s, e, d, t, x};
  for (size_t q = 0; q < sizeof(v) / sizeof(v[0]); q++) BN_free(v[q]);
  BN_CTX_free(ctx);
  EC_GROUP_free(g);
  return NULL;
}

typedef struct {
  int lo, hi;
  uint64_t seed;
  uint8_t *pub, *priv;
} kjob;

static void *key_worker(void *arg) {
  kjob *j = (kjob *)arg;
  EC_GROUP *g = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
  BN_CTX *ctx = BN_CTX_new();
  BIGNUM *n = BN_new(), *d = BN_new(), *x = BN_new(), *y = BN_new();
  EC_GROUP_get_order(g, n, ctx);
  EC_POINT *Q = EC_POINT_new(g);
  for (int i = j->lo; i < j->hi; i++) {
    uint64_t st = j->seed * 0xff51afd7ed558ccdull + (uint64_t)i * 0xc4ceb9fe1a85ec53ull + 99;
    rand_scalar(&st, d, n, ctx);
    EC_POINT_mul(g, Q, d, NULL, NULL, ctx);
    EC_POINT_get_affine_coordinates(g, Q, x, y, ctx);
    BN_bn2binpad(d, j->priv + 32 * (size_t)i, 32);
    BN_bn2binpad(x, j->pub + 64 * (size_t)i, 32);
    BN_bn2binpad(y, j->pub + 64 * (size_t)i + 32, 32);
  }
  EC_POINT_free(Q);
  BN_free(n); BN_free(d); BN_free(x); BN_free(y);
  BN_CTX_free(ctx);
  EC_GROUP_free(g);
  return NULL;
}

/* Records [lo, lo + count) of one seeded batch of n_total records (a shard:
 * the union over shards is the same batch for any split). Caller allocates
 * for `count` records: pub *64, msg *msg_len, sig *80, moff/soff u64,
 * mlen/slen u32, reason/cls u8; offsets are shard-local. nkeys >= n_total:
 * one distinct key per record (config 5), derived per record. */
int gen_p256_shard(size_t n_total, size_t lo, size_t count, size_t nkeys, int msg_len,
                   int corrupt_den, uint64_t seed, int nthreads, int family, uint8_t *pub,
                   uint8_t *msg, uint64_t *moff, uint32_t *mlen, uint8_t *sig, uint64_t *soff,
                   uint32_t *slen, uint8_t *reason, uint8_t *cls) {
  if (family != 0 && family != 1) return -3;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 128) nthreads = 128;
  if (nkeys < 1 || msg_len < 1 || lo + count > n_total) return -1;
  const int unique = nkeys >= n_total;
  uint8_t *kpub = NULL, *kpriv = NULL;
  pthread_t th[128];
  int used = 0;
  if (!unique) {
    if (nkeys > (1u << 30)) return -1;
    kpub = malloc(nkeys * 64);
    kpriv = malloc(nkeys * 32);
    if (!kpub || !kpriv) return -2;
    kjob kj[128];
    int nk = (int)nkeys, per = (nk + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
      int a = t * per, b = a + per > nk ? nk : a + per;
      if (a >= b) break;
      kj[t] = (kjob){a, b, seed, kpub, kpriv};
      pthread_create(&th[t], NULL, key_worker, &kj[t]);
      used++;
    }
    for (int t = 0; t < used; t++) pthread_join(th[t], NULL);
  }
  gjob gj[128];
  size_t gper = (count + nthreads - 1) / nthreads;
  used = 0;
  for (int t = 0; t < nthreads; t++) {
    size_t a = lo + t * gper, b = a + gper > lo + count ? lo + count : a + gper;
    if (a >= b) break;
    gj[t] = (gjob){a, b, n_total, lo, seed, (int)(nkeys > 0x7fffffff ? 0x7fffffff : nkeys),
                   msg_len, corrupt_den, kpub, kpriv, pub, msg, sig, reason, cls, moff, soff,
                   mlen, slen, family};
    pthread_create(&th[t], NULL, gen_worker, &gj[t]);
    used++;
  }
  for (int t = 0; t < used; t++) pthread_join(th[t], NULL);
  free(kpub);
  free(kpriv);
  return 0;
}

int gen_p256_family(size_t n, int nkeys, int msg_len, int corrupt_den, uint64_t seed,
                    int nthreads, int family, uint8_t *pub, uint8_t *msg, uint64_t *moff,
                    uint32_t *mlen, uint8_t *sig, uint64_t *soff, uint32_t *slen,
                    uint8_t *reason, uint8_t *cls) {
  if (nkeys < 1) return -1;
  return gen_p256_shard(n, 0, n, (size_t)nkeys, msg_len, corrupt_den, seed, nthreads, family, pub,
                        msg, moff, mlen, sig, soff, slen, reason, cls);
}

int gen_p256(size_t n, int nkeys, int msg_len, int corrupt_den, uint64_t seed, int nthreads,
             uint8_t *pub, uint8_t *msg, uint64_t *moff, uint32_t *mlen, uint8_t *sig,
             uint64_t *soff, uint32_t *slen, uint8_t *reason, uint8_t *cls) {
  return gen_p256_family(n, nkeys, msg_len, corrupt_den, seed, nthreads, 0, pub, msg, moff, mlen,
                         sig, soff, slen, reason, cls);
}

/* ---------------------------------------------------------------------------
 * BDLS round (BASELINE config 4): one height/round at `nval` validators as
 * consensus.go drives it: nval <roundchange>, one <lock> from the leader whose
 * message embeds t2p1 = 2t+1 roundchange proofs, those t2p1 proof SignedProtos
 * (re-verified by verifyLockMessage, consensus.go:549-584), nval <commit>, one
 * <decide> embedding t2p1 commit proofs and those proofs again
 * (verifyDecideMessage, :852-885). Records are SignedProto (message.go):
 * X, Y (32 B), R, S (big.Int.Bytes()), Version = 1, Message; hash =
 * BLAKE2b-256(prefix || ver || X || Y || len || msg) (:97-138).
 * ------------------------------------------------------------------------- */
static const uint64_t B2IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull,
                                 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
                                 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
static const uint8_t B2S[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
#define ROTR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))
#define B2G(a, b, c, d, x, y)              \
  do {                                     \
    v[a] = v[a] + v[b] + (x);              \
    v[d] = ROTR64(v[d] ^ v[a], 32);        \
    v[c] = v[c] + v[d];                    \
    v[b] = ROTR64(v[b] ^ v[c], 24);        \
    v[a] = v[a] + v[b] + (y);              \
    v[d] = ROTR64(v[d] ^ v[a], 16);        \
    v[c] = v[c] + v[d];                    \
    v[b] = ROTR64(v[b] ^ v[c], 63);        \
  } while (0)

static void b2_block(uint64_t h[8], const uint8_t blk[128], uint64_t t, int last) {
  uint64_t m[16], v[16];
  for (int i = 0; i < 16; i++) {
    uint64_t w = 0;
    for (int b = 7; b >= 0; b--) w = (w << 8) | blk[8 * i + b];
    m[i] = w;
  }
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = B2IV[i];
  }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
  for (int r = 0; r < 12; r++) {
    const uint8_t *s = B2S[r];
    B2G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    B2G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    B2G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    B2G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    B2G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    B2G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    B2G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    B2G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

/* SignedProto.Hash */
static void bdls_hash(uint8_t out[32], uint32_t ver, const uint8_t *x, const uint8_t *y,
                      const uint8_t *msg, uint32_t len) {
  static const char prefix[] = "BDLS_CONSENSUS_SIGNATURE";
  size_t total = 96 + (size_t)len;
  uint8_t *buf = malloc(total + 128);
  memcpy(buf, prefix, 24);
  for (int i = 0; i < 4; i++) buf[24 + i] = (uint8_t)(ver >> (8 * i));
  memcpy(buf + 28, x, 32);
  memcpy(buf + 60, y, 32);
  for (int i = 0; i < 4; i++) buf[92 + i] = (uint8_t)(len >> (8 * i));
  memcpy(buf + 96, msg, len);
  uint64_t h[8];
  for (int i = 0; i < 8; i++) h[i] = B2IV[i];
  h[0] ^= 0x01010000ull ^ 32ull;
  size_t pos = 0;
  for (;;) {
    uint8_t blk[128] = {0};
    int last = total - pos <= 128;
    size_t take = last ? total - pos : 128;
    memcpy(blk, buf + pos, take);
    b2_block(h, blk, last ? total : pos + 128, last);
    if (last) break;
    pos += 128;
  }
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(h[i >> 3] >> (8 * (i & 7)));
  free(buf);
}

typedef struct {
  uint8_t x[32], y[32], r[33], s[33];
  uint32_t rl, sl, ver, ml;
  uint8_t *msg;
} sproto;

static void sp_sign(sproto *o, EC_GROUP *g, BN_CTX *ctx, const BIGNUM *d, const uint8_t *x,
                    const uint8_t *y, const uint8_t *msg, uint32_t ml, uint64_t *st) {
  BIGNUM *n = BN_new(), *k = BN_new(), *kinv = BN_new(), *r = BN_new(), *s = BN_new(),
         *e = BN_new(), *t = BN_new(), *xr = BN_new();
  EC_POINT *R = EC_POINT_new(g);
  EC_GROUP_get_order(g, n, ctx);
  memcpy(o->x, x, 32);
  memcpy(o->y, y, 32);
  o->ver = 1;
  o->ml = ml;
  o->msg = malloc(ml ? ml : 1);
  memcpy(o->msg, msg, ml);
  uint8_t dg[32];
  bdls_hash(dg, 1, x, y, msg, ml);
  BN_bin2bn(dg, 32, e);
  BN_nnmod(e, e, n, ctx);
  do {
    rand_scalar(st, k, n, ctx);
    EC_POINT_mul(g, R, k, NULL, NULL, ctx);
    EC_POINT_get_affine_coordinates(g, R, xr, NULL, ctx);
    BN_nnmod(r, xr, n, ctx);
    BN_mod_inverse(kinv, k, n, ctx);
    BN_mod_mul(t, r, d, n, ctx);
    BN_mod_add(t, t, e, n, ctx);
    BN_mod_mul(s, kinv, t, n, ctx);
  } while (BN_is_zero(r) || BN_is_zero(s));
  o->rl = (uint32_t)BN_bn2bin(r, o->r);
  o->sl = (uint32_t)BN_bn2bin(s, o->s);
  EC_POINT_free(R);
  BIGNUM *v[] = {n, k, kinv, r, s, e, t, xr};
  for (int i = 0; i < 8; i++) BN_free(v[i]);
}

/* Writes up to cap records; returns the record count (2 nval + 2 (1 + t2p1)).
 * Buffers: xy cap*64, r/s cap*33 (+off/len), ver cap, msg msg_cap bytes. */
int gen_bdls_round(int curve, int nval, int t2p1, int small_len, uint64_t seed, int cap,
                   uint8_t *xy, uint8_t *rbuf, uint64_t *roff, uint32_t *rlen, uint8_t *sbuf,
                   uint64_t *soff, uint32_t *slen, uint32_t *ver, uint8_t *msg, uint64_t msg_cap,
                   uint64_t *moff, uint32_t *mlen) {
  const int total = 2 * nval + 2 * (1 + t2p1);
  if (total > cap || t2p1 > nval || nval < 1) return -1;
  EC_GROUP *g = EC_GROUP_new_by_curve_name(curve == 0 ? NID_X9_62_prime256v1 : NID_secp256k1);
  BN_CTX *ctx = BN_CTX_new();
  BIGNUM *n = BN_new(), *px = BN_new(), *py = BN_new();
  EC_GROUP_get_order(g, n, ctx);
  EC_POINT *Q = EC_POINT_new(g);
  BIGNUM **d = malloc(sizeof(BIGNUM *) * nval);
  uint8_t(*kx)[32] = malloc(32 * (size_t)nval), (*ky)[32] = malloc(32 * (size_t)nval);
  uint64_t st = seed * 0x9e3779b97f4a7c15ull + 0xbd15ull;
  for (int v = 0; v < nval; v++) {
    d[v] = BN_new();
    rand_scalar(&st, d[v], n, ctx);
    EC_POINT_mul(g, Q, d[v], NULL, NULL, ctx);
    EC_POINT_get_affine_coordinates(g, Q, px, py, ctx);
    BN_bn2binpad(px, kx[v], 32);
    BN_bn2binpad(py, ky[v], 32);
  }
  sproto *rec = calloc((size_t)total, sizeof(sproto));
  uint8_t *tmp = malloc((size_t)small_len + 64);
  int k = 0;
  /* phase 0: roundchange, phase 1: commit */
  for (int ph = 0; ph < 2; ph++) {
    int first = k;
    for (int v = 0; v < nval; v++) {
      rand_bytes(&st, tmp, (size_t)small_len);
      tmp[0] = (uint8_t)(ph ? 0x3a : 0x2a); /* message type tag */
      sp_sign(&rec[k++], g, ctx, d[v], kx[v], ky[v], tmp, (uint32_t)small_len, &st);
    }
    /* <lock> / <decide> by the leader, embedding t2p1 proofs */
    size_t agg_len = 0;
    for (int p = 0; p < t2p1; p++) agg_len += 64 + rec[first + p].rl + rec[first + p].sl + rec[first + p].ml + 8;
    uint8_t *agg = malloc(agg_len + 16), *a = agg;
    for (int p = 0; p < t2p1; p++) {
      sproto *q = &rec[first + p];
      memcpy(a, q->x, 32); a += 32;
      memcpy(a, q->y, 32); a += 32;
      memcpy(a, q->r, q->rl); a += q->rl;
      memcpy(a, q->s, q->sl); a += q->sl;
      memcpy(a, q->msg, q->ml); a += q->ml;
      for (int b = 0; b < 8; b++) *a++ = (uint8_t)p;
    }
    sp_sign(&rec[k++], g, ctx, d[0], kx[0], ky[0], agg, (uint32_t)agg_len, &st);
    free(agg);
    for (int p = 0; p < t2p1; p++) { /* proofs re-verified as their own records */
      sproto *q = &rec[k++];
      *q = rec[first + p];
      q->msg = malloc(q->ml ? q->ml : 1);
      memcpy(q->msg, rec[first + p].msg, q->ml);
    }
  }
  uint64_t mo = 0;
  int rc = total;
  for (int i = 0; i < total; i++) {
    memcpy(xy + 64 * (size_t)i, rec[i].x, 32);
    memcpy(xy + 64 * (size_t)i + 32, rec[i].y, 32);
    memcpy(rbuf + 33 * (size_t)i, rec[i].r, rec[i].rl);
    memcpy(sbuf + 33 * (size_t)i, rec[i].s, rec[i].sl);
    roff[i] = 33 * (uint64_t)i;
    soff[i] = 33 * (uint64_t)i;
    rlen[i] = rec[i].rl;
    slen[i] = rec[i].sl;
    ver[i] = rec[i].ver;
    if (mo + rec[i].ml > msg_cap) rc = -2;
    else memcpy(msg + mo, rec[i].msg, rec[i].ml);
    moff[i] = mo;
    mlen[i] = rec[i].ml;
    mo += rec[i].ml;
    free(rec[i].msg);
  }
  free(rec);
  free(tmp);
  for (int v = 0; v < nval; v++) BN_free(d[v]);
  free(d);
  free(kx);
  free(ky);
  EC_POINT_free(Q);
  BN_free(n); BN_free(px); BN_free(py);
  BN_CTX_free(ctx);
  EC_GROUP_free(g);
  return rc;
}

/* ---------------------------------------------------------------------------
 * BDLS round as raw wire messages (input of bh_bdls_preverify): SignedProto
 * encodings (message.pb.go MarshalToSizedBuffer :300-356) of signed Messages
 * (:358-): nval <roundchange> (Type 1) + the leader's <lock> (Type 2) with
 * t2p1 roundchange proofs + nval <commit> (Type 4) + the leader's <decide>
 * (Type 6) with t2p1 commit proofs. Height 1, round 0, so the leader is
 * participant 0 (consensus.go roundLeader :1148-1154). All valid.
 * ------------------------------------------------------------------------- */
static size_t pb_varint(uint8_t *o, uint64_t v) {
  size_t k = 0;
  while (v >= 0x80) { o[k++] = (uint8_t)(v | 0x80); v >>= 7; }
  o[k++] = (uint8_t)v;
  return k;
}

static size_t pb_bytes(uint8_t *o, uint8_t tag, const uint8_t *b, size_t n) {
  size_t k = 0;
  o[k++] = tag;
  k += pb_varint(o + k, n);
  memcpy(o + k, b, n);
  return k + n;
}

static size_t pb_signed(uint8_t *o, const sproto *s) { /* worst case 16 + ml + 2*34 + 2*35 */
  size_t k = 0;
  if (s->ver) { o[k++] = 0x08; k += pb_varint(o + k, s->ver); }
  if (s->ml) k += pb_bytes(o + k, 0x12, s->msg, s->ml);
  k += pb_bytes(o + k, 0x1a, s->x, 32);
  k += pb_bytes(o + k, 0x22, s->y, 32);
  if (s->rl) k += pb_bytes(o + k, 0x2a, s->r, s->rl);
  if (s->sl) k += pb_bytes(o + k, 0x32, s->s, s->sl);
  return k;
}

static size_t pb_message(uint8_t *o, uint32_t type, uint64_t h, uint64_t r, const uint8_t *st,
                         size_t stl, const sproto *proofs, int np) {
  size_t k = 0;
  if (type) { o[k++] = 0x08; k += pb_varint(o + k, type); }
  if (h) { o[k++] = 0x10; k += pb_varint(o + k, h); }
  if (r) { o[k++] = 0x18; k += pb_varint(o + k, r); }
  if (stl) k += pb_bytes(o + k, 0x22, st, stl);
  for (int p = 0; p < np; p++) {
    uint8_t tmp[1024];
    size_t l = pb_signed(tmp, &proofs[p]);
    k += pb_bytes(o + k, 0x2a, tmp, l);
  }
  return k;
}

/* parts: nval*64 (X || Y); out: cap bytes of raw messages; off/len: 2*nval+2.
 * Returns the message count, or < 0. */
int gen_bdls_wire_round(int curve, int nval, int t2p1, uint64_t seed, uint8_t *parts,
                        uint8_t *out, uint64_t cap, uint64_t *off, uint32_t *len) {
  if (nval < 1 || t2p1 > nval) return -1;
  EC_GROUP *g = EC_GROUP_new_by_curve_name(curve == 0 ? NID_X9_62_prime256v1 : NID_secp256k1);
  BN_CTX *ctx = BN_CTX_new();
  BIGNUM *n = BN_new(), *px = BN_new(), *py = BN_new();
  EC_GROUP_get_order(g, n, ctx);
  EC_POINT *Q = EC_POINT_new(g);
  BIGNUM **d = malloc(sizeof(BIGNUM *) * nval);
  uint64_t st = seed * 0x9e3779b97f4a7c15ull + 0x3172ull;
  for (int v = 0; v < nval; v++) {
    d[v] = BN_new();
    rand_scalar(&st, d[v], n, ctx);
    EC_POINT_mul(g, Q, d[v], NULL, NULL, ctx);
    EC_POINT_get_affine_coordinates(g, Q, px, py, ctx);
    BN_bn2binpad(px, parts + 64 * (size_t)v, 32);
    BN_bn2binpad(py, parts + 64 * (size_t)v + 32, 32);
  }
  uint8_t state[64];
  rand_bytes(&st, state, sizeof state);
  sproto *rc = calloc((size_t)nval, sizeof(sproto)), *cm = calloc((size_t)nval, sizeof(sproto));
  uint8_t mb[256];
  for (int v = 0; v < nval; v++) {
    size_t ml = pb_message(mb, 1, 1, 0, state, sizeof state, NULL, 0);
    sp_sign(&rc[v], g, ctx, d[v], parts + 64 * (size_t)v, parts + 64 * (size_t)v + 32, mb,
            (uint32_t)ml, &st);
    ml = pb_message(mb, 4, 1, 0, state, sizeof state, NULL, 0);
    sp_sign(&cm[v], g, ctx, d[v], parts + 64 * (size_t)v, parts + 64 * (size_t)v + 32, mb,
            (uint32_t)ml, &st);
  }
  const size_t big = 256 + (size_t)t2p1 * 512;
  uint8_t *lm = malloc(big), *dm = malloc(big);
  sproto lock, dec;
  size_t ll = pb_message(lm, 2, 1, 0, state, sizeof state, rc, t2p1);
  size_t dl = pb_message(dm, 6, 1, 0, state, sizeof state, cm, t2p1);
  sp_sign(&lock, g, ctx, d[0], parts, parts + 32, lm, (uint32_t)ll, &st);
  sp_sign(&dec, g, ctx, d[0], parts, parts + 32, dm, (uint32_t)dl, &st);
  uint64_t pos = 0;
  int k = 0, rc_ = 0;
  const sproto *seq[4] = {rc, &lock, cm, &dec};
  const int cnt[4] = {nval, 1, nval, 1};
  for (int q = 0; q < 4 && rc_ == 0; q++)
    for (int v = 0; v < cnt[q]; v++) {
      const size_t need = 96 + seq[q][v].ml + 80;
      if (pos + need > cap) { rc_ = -2; break; }
      const size_t l = pb_signed(out + pos, &seq[q][v]);
      off[k] = pos;
      len[k] = (uint32_t)l;
      pos += l;
      k++;
    }
  for (int v = 0; v < nval; v++) { free(rc[v].msg); free(cm[v].msg); BN_free(d[v]); }
  free(lock.msg); free(dec.msg); free(lm); free(dm); free(rc); free(cm); free(d);
  EC_POINT_free(Q);
  BN_free(n); BN_free(px); BN_free(py);
  BN_CTX_free(ctx);
  EC_GROUP_free(g);
  return rc_ ? rc_ : k;
}

/* ---------------------------------------------------------------------------
 * Helpers for the Fabric block generator (bdls_amd/workload/fabric.py): seeded
 * P-256 key pairs and DER signatures over given 32-byte digests, signed as
 * bccsp/sw/ecdsa.go:27-39 signs (ecdsa.Sign, ToLowS, MarshalECDSASignature).
 * ------------------------------------------------------------------------- */
int gen_p256_keypair(uint64_t seed, uint64_t idx, uint8_t *priv32, uint8_t *pub64) {
  EC_GROUP *g = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
  BN_CTX *ctx = BN_CTX_new();
  BIGNUM *n = BN_new(), *d = BN_new(), *x = BN_new(), *y = BN_new();
  EC_GROUP_get_order(g, n, ctx);
  EC_POINT *Q = EC_POINT_new(g);
  uint64_t st = seed * 0xff51afd7ed558ccdull + idx * 0xc4ceb9fe1a85ec53ull + 7;
  rand_scalar(&st, d, n, ctx);
  EC_POINT_mul(g, Q, d, NULL, NULL, ctx);
  EC_POINT_get_affine_coordinates(g, Q, x, y, ctx);
  BN_bn2binpad(d, priv32, 32);
  BN_bn2binpad(x, pub64, 32);
  BN_bn2binpad(y, pub64 + 32, 32);
  EC_POINT_free(Q);
  BN_free(n); BN_free(d); BN_free(x); BN_free(y);
  BN_CTX_free(ctx);
  EC_GROUP_free(g);
  return 0;
}

/* n signatures: record i signs digest i (32 B) with private key i (32 B);
 * out + 80 i receives the DER signature, len[i] its length. high_s != 0
 * leaves S as drawn (possibly > n/2) instead of normalising to low-S. */
int gen_p256_sign_batch(size_t n, const uint8_t *priv, const uint8_t *digest, uint64_t seed,
                        int high_s, uint8_t *out, uint32_t *len) {
  EC_GROUP *g = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
  BN_CTX *ctx = BN_CTX_new();
  BIGNUM *nn = BN_new(), *half = BN_new(), *k = BN_new(), *kinv = BN_new(), *r = BN_new(),
         *s = BN_new(), *e = BN_new(), *d = BN_new(), *t = BN_new(), *x = BN_new();
  EC_GROUP_get_order(g, nn, ctx);
  BN_rshift1(half, nn);
  EC_POINT *R = EC_POINT_new(g);
  for (size_t i = 0; i < n; i++) {
    uint64_t st = seed * 0x100000001b3ull + i * 0x9e3779b97f4a7c15ull + 0x51;
    BN_bin2bn(priv + 32 * i, 32, d);
    BN_bin2bn(digest + 32 * i, 32, e);
    BN_nnmod(e, e, nn, ctx);
    do {
      rand_scalar(&st, k, nn, ctx);
      EC_POINT_mul(g, R, k, NULL, NULL, ctx);
      EC_POINT_get_affine_coordinates(g, R, x, NULL, ctx);
      BN_nnmod(r, x, nn, ctx);
      BN_mod_inverse(kinv, k, nn, ctx);
      BN_mod_mul(t, r, d, nn, ctx);
      BN_mod_add(t, t, e, nn, ctx);
      BN_mod_mul(s, kinv, t, nn, ctx);
    } while (BN_is_zero(r) || BN_is_zero(s));
    if (high_s) {
      if (BN_cmp(s, half) <= 0) BN_sub(s, nn, s);
    } else if (BN_cmp(s, half) > 0) {
      BN_sub(s, nn, s);
    }
    uint8_t body[SIG_STRIDE], *o = out + (size_t)i * SIG_STRIDE;
    size_t bl = der_int(body, r, 0, 0);
    bl += der_int(body + bl, s, 0, 0);
    o[0] = 0x30;
    o[1] = (uint8_t)bl;
    memcpy(o + 2, body, bl);
    len[i] = (uint32_t)(bl + 2);
  }
  EC_POINT_free(R);
  BIGNUM *v[] = {nn, half, k, kinv, r, s, e, d, t, x};
  for (size_t q = 0; q < sizeof(v) / sizeof(v[0]); q++) BN_free(v[q]);
  BN_CTX_free(ctx);
  EC_GROUP_free(g);
  return 0;
}
