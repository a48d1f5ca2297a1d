/*
 * Synthetic workload generator for bench.py and the large parity tests.
 * Produces BASELINE.json configs as verify records:
 *   config 2: n records, `nkeys` distinct P-256 keys, `msg_len`-byte random
 *             messages (fused SHA-256), 1/`corrupt_den` of the records
 *             corrupted over the eleven classes below, seeded.
 *   config 5: nkeys == n (one distinct key per record).
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
  size_t lo, hi, n;
  uint64_t seed;
  int nkeys, msg_len, corrupt_den;
  const uint8_t *keypub; /* nkeys * 64 */
  const uint8_t *keypriv; /* nkeys * 32 */
  uint8_t *pub, *msg, *sig, *reason, *cls;
  uint64_t *moff, *soff;
  uint32_t *mlen, *slen;
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
  EC_POINT *R = EC_POINT_new(g);
  uint8_t dg[32], b32[32];
  for (size_t i = j->lo; i < j->hi; i++) {
    uint64_t st = j->seed * 0x100000001b3ull + i * 0x9e3779b97f4a7c15ull + 17;
    splitmix(&st);
    const int key = (int)(splitmix(&st) % (uint64_t)j->nkeys);
    int cls = C_NONE;
    if (j->corrupt_den > 0 && splitmix(&st) % (uint64_t)j->corrupt_den == 0)
      cls = 1 + (int)(splitmix(&st) % (C_NUM - 1));
    uint8_t *m = j->msg + (size_t)i * j->msg_len;
    rand_bytes(&st, m, j->msg_len);
    j->moff[i] = (uint64_t)i * j->msg_len;
    j->mlen[i] = (uint32_t)j->msg_len;
    SHA256(m, j->msg_len, dg);
    /* sign: r = x(kG) mod n, s = k^-1 (e + r d) mod n, low-S */
    BN_bin2bn(j->keypriv + 32 * key, 32, d);
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
    memcpy(q, j->keypub + 64 * key, 64);
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

/* Caller allocates: pub n*64, msg n*msg_len, sig n*80, moff/soff n u64,
 * mlen/slen n u32, reason/cls n u8. */
int gen_p256(size_t n, int nkeys, int msg_len, int corrupt_den, uint64_t seed, int nthreads,
             uint8_t *pub, uint8_t *msg, uint64_t *moff, uint32_t *mlen, uint8_t *sig,
             uint64_t *soff, uint32_t *slen, uint8_t *reason, uint8_t *cls) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 128) nthreads = 128;
  if (nkeys < 1 || msg_len < 1) return -1;
  uint8_t *kpub = malloc((size_t)nkeys * 64), *kpriv = malloc((size_t)nkeys * 32);
  if (!kpub || !kpriv) return -2;
  pthread_t th[128];
  kjob kj[128];
  int per = (nkeys + nthreads - 1) / nthreads, used = 0;
  for (int t = 0; t < nthreads; t++) {
    int lo = t * per, hi = lo + per > nkeys ? nkeys : lo + per;
    if (lo >= hi) break;
    kj[t] = (kjob){lo, hi, seed, kpub, kpriv};
    pthread_create(&th[t], NULL, key_worker, &kj[t]);
    used++;
  }
  for (int t = 0; t < used; t++) pthread_join(th[t], NULL);
  gjob gj[128];
  size_t gper = (n + nthreads - 1) / nthreads;
  used = 0;
  for (int t = 0; t < nthreads; t++) {
    size_t lo = t * gper, hi = lo + gper > n ? n : lo + gper;
    if (lo >= hi) break;
    gj[t] = (gjob){lo, hi, n, seed, nkeys, msg_len, corrupt_den, kpub, kpriv,
                   pub, msg, sig, reason, cls, moff, soff, mlen, slen};
    pthread_create(&th[t], NULL, gen_worker, &gj[t]);
    used++;
  }
  for (int t = 0; t < used; t++) pthread_join(th[t], NULL);
  free(kpub);
  free(kpriv);
  return 0;
}
