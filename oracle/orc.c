/*
 * CPU ORACLE (test infrastructure only) -- C restatement of the reference's
 * ECDSA acceptance predicate, multi-threaded, used
 *   (1) by tests/ to cross-check oracle/ecdsa_ref.py and the HIP path, and
 *   (2) by bench.py's cpu_baseline leg ("kind": "port").
 * The product library (libbdlship.so) never links or calls this file.
 *
 * Restated reference code (/root/reference):
 *   bccsp/sw/impl.go:247-270        CSP.Verify argument checks
 *   bccsp/sw/ecdsa.go:41-57         verifyECDSA (unmarshal -> low-S -> ecdsa.Verify)
 *   bccsp/utils/ecdsa.go:41-65,82-89 UnmarshalECDSASignature / IsLowS
 *   msp/identities.go:170-199       identity.Verify = SHA-256(msg) then Verify
 *   Go 1.21.4 encoding/asn1 (parseTagAndLength, parseField, checkInteger) and
 *   crypto/ecdsa verifyNISTEC / hashToNat / pointFromAffine (stdlib, not
 *   vendored; pinned by the reference Makefile:81 GO_VER = 1.21.4).
 * The DER rules, argument checks, low-S rule, key and r/s range checks are
 * restated here; the final group equation x(u1 G + u2 Q) mod n == r is
 * delegated to OpenSSL libcrypto 3.0 ECDSA_do_verify (prime256v1 / secp256k1),
 * an implementation independent of both this repo's HIP kernels and
 * oracle/ecdsa_ref.py, and comparable in speed to Go's P-256 assembly (hence
 * also the cpu_baseline proxy for bccsp/sw).
 */
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* reason codes: keep equal to include/bdls_hip.h BH_R_* and ecdsa_ref.py */
enum { R_OK = 0, R_EMPTY_SIG = 1, R_EMPTY_DIGEST = 2, R_DER = 3, R_R_NONPOS = 4,
       R_S_NONPOS = 5, R_HIGH_S = 6, R_BAD_KEY = 7, R_R_RANGE = 8, R_MATH = 9,
       R_S_RANGE = 10 };

/* ---- encoding/asn1 restatement ------------------------------------------ */
/* parseTagAndLength (Go 1.21.4). Returns 0 on success. */
static int tag_len(const uint8_t *b, size_t n, size_t *off, int *cls, int *cmp, long *tag,
                   size_t *len) {
  if (*off >= n) return -1;
  uint8_t t = b[(*off)++];
  *cls = t >> 6;
  *cmp = (t & 0x20) != 0;
  *tag = t & 0x1f;
  if (*tag == 0x1f) { /* parseBase128Int */
    long v = 0;
    int shifted = 0;
    for (;;) {
      if (*off >= n) return -1;
      if (shifted == 5) return -1;
      uint8_t x = b[*off];
      if (shifted == 0 && x == 0x80) return -1;
      v = (v << 7) | (x & 0x7f);
      (*off)++;
      shifted++;
      if (!(x & 0x80)) break;
    }
    if (v > 0x7fffffffL) return -1;
    if (v < 0x1f) return -1;
    *tag = v;
  }
  if (*off >= n) return -1;
  uint8_t lb = b[(*off)++];
  if (!(lb & 0x80)) {
    *len = lb & 0x7f;
    return 0;
  }
  int nb = lb & 0x7f;
  if (nb == 0) return -1;
  size_t L = 0;
  for (int i = 0; i < nb; i++) {
    if (*off >= n) return -1;
    uint8_t x = b[(*off)++];
    if (L >= (1u << 23)) return -1;
    L = (L << 8) | x;
    if (L == 0) return -1;
  }
  if (L < 0x80) return -1;
  *len = L;
  return 0;
}

/* parseField for a *big.Int: returns 0 ok; *sign = -1/0/+1; mag = magnitude
 * bytes (leading zero stripped) for positive values. */
static int parse_int(const uint8_t *b, size_t n, size_t *off, int *sign, const uint8_t **mag,
                     size_t *maglen) {
  if (*off == n) return -1; /* sequence truncated */
  int cls, cmp;
  long tag;
  size_t len;
  if (tag_len(b, n, off, &cls, &cmp, &tag, &len)) return -1;
  if (cls != 0 || tag != 2 || cmp) return -1;
  if (*off + len > n || *off + len < *off) return -1;
  const uint8_t *p = b + *off;
  *off += len;
  if (len == 0) return -1; /* empty integer */
  if (len > 1 && ((p[0] == 0 && !(p[1] & 0x80)) || (p[0] == 0xff && (p[1] & 0x80))))
    return -1; /* not minimally encoded */
  if (p[0] & 0x80) {
    *sign = -1;
    *mag = NULL;
    *maglen = 0;
    return 0;
  }
  if (len == 1 && p[0] == 0) {
    *sign = 0;
    *mag = NULL;
    *maglen = 0;
    return 0;
  }
  *sign = 1;
  if (p[0] == 0) {
    p++;
    len--;
  }
  *mag = p;
  *maglen = len;
  return 0;
}

/* bccsp/utils/ecdsa.go:41-65 -> reason; on R_OK fills r, s magnitudes. */
static int unmarshal_sig(const uint8_t *sig, size_t n, const uint8_t **r, size_t *rl,
                         const uint8_t **s, size_t *sl) {
  size_t off = 0;
  int cls, cmp;
  long tag;
  size_t len;
  if (n == 0) return R_DER;
  if (tag_len(sig, n, &off, &cls, &cmp, &tag, &len)) return R_DER;
  if (cls != 0 || tag != 16 || !cmp) return R_DER;
  if (off + len > n) return R_DER;
  const uint8_t *in = sig + off;
  size_t io = 0;
  int rs, ss;
  if (parse_int(in, len, &io, &rs, r, rl)) return R_DER;
  if (parse_int(in, len, &io, &ss, s, sl)) return R_DER;
  /* extra SEQUENCE elements and trailing bytes are accepted (Go asn1) */
  if (rs <= 0) return R_R_NONPOS;
  if (ss <= 0) return R_S_NONPOS;
  return R_OK;
}

/* ---- per-thread curve context ------------------------------------------- */
typedef struct {
  EC_GROUP *g;
  BN_CTX *ctx;
  BIGNUM *p, *a, *b, *n, *half, *r, *s, *e, *w, *u1, *u2, *x, *y, *t;
  EC_POINT *Q, *X;
  EC_KEY *key;
  int nist;
} orc_ctx;

static void ctx_init(orc_ctx *c, int curve) {
  c->nist = (curve == 0);
  c->g = EC_GROUP_new_by_curve_name(curve == 0 ? NID_X9_62_prime256v1 : NID_secp256k1);
  c->ctx = BN_CTX_new();
  BIGNUM **v[] = {&c->p, &c->a, &c->b, &c->n, &c->half, &c->r, &c->s, &c->e,
                  &c->w, &c->u1, &c->u2, &c->x, &c->y, &c->t};
  for (size_t i = 0; i < sizeof(v) / sizeof(v[0]); i++) *v[i] = BN_new();
  EC_GROUP_get_curve(c->g, c->p, c->a, c->b, c->ctx);
  EC_GROUP_get_order(c->g, c->n, c->ctx);
  BN_rshift1(c->half, c->n);
  c->Q = EC_POINT_new(c->g);
  c->X = EC_POINT_new(c->g);
  c->key = EC_KEY_new_by_curve_name(curve == 0 ? NID_X9_62_prime256v1 : NID_secp256k1);
}

static void ctx_free(orc_ctx *c) {
  BIGNUM *v[] = {c->p, c->a, c->b, c->n, c->half, c->r, c->s, c->e,
                 c->w, c->u1, c->u2, c->x, c->y, c->t};
  for (size_t i = 0; i < sizeof(v) / sizeof(v[0]); i++) BN_free(v[i]);
  EC_POINT_free(c->Q);
  EC_POINT_free(c->X);
  EC_KEY_free(c->key);
  BN_CTX_free(c->ctx);
  EC_GROUP_free(c->g);
}

/* Go crypto/ecdsa.Verify on (Q, digest, r, s) with r, s > 0 (set in c->r/s). */
static int go_verify(orc_ctx *c, const uint8_t q[64], const uint8_t *dg, size_t dl) {
  BN_bin2bn(q, 32, c->x);
  BN_bin2bn(q + 32, 32, c->y);
  if (c->nist) {
    /* pointFromAffine: coordinates < p and on the curve */
    if (BN_cmp(c->x, c->p) >= 0 || BN_cmp(c->y, c->p) >= 0) return R_BAD_KEY;
    if (!EC_POINT_set_affine_coordinates(c->g, c->Q, c->x, c->y, c->ctx)) return R_BAD_KEY;
    if (EC_POINT_is_on_curve(c->g, c->Q, c->ctx) != 1) return R_BAD_KEY;
  }
  if (BN_cmp(c->r, c->n) >= 0) return R_R_RANGE;
  if (BN_cmp(c->s, c->n) >= 0) return R_S_RANGE;
  if (!c->nist) {
    if (!EC_POINT_set_affine_coordinates(c->g, c->Q, c->x, c->y, c->ctx)) return R_MATH;
  }
  /* e = hashToNat / hashToInt (left-most 32 bytes), w = s^-1, u1 = e w,
   * u2 = r w, x(u1 G + u2 Q) mod n == r, infinity -> false: OpenSSL's
   * ECDSA_do_verify computes exactly this predicate for r, s in [1, n-1]
   * (its digest truncation to the order's bit length equals Go's for 256-bit
   * orders), using its optimised P-256 code path. */
  if (!EC_KEY_set_public_key(c->key, c->Q)) return R_MATH;
  ECDSA_SIG *sig = ECDSA_SIG_new();
  ECDSA_SIG_set0(sig, BN_dup(c->r), BN_dup(c->s));
  int ok = ECDSA_do_verify(dg, (int)dl, sig, c->key);
  ECDSA_SIG_free(sig);
  return ok == 1 ? R_OK : R_MATH;
}

/* bccsp/sw/impl.go:247-270 + bccsp/sw/ecdsa.go:41-57 */
static int csp_verify(orc_ctx *c, const uint8_t q[64], const uint8_t *sig, size_t sl,
                      const uint8_t *dg, size_t dl) {
  if (sl == 0) return R_EMPTY_SIG;
  if (dl == 0) return R_EMPTY_DIGEST;
  const uint8_t *r, *s;
  size_t rl, sl2;
  int rc = unmarshal_sig(sig, sl, &r, &rl, &s, &sl2);
  if (rc != R_OK) return rc;
  BN_bin2bn(r, (int)rl, c->r);
  BN_bin2bn(s, (int)sl2, c->s);
  if (c->nist && BN_cmp(c->s, c->half) > 0) return R_HIGH_S;
  return go_verify(c, q, dg, dl);
}

/* ---- exported API (ctypes) ---------------------------------------------- */
int orc_unmarshal(const uint8_t *sig, size_t n, uint8_t r32[32], uint8_t s32[32], int *r_big,
                  int *s_big) {
  const uint8_t *r, *s;
  size_t rl, sl;
  int rc = unmarshal_sig(sig, n, &r, &rl, &s, &sl);
  memset(r32, 0, 32);
  memset(s32, 0, 32);
  *r_big = *s_big = 0;
  if (rc != R_OK) return rc;
  if (rl > 32) *r_big = 1; else memcpy(r32 + 32 - rl, r, rl);
  if (sl > 32) *s_big = 1; else memcpy(s32 + 32 - sl, s, sl);
  return rc;
}

int orc_csp_verify(int curve, const uint8_t q[64], const uint8_t *sig, size_t sl,
                   const uint8_t *dg, size_t dl) {
  orc_ctx c;
  ctx_init(&c, curve);
  int rc = csp_verify(&c, q, sig, sl, dg, dl);
  ctx_free(&c);
  return rc;
}

/* Go ecdsa.Verify with integer r, s given as 32-byte big-endian (r, s > 0). */
int orc_go_verify(int curve, const uint8_t q[64], const uint8_t *dg, size_t dl,
                  const uint8_t r32[32], const uint8_t s32[32]) {
  orc_ctx c;
  ctx_init(&c, curve);
  BN_bin2bn(r32, 32, c.r);
  BN_bin2bn(s32, 32, c.s);
  int rc = (BN_is_zero(c.r) ? R_R_NONPOS : BN_is_zero(c.s) ? R_S_NONPOS : go_verify(&c, q, dg, dl));
  ctx_free(&c);
  return rc;
}

typedef struct {
  size_t lo, hi;
  int curve, fused;
  const uint8_t *q;
  const uint8_t *msg;
  const uint64_t *moff;
  const uint32_t *mlen;
  const uint8_t *sig;
  const uint64_t *soff;
  const uint32_t *slen;
  uint8_t *reason;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  orc_ctx c;
  ctx_init(&c, j->curve);
  uint8_t dg[32];
  for (size_t i = j->lo; i < j->hi; i++) {
    const uint8_t *m = j->msg + j->moff[i];
    size_t ml = j->mlen[i];
    if (j->fused) { /* msp/identities.go:179 Hash then :190 Verify */
      if (j->fused == 2) /* SHA3 family: sha3.New256, bccsp/sw/new.go:72 */
        EVP_Digest(m, ml, dg, NULL, EVP_sha3_256(), NULL);
      else
        SHA256(m, ml, dg);
      m = dg;
      ml = 32;
    }
    j->reason[i] = (uint8_t)csp_verify(&c, j->q + 64 * i, j->sig + j->soff[i], j->slen[i], m, ml);
  }
  ctx_free(&c);
  return NULL;
}

/* Batch: fused == 1 -> msg is hashed with SHA-256 first (identity.Verify,
 * SHA2 family); fused == 2 -> with SHA3-256 (SHA3 family); fused == 0 -> msg
 * is the digest (CSP.Verify). reason[i] == 0 <=> valid. */
int orc_batch_verify(int curve, int fused, size_t n, const uint8_t *q, const uint8_t *msg,
                     const uint64_t *moff, const uint32_t *mlen, const uint8_t *sig,
                     const uint64_t *soff, const uint32_t *slen, uint8_t *reason, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  job_t jobs[256];
  size_t per = (n + nthreads - 1) / nthreads;
  int used = 0;
  for (int t = 0; t < nthreads; t++) {
    size_t lo = t * per, hi = lo + per > n ? n : lo + per;
    if (lo >= hi) break;
    jobs[t] = (job_t){lo, hi, curve, fused, q, msg, moff, mlen, sig, soff, slen, reason};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
    used++;
  }
  for (int t = 0; t < used; t++) pthread_join(th[t], NULL);
  return 0;
}

/* ---- BDLS SignedProto.Verify ---------------------------------------------
 * vendor/github.com/BDLS-bft/bdls/message.go:97-138 (Hash: BLAKE2b-256 over
 * prefix || Version LE || X || Y || len(Message) LE || Message) and :170-184
 * (Verify: ecdsa.Verify(pub, Hash(), SetBytes(R), SetBytes(S))). BLAKE2b per
 * RFC 7693 (Go's golang.org/x/crypto/blake2b New256, unkeyed). */
static const uint64_t kIV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull,
                                0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
                                0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
static const uint8_t kSig[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

static uint64_t rr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void b2_compress(uint64_t h[8], const uint8_t *blk, uint64_t t, int last) {
  uint64_t m[16], v[16];
  for (int i = 0; i < 16; i++) {
    m[i] = 0;
    for (int b = 0; b < 8; b++) m[i] |= (uint64_t)blk[8 * i + b] << (8 * b);
  }
  memcpy(v, h, 64);
  memcpy(v + 8, kIV, 64);
  v[12] ^= t;
  if (last) v[14] ^= ~0ull;
  static const int G[8][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15},
                              {0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}};
  for (int r = 0; r < 12; r++) {
    const uint8_t *s = kSig[r % 10];
    for (int g = 0; g < 8; g++) {
      int a = G[g][0], b = G[g][1], c = G[g][2], d = G[g][3];
      v[a] += v[b] + m[s[2 * g]];
      v[d] = rr64(v[d] ^ v[a], 32);
      v[c] += v[d];
      v[b] = rr64(v[b] ^ v[c], 24);
      v[a] += v[b] + m[s[2 * g + 1]];
      v[d] = rr64(v[d] ^ v[a], 16);
      v[c] += v[d];
      v[b] = rr64(v[b] ^ v[c], 63);
    }
  }
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

static void bdls_hash(uint8_t out[32], uint32_t ver, const uint8_t xy[64], const uint8_t *msg,
                      uint32_t ml) {
  uint8_t hdr[96];
  memcpy(hdr, "BDLS_CONSENSUS_SIGNATURE", 24);
  for (int i = 0; i < 4; i++) hdr[24 + i] = (uint8_t)(ver >> (8 * i));
  memcpy(hdr + 28, xy, 64);
  for (int i = 0; i < 4; i++) hdr[92 + i] = (uint8_t)(ml >> (8 * i));
  uint64_t h[8];
  memcpy(h, kIV, 64);
  h[0] ^= 0x01010020ull;
  const uint64_t total = 96 + (uint64_t)ml;
  uint8_t blk[128];
  for (uint64_t pos = 0;; pos += 128) {
    const int last = total - pos <= 128;
    for (int k = 0; k < 128; k++) {
      uint64_t p = pos + k;
      blk[k] = p >= total ? 0 : p < 96 ? hdr[p] : msg[p - 96];
    }
    b2_compress(h, blk, last ? total : pos + 128, last);
    if (last) break;
  }
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(h[i / 8] >> (8 * (i % 8)));
}

int orc_bdls_hash(uint32_t ver, const uint8_t xy[64], const uint8_t *msg, uint32_t ml,
                  uint8_t out[32]) {
  bdls_hash(out, ver, xy, msg, ml);
  return 0;
}

/* Serial, as the consensus loop verifies (consensus.go:456-466 then the
 * message's own Verify and, for <lock>/<decide>, each proof). */
int orc_bdls_verify(int curve, size_t n, const uint8_t *xy, const uint8_t *r, const uint64_t *roff,
                    const uint32_t *rlen, const uint8_t *s, const uint64_t *soff,
                    const uint32_t *slen, const uint32_t *ver, const uint8_t *msg,
                    const uint64_t *moff, const uint32_t *mlen, uint8_t *reason) {
  orc_ctx c;
  ctx_init(&c, curve);
  uint8_t dg[32];
  for (size_t i = 0; i < n; i++) {
    bdls_hash(dg, ver[i], xy + 64 * i, msg + moff[i], mlen[i]);
    BN_bin2bn(r + roff[i], (int)rlen[i], c.r);
    BN_bin2bn(s + soff[i], (int)slen[i], c.s);
    reason[i] = (uint8_t)(BN_is_zero(c.r)   ? R_R_NONPOS
                          : BN_is_zero(c.s) ? R_S_NONPOS
                                            : go_verify(&c, xy + 64 * i, dg, 32));
  }
  ctx_free(&c);
  return 0;
}
