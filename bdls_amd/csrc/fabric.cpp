// Fabric block pre-verification (bh_fabric_block_preverify, include/bdls_hip.h).
//
// Host side of SURVEY.md 8(f) rank 1 (rows A9-A12): the peer validates a block
// with one goroutine per transaction (core/committer/txvalidator/v20/
// validator.go:180-265, validateTx :297-453), and every transaction costs one
// creator signature check (core/common/validation/msgvalidation.go:26-64 via
// ValidateTransaction :248-320) plus one check per endorsement inside the
// endorsement-policy evaluation (statebased/validator_keylevel.go:244-282 ->
// common/policies/policy.go:363-395 SignatureSetToValidIdentities), each a
// separate bccsp Verify. Here the serialized block is decoded once, every
// signature the validator would check is put into ONE device batch
// (bh_verify, fused SHA-256 / SHA3-256 of the signed bytes), and the result
// per transaction is returned in the validator's order of checks: the
// verified-signature set the unchanged validator then consults.
//
// Wire decoding restates google.golang.org/protobuf v1.30.0 (vendored; the
// runtime behind github.com/golang/protobuf v1.5.3 and fabric-protos-go
// v0.3.1) internal/impl/decode.go unmarshalPointer + encoding/protowire:
//   * tag: varint; field number in [1, 2^29-1]; wire type 4 (end group) at
//     message level is an error; wire types 6 and 7 are errors;
//   * a known field arriving with another wire type is an UNKNOWN field (kept,
//     no error); unknown fields are consumed by ConsumeFieldValue (groups
//     nest, end-group number must match);
//   * varint: at most 10 bytes, the 10th <= 1; lengths past the end: error;
//   * singular bytes / scalars: last occurrence wins; singular message fields
//     MERGE across occurrences; repeated fields append;
//   * proto3 `string` fields are UTF-8 validated (unicode/utf8.Valid) -- an
//     invalid string fails the whole Unmarshal.
// Identities: msp/mspimpl.go:398-422 deserializeIdentityInternal (pem.Decode,
// x509.ParseCertificate, key import) is restated far enough to get the P-256
// public key; an identity this code cannot resolve is reported as such and
// left to the Go path (the verified set never claims what it did not check).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/bdls_hip.h"
#include "bh_common.h"
#include "der.h"

namespace bh {
int host_fail(int code, const char* msg);
}

namespace {

// ---------------------------------------------------------------- protobuf-go
struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
  bool set = false;  // Go: non-nil slice
};

constexpr uint64_t kMaxField = (1ull << 29) - 1;  // protowire.MaxValidNumber

// protowire.ConsumeVarint: bytes consumed, or 0 on error
size_t pb_varint(const uint8_t* b, size_t n, uint64_t* v) {
  uint64_t x = 0;
  for (size_t i = 0; i < 10; i++) {
    if (i >= n) return 0;                   // errCodeTruncated
    const uint64_t y = b[i];
    if (i == 9) {
      if (y > 1) return 0;                  // errCodeOverflow
      *v = x | (y << 63);
      return 10;
    }
    x |= (y & 0x7f) << (7 * i);
    if (y < 0x80) {
      *v = x;
      return i + 1;
    }
  }
  return 0;
}

// protowire.consumeFieldValueD: bytes consumed by the value of a field with
// wire type `typ` (and number `num` for groups), or 0 on error (a valid value
// always consumes >= 1 byte: a bytes value has its length varint).
size_t pb_field_value(uint64_t num, uint32_t typ, const uint8_t* b, size_t n, int depth) {
  uint64_t v;
  switch (typ) {
    case 0:
      return pb_varint(b, n, &v);
    case 1:
      return n >= 8 ? 8 : 0;
    case 5:
      return n >= 4 ? 4 : 0;
    case 2: {
      const size_t k = pb_varint(b, n, &v);
      if (!k || v > n - k) return 0;
      return k + (size_t)v;
    }
    case 3: {
      if (depth < 0) return 0;  // errCodeRecursionDepth
      size_t i = 0;
      for (;;) {
        uint64_t tag;
        const size_t k = pb_varint(b + i, n - i, &tag);
        if (!k) return 0;
        const uint64_t num2 = tag >> 3;
        if (num2 > 0x7fffffffull || num2 < 1) return 0;  // DecodeTag -1 / < MinValidNumber
        i += k;
        const uint32_t typ2 = (uint32_t)(tag & 7);
        if (typ2 == 4) return num2 == num ? i : 0;
        const size_t m = pb_field_value(num2, typ2, b + i, n - i, depth - 1);
        if (!m) return 0;
        i += m;
      }
    }
    default:  // 4: errCodeEndGroup, 6/7: errCodeReserved
      return 0;
  }
}

// One decoded field of a message.
struct Field {
  uint64_t num;
  uint32_t typ;
  uint64_t v;  // varint value (typ 0)
  Span s;      // bytes value (typ 2)
};

// Walks the fields of a message in order; `on` returns false to fail the
// Unmarshal (a known field's own error). Returns false on a wire error.
template <class F>
bool pb_walk(const uint8_t* b, size_t n, F&& on) {
  size_t i = 0;
  while (i < n) {
    uint64_t tag;
    const size_t k = pb_varint(b + i, n - i, &tag);
    if (!k) return false;
    i += k;
    const uint64_t num = tag >> 3;
    if (num < 1 || num > kMaxField) return false;
    const uint32_t typ = (uint32_t)(tag & 7);
    if (typ == 4) return false;  // end group without a group (groupTag 0)
    Field f{num, typ, 0, {}};
    size_t m;
    if (typ == 0) {
      m = pb_varint(b + i, n - i, &f.v);
    } else if (typ == 2) {
      uint64_t len;
      const size_t h = pb_varint(b + i, n - i, &len);
      if (!h || len > n - i - h) return false;
      f.s = Span{b + i + h, (size_t)len, true};
      m = h + (size_t)len;
    } else {
      m = pb_field_value(num, typ, b + i, n - i, 10000);
    }
    if (!m) return false;
    i += m;
    if (!on(f)) return false;
  }
  return true;
}

// unicode/utf8.Valid
bool utf8_valid(const uint8_t* p, size_t n) {
  size_t i = 0;
  while (i < n) {
    const uint8_t c = p[i];
    if (c < 0x80) {
      i++;
      continue;
    }
    size_t len;
    uint8_t lo = 0x80, hi = 0xbf;
    if (c >= 0xc2 && c <= 0xdf) len = 2;
    else if (c == 0xe0) { len = 3; lo = 0xa0; }
    else if (c >= 0xe1 && c <= 0xec) len = 3;
    else if (c == 0xed) { len = 3; hi = 0x9f; }
    else if (c >= 0xee && c <= 0xef) len = 3;
    else if (c == 0xf0) { len = 4; lo = 0x90; }
    else if (c >= 0xf1 && c <= 0xf3) len = 4;
    else if (c == 0xf4) { len = 4; hi = 0x8f; }
    else return false;
    if (i + len > n) return false;
    if (p[i + 1] < lo || p[i + 1] > hi) return false;
    for (size_t k = 2; k < len; k++)
      if (p[i + k] < 0x80 || p[i + k] > 0xbf) return false;
    i += len;
  }
  return true;
}

// field helpers: true if the field was this one and consumed (or failed)
inline bool is_bytes(const Field& f, uint64_t num) { return f.num == num && f.typ == 2; }
inline bool is_varint(const Field& f, uint64_t num) { return f.num == num && f.typ == 0; }

// ---- messages on the validation path (fabric-protos-go v0.3.1) ----
struct Envelope {  // common.Envelope
  Span payload, signature;
};
bool dec_envelope(Span in, Envelope* o) {
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_bytes(f, 1)) o->payload = f.s;
    else if (is_bytes(f, 2)) o->signature = f.s;
    return true;
  });
}

struct Header {  // common.Header
  Span channel_header, signature_header;
};
bool dec_header_into(Span in, Header* o) {  // merges into *o
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_bytes(f, 1)) o->channel_header = f.s;
    else if (is_bytes(f, 2)) o->signature_header = f.s;
    return true;
  });
}

struct Payload {  // common.Payload
  bool has_header = false;
  Header header;
  Span data;
};
bool dec_payload(Span in, Payload* o) {
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_bytes(f, 1)) {
      o->has_header = true;
      return dec_header_into(f.s, &o->header);
    }
    if (is_bytes(f, 2)) o->data = f.s;
    return true;
  });
}

bool dec_timestamp(Span in) {  // google.protobuf.Timestamp: only wire errors matter
  return pb_walk(in.p, in.n, [&](const Field&) { return true; });
}

struct ChannelHeader {  // common.ChannelHeader
  int32_t type = 0;
  uint64_t epoch = 0;
  Span channel_id, tx_id;
};
bool dec_channel_header(Span in, ChannelHeader* o) {
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_varint(f, 1)) o->type = (int32_t)f.v;
    else if (is_bytes(f, 3)) return dec_timestamp(f.s);
    else if (is_bytes(f, 4)) { o->channel_id = f.s; return utf8_valid(f.s.p, f.s.n); }
    else if (is_bytes(f, 5)) { o->tx_id = f.s; return utf8_valid(f.s.p, f.s.n); }
    else if (is_varint(f, 6)) o->epoch = f.v;
    return true;  // 2 version (int32), 7 extension, 8 tls_cert_hash: no checks
  });
}

struct SignatureHeader {  // common.SignatureHeader
  Span creator, nonce;
};
bool dec_signature_header(Span in, SignatureHeader* o) {
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_bytes(f, 1)) o->creator = f.s;
    else if (is_bytes(f, 2)) o->nonce = f.s;
    return true;
  });
}

struct TxAction {  // peer.TransactionAction
  Span header, payload;
};
bool dec_transaction(Span in, std::vector<TxAction>* acts) {  // peer.Transaction
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (!is_bytes(f, 1)) return true;
    TxAction a;
    bool ok = pb_walk(f.s.p, f.s.n, [&](const Field& g) {
      if (is_bytes(g, 1)) a.header = g.s;
      else if (is_bytes(g, 2)) a.payload = g.s;
      return true;
    });
    acts->push_back(a);
    return ok;
  });
}

struct Endorsement {  // peer.Endorsement
  Span endorser, signature;
};
struct EndorsedAction {  // peer.ChaincodeEndorsedAction
  Span prp;
  std::vector<Endorsement> endorsements;
};
bool dec_endorsed_action_into(Span in, EndorsedAction* o) {
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_bytes(f, 1)) {
      o->prp = f.s;
    } else if (is_bytes(f, 2)) {
      Endorsement e;
      bool ok = pb_walk(f.s.p, f.s.n, [&](const Field& g) {
        if (is_bytes(g, 1)) e.endorser = g.s;
        else if (is_bytes(g, 2)) e.signature = g.s;
        return true;
      });
      o->endorsements.push_back(e);
      return ok;
    }
    return true;
  });
}

struct ActionPayload {  // peer.ChaincodeActionPayload
  Span ccpp;
  bool has_action = false;
  EndorsedAction action;
};
bool dec_action_payload(Span in, ActionPayload* o) {
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_bytes(f, 1)) o->ccpp = f.s;
    else if (is_bytes(f, 2)) {
      o->has_action = true;
      return dec_endorsed_action_into(f.s, &o->action);
    }
    return true;
  });
}

bool dec_prp(Span in) {  // peer.ProposalResponsePayload: bytes fields only
  return pb_walk(in.p, in.n, [&](const Field&) { return true; });
}

struct SerializedIdentity {  // msp.SerializedIdentity
  Span mspid, id_bytes;
};
bool dec_serialized_identity(Span in, SerializedIdentity* o) {
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_bytes(f, 1)) { o->mspid = f.s; return utf8_valid(f.s.p, f.s.n); }
    if (is_bytes(f, 2)) o->id_bytes = f.s;
    return true;
  });
}

bool dec_block(Span in, std::vector<Span>* data) {  // common.Block -> BlockData.data
  return pb_walk(in.p, in.n, [&](const Field& f) {
    if (is_bytes(f, 1)) {  // BlockHeader
      return pb_walk(f.s.p, f.s.n, [&](const Field&) { return true; });
    }
    if (is_bytes(f, 2)) {  // BlockData (merges: entries append)
      return pb_walk(f.s.p, f.s.n, [&](const Field& g) {
        if (is_bytes(g, 1)) data->push_back(g.s);
        return true;
      });
    }
    if (is_bytes(f, 3)) {  // BlockMetadata
      return pb_walk(f.s.p, f.s.n, [&](const Field&) { return true; });
    }
    return true;
  });
}

// ---------------------------------------------------------------- PEM
// Restates Go encoding/pem Decode (first block; type not checked by the MSP,
// msp/mspimpl.go:400). Returns false when Go returns a nil block.
size_t find(const uint8_t* d, size_t n, const char* pat, size_t from = 0) {
  const size_t m = strlen(pat);
  if (m > n) return SIZE_MAX;
  for (size_t i = from; i + m <= n; i++)
    if (!memcmp(d + i, pat, m)) return i;
  return SIZE_MAX;
}

// getLine: first \n (or \r\n) delimited line, trailing spaces/tabs trimmed
void get_line(const uint8_t* d, size_t n, size_t* line_len, size_t* rest_off) {
  size_t i = 0;
  while (i < n && d[i] != '\n') i++;
  size_t j;
  if (i == n) {
    j = n;
  } else {
    j = i + 1;
    if (i > 0 && d[i - 1] == '\r') i--;
  }
  while (i > 0 && (d[i - 1] == ' ' || d[i - 1] == '\t')) i--;
  *line_len = i;
  *rest_off = j;
}

int b64val(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

// base64.StdEncoding.Decode with \r and \n ignored (padding required).
bool b64_decode(const std::vector<uint8_t>& in, std::vector<uint8_t>* out) {
  std::vector<uint8_t> c;
  c.reserve(in.size());
  for (uint8_t x : in)
    if (x != '\r' && x != '\n') c.push_back(x);
  if (c.size() % 4) return false;
  out->clear();
  for (size_t q = 0; q < c.size(); q += 4) {
    const bool last = q + 4 == c.size();
    int v[4];
    int pad = 0;
    for (int k = 0; k < 4; k++) {
      if (c[q + k] == '=') {
        if (!last || k < 2) return false;
        pad++;
        v[k] = 0;
        continue;
      }
      if (pad) return false;  // data after padding
      v[k] = b64val(c[q + k]);
      if (v[k] < 0) return false;
    }
    const uint32_t w = (uint32_t)v[0] << 18 | (uint32_t)v[1] << 12 | (uint32_t)v[2] << 6 | (uint32_t)v[3];
    out->push_back((uint8_t)(w >> 16));
    if (pad < 2) out->push_back((uint8_t)(w >> 8));
    if (pad < 1) out->push_back((uint8_t)w);
  }
  return true;
}

bool pem_decode(const uint8_t* data, size_t n, std::vector<uint8_t>* der) {
  static const char kStart[] = "\n-----BEGIN ";
  static const char kEnd[] = "\n-----END ";
  size_t rest = 0;  // offset of `rest` in data
  for (;;) {
    if (n - rest >= 11 && !memcmp(data + rest, kStart + 1, 11)) {
      rest += 11;
    } else {
      const size_t at = find(data, n, kStart, rest);
      if (at == SIZE_MAX) return false;
      rest = at + 12;
    }
    size_t ll, ro;
    get_line(data + rest, n - rest, &ll, &ro);
    const uint8_t* type_line = data + rest;
    if (ll < 5 || memcmp(type_line + ll - 5, "-----", 5)) {
      rest += ro;
      continue;
    }
    const size_t tlen = ll - 5;
    rest += ro;
    int headers = 0;
    for (;;) {
      if (rest >= n) return false;
      get_line(data + rest, n - rest, &ll, &ro);
      const uint8_t* colon = (const uint8_t*)memchr(data + rest, ':', ll);
      if (!colon) break;
      headers++;  // (a repeated key still counts; the MSP's PEMs carry none)
      rest += ro;
    }
    size_t end_idx, trailer;
    if (headers == 0 && n - rest >= 9 && !memcmp(data + rest, kEnd + 1, 9)) {
      end_idx = rest;
      trailer = rest + 9;
    } else {
      end_idx = find(data, n, kEnd, rest);
      if (end_idx == SIZE_MAX) continue;  // Go: continue (searches again from rest)
      trailer = end_idx + 10;
    }
    const size_t tl = tlen + 5;
    if (n - trailer < tl) continue;
    if (memcmp(data + trailer, type_line, tlen) || memcmp(data + trailer + tlen, "-----", 5))
      continue;
    get_line(data + trailer + tl, n - trailer - tl, &ll, &ro);
    if (ll != 0) continue;
    std::vector<uint8_t> b64;
    for (size_t i = rest; i < end_idx; i++)
      if (data[i] != ' ' && data[i] != '\t') b64.push_back(data[i]);
    if (!b64_decode(b64, der)) continue;
    return true;
  }
}

// ---------------------------------------------------------------- X.509
// Minimal DER walk to the subject public key (RFC 5280 Certificate ->
// tbsCertificate -> subjectPublicKeyInfo) and the certificate signature.
struct Tlv {
  uint8_t tag;
  const uint8_t* p;  // content
  size_t n;
  const uint8_t* raw;  // whole TLV
  size_t raw_n;
};

bool tlv(const uint8_t* b, size_t n, size_t* off, Tlv* t) {
  if (*off >= n) return false;
  const size_t start = *off;
  t->tag = b[(*off)++];
  if ((t->tag & 0x1f) == 0x1f) return false;
  if (*off >= n) return false;
  size_t len = b[(*off)++];
  if (len & 0x80) {
    const size_t k = len & 0x7f;
    if (k == 0 || k > 4 || *off + k > n) return false;
    len = 0;
    for (size_t i = 0; i < k; i++) len = len << 8 | b[(*off)++];
    if (len < 0x80 || (k > 1 && (len >> ((k - 1) * 8)) == 0)) return false;  // non-minimal
  }
  if (len > n - *off) return false;
  t->p = b + *off;
  t->n = len;
  t->raw = b + start;
  t->raw_n = *off + len - start;
  *off += len;
  return true;
}

const uint8_t kOidEcPub[] = {0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02, 0x01};
const uint8_t kOidP256[] = {0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07};
const uint8_t kOidEcdsaSha256[] = {0x2a, 0x86, 0x48, 0xce, 0x3d, 0x04, 0x03, 0x02};

struct Cert {
  Tlv tbs;               // tbsCertificate (raw = the signed bytes)
  uint8_t pub[64];       // subject P-256 key X || Y
  bool p256 = false;
  Tlv sig_alg_oid;       // outer signatureAlgorithm OID
  Tlv sig;               // signatureValue BIT STRING content (after the unused-bits byte)
  bool has_sig = false;
};

bool parse_cert(const uint8_t* d, size_t n, Cert* c) {
  size_t off = 0;
  Tlv cert;
  if (!tlv(d, n, &off, &cert) || cert.tag != 0x30 || off != n) return false;
  size_t o = 0;
  if (!tlv(cert.p, cert.n, &o, &c->tbs) || c->tbs.tag != 0x30) return false;
  Tlv alg, sv;
  if (!tlv(cert.p, cert.n, &o, &alg) || alg.tag != 0x30) return false;
  if (!tlv(cert.p, cert.n, &o, &sv) || sv.tag != 0x03 || sv.n < 1 || sv.p[0] != 0) return false;
  size_t ao = 0;
  if (!tlv(alg.p, alg.n, &ao, &c->sig_alg_oid) || c->sig_alg_oid.tag != 0x06) return false;
  c->sig = Tlv{0x03, sv.p + 1, sv.n - 1, sv.raw, sv.raw_n};
  c->has_sig = true;
  // tbs: [0] version?, serial, signature, issuer, validity, subject, spki
  size_t t = 0;
  Tlv f;
  if (!tlv(c->tbs.p, c->tbs.n, &t, &f)) return false;
  if (f.tag == 0xa0 && !tlv(c->tbs.p, c->tbs.n, &t, &f)) return false;  // then serial
  if (f.tag != 0x02) return false;
  for (int k = 0; k < 4; k++)  // signature, issuer, validity, subject
    if (!tlv(c->tbs.p, c->tbs.n, &t, &f) || f.tag != 0x30) return false;
  Tlv spki;
  if (!tlv(c->tbs.p, c->tbs.n, &t, &spki) || spki.tag != 0x30) return false;
  size_t s = 0;
  Tlv algid, bits;
  if (!tlv(spki.p, spki.n, &s, &algid) || algid.tag != 0x30) return false;
  if (!tlv(spki.p, spki.n, &s, &bits) || bits.tag != 0x03 || s != spki.n) return false;
  size_t a = 0;
  Tlv oid1, oid2;
  if (!tlv(algid.p, algid.n, &a, &oid1) || oid1.tag != 0x06) return false;
  if (!tlv(algid.p, algid.n, &a, &oid2)) return false;
  c->p256 = oid1.n == sizeof(kOidEcPub) && !memcmp(oid1.p, kOidEcPub, sizeof(kOidEcPub)) &&
            oid2.tag == 0x06 && oid2.n == sizeof(kOidP256) &&
            !memcmp(oid2.p, kOidP256, sizeof(kOidP256)) && a == algid.n && bits.n == 66 &&
            bits.p[0] == 0 && bits.p[1] == 0x04;
  if (c->p256) memcpy(c->pub, bits.p + 2, 64);
  return true;
}

// ---------------------------------------------------------------- identities
// SerializedIdentity bytes -> resolved P-256 key + the identity key used by
// SignatureSetToValidIdentities' de-duplication (Mspid + Id, where Id hashes
// the SANITIZED certificate: newIdentity, msp/identities.go:55-85 ->
// sanitizeCert, msp/mspimpl.go:892-935 -> sanitizeECDSASignedCert,
// msp/cert.go:76-116, which rewrites the certificate signature's S to low-S
// with the ISSUER's curve order). Here: mspid || tbs || r. For a given TBS and
// r, the only signatures Go's chain validation can accept are (r, s) and its
// twin (r, n_issuer - s), which sanitize to the same certificate, so dropping
// s gives Go's equivalence without knowing the issuer's curve (a P-384 CA's
// twins included). A signature that does not parse keeps its raw bytes.
//
// What this cannot see: Go's DeserializeIdentity also builds the certificate
// chain to the MSP's roots (getUniqueValidationChain) and rejects identities
// that do not chain, are revoked, or fail the OU rules. Those identities are
// resolved here, so valid_endorsers / valid_identities are UPPER BOUNDS of
// what Go's policy evaluation receives: informational counts that must not
// decide a policy on their own (the unchanged Go evaluation consults the
// per-signature results).
struct Ident {
  bool ok = false;
  uint8_t pub[64];
  std::string key;
  uint64_t key_id = 0;  // interned key (IdentCache): equal keys <=> equal ids
};

// r's magnitude (big-endian, no leading zeros, any size) of a signature that
// Go's asn1 parses with r, s > 0; false otherwise.
bool sig_r_bytes(const uint8_t* b, size_t n, std::string* out) {
  bh::DerSig ds;
  if (n > 0xffffffffu || bh::der_parse_sig(b, (uint32_t)n, &ds) != bh::R_OK) return false;
  uint32_t off = 0, cls, cmp, tag, len, io = 0, rl;
  if (bh::der_tag_len(b, (uint32_t)n, &off, &cls, &cmp, &tag, &len)) return false;
  const uint8_t* in = b + off;
  if (bh::der_tag_len(in, len, &io, &cls, &cmp, &tag, &rl)) return false;
  const uint8_t* p = in + io;
  while (rl > 1 && *p == 0) {
    p++;
    rl--;
  }
  out->assign((const char*)p, rl);
  return true;
}

std::string dedupe_key(const Span& mspid, const Cert& c) {
  std::string k((const char*)mspid.p, mspid.n);
  k.push_back('\0');
  k.append((const char*)c.tbs.raw, c.tbs.raw_n);
  std::string r;
  if (c.has_sig && sig_r_bytes(c.sig.p, c.sig.n, &r)) {
    k.push_back((char)(r.size() >> 8));
    k.push_back((char)(r.size() & 0xff));
    k.append(r);
  } else if (c.has_sig) {
    k.push_back('\xff');
    k.push_back('\xff');
    k.append((const char*)c.sig.p, c.sig.n);
  }
  return k;
}

Ident resolve(Span ser) {
  Ident id;
  SerializedIdentity si;
  if (!dec_serialized_identity(ser, &si)) return id;
  std::vector<uint8_t> der;
  if (!si.id_bytes.set || !pem_decode(si.id_bytes.p, si.id_bytes.n, &der)) return id;
  Cert c;
  if (!parse_cert(der.data(), der.size(), &c) || !c.p256) return id;
  id.ok = true;
  memcpy(id.pub, c.pub, 64);
  id.key = dedupe_key(si.mspid, c);
  return id;
}

// Long-lived cache of resolved identities (the device-side twin of the MSP's
// deserializer cache, msp/cache/cache.go): serialized bytes -> Ident.
using IdentP = std::shared_ptr<const Ident>;

// 64-bit hash of a byte span (8 bytes per step, no copy): identities are
// ~0.9 KB PEM certificates looked up twice or more per transaction.
uint64_t span_hash(const uint8_t* p, size_t n) {
  // Serialized identities are ~1 KB PEM certificates that share long
  // prefixes: hash the length and 16 words spread over the span (the tail
  // holds the certificate signature) instead of a serial multiply chain over
  // every byte (4 lookups per transaction made that half the block decode).
  // Every hit is confirmed by a full compare, so this only spreads buckets.
  uint64_t h = 0x9e3779b97f4a7c15ull ^ n;
  if (n < 8) {
    uint64_t v = 0;
    memcpy(&v, p, n);
    h = (h ^ v) * 0xc4ceb9fe1a85ec53ull;
    return h ^ (h >> 29);
  }
  const size_t step = n <= 128 ? 8 : (n - 8) / 15;
  const size_t cnt = n <= 128 ? (n - 8) / 8 + 1 : 16;
  for (size_t k = 0; k < cnt; k++) {
    uint64_t v;
    memcpy(&v, p + (k == cnt - 1 ? n - 8 : k * step), 8);
    h = (h ^ v) * 0xff51afd7ed558ccdull;
    h ^= h >> 32;
  }
  return h ^ (h >> 29);
}

struct IdentEntry {
  std::string bytes;  // the serialized identity (full compare on every hit)
  IdentP id;
};

// Long-lived cache of resolved identities (the device-side twin of the MSP's
// deserializer cache, msp/cache/cache.go): serialized bytes -> Ident. Callers
// hold one Session for a whole block / batch: one lock, no copies on a hit.
// Dedup keys are interned to integers (Ident::key_id), so the signature-set
// replay compares ids instead of ~1 KB strings. Both maps are only cleared
// when a session starts (never in the middle of one), so the identities one
// call resolves always agree on their ids.
struct IdentCache {
  std::mutex mu;
  std::unordered_multimap<uint64_t, IdentEntry> m;
  std::unordered_map<std::string, uint64_t> keys;
  uint64_t next_key = 1;
  static constexpr size_t kCap = 1 << 16;
  struct Session {
    IdentCache& c;
    std::lock_guard<std::mutex> g;
    explicit Session(IdentCache& cc) : c(cc), g(cc.mu) {
      if (c.m.size() >= kCap || c.keys.size() >= kCap) {
        c.m.clear();
        c.keys.clear();
      }
    }
    IdentP get(Span ser) {
      const uint64_t h = span_hash(ser.p, ser.n);
      auto r = c.m.equal_range(h);
      for (auto it = r.first; it != r.second; ++it)
        if (it->second.bytes.size() == ser.n && !memcmp(it->second.bytes.data(), ser.p, ser.n))
          return it->second.id;
      Ident id = resolve(ser);
      if (id.ok) {
        auto k = c.keys.emplace(id.key, c.next_key);
        if (k.second) c.next_key++;
        id.key_id = k.first->second;
      }
      IdentP p = std::make_shared<const Ident>(std::move(id));
      c.m.emplace(h, IdentEntry{std::string((const char*)ser.p, ser.n), p});
      return p;
    }
  };
};

IdentCache& ident_cache() {
  static IdentCache* c = new IdentCache();
  return *c;
}

// ---------------------------------------------------------------- signature sets
// One SignedData (protoutil/signeddata.go:25-29): the signer's identity, the
// signed bytes (up to three pieces, concatenated) and the signature.
struct SdEntry {
  IdentP id;  // resolved identity (id->ok false: DeserializeIdentity fails)
  Span id_ser;  // serialized identity (block decode resolves it after parsing)
  Span seg[3];
  int nseg = 0;
  Span sig;
  uint8_t out = BH_SP_NOT_VERIFIED;
};

// One device batch of signatures (messages hashed on the device). With `base`
// set (a serialized block), signatures and the one or two message spans of
// every record index that buffer directly (bh_verify_2seg): no host copy of
// the signed bytes, and one upload of the block instead of their
// concatenation. Otherwise pieces are concatenated into `msg` / `sig`.
struct Batch {
  const uint8_t* base = nullptr;
  size_t base_len = 0;
  std::vector<uint8_t> pub, sig, msg;
  std::vector<uint64_t> sig_off, msg_off, msg2_off;
  std::vector<uint32_t> sig_len, msg_len, msg2_len;
  std::vector<uint8_t*> dst;  // where each record's reason goes
  uint64_t rel(Span x) const {  // offset of a span inside base (empty spans: 0)
    return x.n ? (uint64_t)(x.p - base) : 0u;
  }
  bool inside(Span x) const { return !x.n || (x.p >= base && x.p + x.n <= base + base_len); }
  void add(const uint8_t pub64[64], Span s, const Span* m, int nm, uint8_t* out) {
    pub.insert(pub.end(), pub64, pub64 + 64);
    dst.push_back(out);
    if (base) {  // every span of a block's SignedData lies in the block
      sig_off.push_back(rel(s));
      sig_len.push_back((uint32_t)s.n);
      msg_off.push_back(nm > 0 ? rel(m[0]) : 0u);
      msg_len.push_back(nm > 0 ? (uint32_t)m[0].n : 0u);
      msg2_off.push_back(nm > 1 ? rel(m[1]) : 0u);
      msg2_len.push_back(nm > 1 ? (uint32_t)m[1].n : 0u);
      return;
    }
    sig_off.push_back(sig.size());
    sig_len.push_back((uint32_t)s.n);
    if (s.n) sig.insert(sig.end(), s.p, s.p + s.n);
    msg_off.push_back(msg.size());
    size_t L = 0;
    for (int k = 0; k < nm; k++) {
      if (m[k].n) msg.insert(msg.end(), m[k].p, m[k].p + m[k].n);
      L += m[k].n;
    }
    msg_len.push_back((uint32_t)L);
  }
  // zero-copy needs every span inside base and at most two message pieces
  bool fits(const SdEntry& e) const {
    bool ok = e.nseg <= 2 && inside(e.sig);
    for (int k = 0; k < e.nseg; k++) ok = ok && inside(e.seg[k]);
    return ok;
  }
  void add(SdEntry& e) { add(e.id->pub, e.sig, e.seg, e.nseg, &e.out); }
  void reserve(size_t n, size_t msg_bytes, size_t sig_bytes) {
    pub.reserve(64 * n);
    sig_off.reserve(n);
    sig_len.reserve(n);
    msg_off.reserve(n);
    msg_len.reserve(n);
    dst.reserve(n);
    if (base) {
      msg2_off.reserve(n);
      msg2_len.reserve(n);
    } else {
      msg.reserve(msg_bytes + 1);
      sig.reserve(sig_bytes + 1);
    }
  }
  size_t size() const { return dst.size(); }
  int run(uint32_t flags) {
    const size_t n = size();
    if (!n) return BH_OK;
    std::vector<uint8_t> bitmap((n + 7) / 8), reason(n);
    int rc;
    if (base) {
      bh_batch b{pub.data(), base, sig_off.data(), sig_len.data(),
                 base, msg_off.data(), msg_len.data()};
      rc = bh_verify_2seg(BH_CURVE_P256, &b, msg2_off.data(), msg2_len.data(), n, flags,
                          bitmap.data(), reason.data());
    } else {
      sig.push_back(0);
      msg.push_back(0);
      bh_batch b{pub.data(), sig.data(), sig_off.data(), sig_len.data(),
                 msg.data(), msg_off.data(), msg_len.data()};
      rc = bh_verify(BH_CURVE_P256, &b, n, flags, bitmap.data(), reason.data());
    }
    if (rc) return rc;
    for (size_t i = 0; i < n; i++) *dst[i] = reason[i];
    return BH_OK;
  }
};

struct SetRange {
  size_t first, count;
};

// common/policies/policy.go:363-395 SignatureSetToValidIdentities over each
// set, batched: round 1 verifies the first entry of every identity of every
// set (plus `extra`, e.g. creator signatures, in the same device batch). Go
// checks a later entry of an identity only while no earlier one verified, so
// round 2 verifies -- speculatively, in ONE more device batch -- every later
// entry of the identities whose first entry failed (rare: a signer repeating
// itself after a bad signature); the in-order replay then marks the entries
// Go skips as duplicates (an identity already validated earlier in the set).
// At most two device passes, however the duplicates are arranged. Entries
// whose identity does not resolve are skipped, as Go skips them.
int verify_sets(std::vector<SdEntry>& e, const std::vector<SetRange>& sets, uint32_t vflags,
                bool decode_only, std::vector<uint32_t>* valid, Batch* extra) {
  Batch b;
  if (extra) b = std::move(*extra);
  if (b.base)  // a record that does not index the block goes the copying way
    for (const SdEntry& x : e)
      if (x.id && x.id->ok && !b.fits(x))
        return bh::host_fail(BH_E_INVALID, "span outside the block");
  {
    size_t bytes = 0, sig_bytes = 0;
    for (const SdEntry& x : e) {
      for (int k = 0; k < x.nseg; k++) bytes += x.seg[k].n;
      sig_bytes += x.sig.n;
    }
    b.reserve(b.size() + e.size(), b.msg.size() + bytes, b.sig.size() + sig_bytes);
  }
  std::vector<uint64_t> seen, failed;
  for (const SetRange& r : sets) {
    seen.clear();
    for (size_t i = r.first; i < r.first + r.count; i++) {
      SdEntry& x = e[i];
      if (!x.id || !x.id->ok) {
        x.out = BH_FAB_E_BAD_IDENTITY;
        continue;
      }
      if (std::find(seen.begin(), seen.end(), x.id->key_id) != seen.end()) continue;
      seen.push_back(x.id->key_id);
      b.add(x);
    }
  }
  if (!decode_only) {
    if (int rc = b.run(vflags)) return rc;
    Batch more;
    more.base = b.base;
    more.base_len = b.base_len;
    for (const SetRange& r : sets) {
      failed.clear();  // identities whose round-1 entry failed
      for (size_t i = r.first; i < r.first + r.count; i++) {
        SdEntry& x = e[i];
        if (!x.id || !x.id->ok) continue;
        if (x.out != BH_SP_NOT_VERIFIED) {
          if (x.out != BH_R_OK) failed.push_back(x.id->key_id);
        } else if (std::find(failed.begin(), failed.end(), x.id->key_id) != failed.end()) {
          more.add(x);
        }
      }
    }
    if (int rc = more.run(vflags)) return rc;
  }
  valid->assign(sets.size(), 0);
  std::vector<uint64_t> ok;
  for (size_t k = 0; k < sets.size(); k++) {
    const SetRange& r = sets[k];
    ok.clear();
    for (size_t i = r.first; i < r.first + r.count; i++) {
      SdEntry& x = e[i];
      if (!x.id || !x.id->ok) continue;
      if (std::find(ok.begin(), ok.end(), x.id->key_id) != ok.end()) {
        x.out = BH_FAB_E_DUPLICATE;  // Go skips it (verified speculatively or not at all)
        continue;
      }
      if (x.out == BH_R_OK) ok.push_back(x.id->key_id);
    }
    (*valid)[k] = (uint32_t)ok.size();
  }
  return BH_OK;
}

uint32_t verify_flags(uint32_t flags) {
  return ((flags & BH_FAB_F_SHA3) ? BH_F_HASH_SHA3_256 : BH_F_HASH_SHA256) |
         ((flags & BH_FAB_F_KEEP_KEYS) ? BH_F_KEEP_KEYS : 0u);
}

// ---------------------------------------------------------------- the block
struct TxRec {
  int32_t status = BH_FAB_OK;
  int32_t type = 0;
  bool creator_check = false;  // creator signature goes to the device
  bool resolve_creator = false;  // creator identity still to be resolved
  int32_t post_status = BH_FAB_OK;  // status if the creator identity resolves
  Span creator_ser;
  IdentP creator;
  Span payload, signature;
  uint8_t creator_out = BH_SP_NOT_VERIFIED;
  size_t end_first = 0, end_count = 0;  // endorsements in the shared entry list
};

// Go's order of checks up to the signatures (validateTx, ValidateTransaction,
// validateEndorserTransaction). Checks that do not gate which signatures are
// verified (CheckTxID, the proposal hash, ledger / channel state) are left to
// the unchanged validator. Pure parsing (no identity lookups), so transactions
// decode in parallel; resolve_tx then applies the identity outcomes.
void decode_tx(Span env_bytes, TxRec* t, std::vector<SdEntry>* ends) {
  t->end_first = ends->size();
  Envelope env;
  if (!dec_envelope(env_bytes, &env)) {
    t->status = BH_FAB_ENVELOPE;  // GetEnvelopeFromBlock: INVALID_OTHER_REASON
    return;
  }
  Payload pl;
  if (!dec_payload(env.payload, &pl)) {
    t->status = BH_FAB_PAYLOAD;  // BAD_PAYLOAD
    return;
  }
  ChannelHeader ch;
  SignatureHeader sh;
  // validateCommonHeader: nil header, unmarshal ChannelHeader, SignatureHeader,
  // validateChannelHeader (type, epoch), validateSignatureHeader (nonce, creator)
  if (!pl.has_header || !dec_channel_header(pl.header.channel_header, &ch) ||
      !dec_signature_header(pl.header.signature_header, &sh) ||
      !(ch.type == 1 || ch.type == 2 || ch.type == 3) || ch.epoch != 0 || sh.nonce.n == 0 ||
      sh.creator.n == 0) {
    t->status = BH_FAB_HEADER;  // BAD_COMMON_HEADER
    return;
  }
  t->type = ch.type;
  // checkSignatureFromCreator: nil arguments, then DeserializeIdentity (in
  // resolve_tx: BH_FAB_CREATOR_IDENTITY overrides everything below), Verify
  t->payload = env.payload;
  t->signature = env.signature;
  if (!env.signature.set || !env.payload.set) {
    t->status = BH_FAB_CREATOR_SIGNATURE;  // "nil arguments"
  } else {
    t->creator_ser = sh.creator;
    t->resolve_creator = true;
  }
  if (ch.type == 2) {  // CONFIG_UPDATE: UNSUPPORTED_TX_PAYLOAD after the creator check
    t->post_status = BH_FAB_UNSUPPORTED;
    return;
  }
  if (ch.type != 3) return;  // CONFIG: no endorsements
  // validateEndorserTransaction structure (reached only if the creator check
  // passes; decoded regardless, so the endorsements ride in the same batch)
  std::vector<TxAction> acts;
  int32_t tx_status = BH_FAB_OK;
  ActionPayload ap;
  if (!dec_transaction(pl.data, &acts) || acts.size() != 1) {
    tx_status = BH_FAB_TX;
  } else {
    SignatureHeader ash;
    if (!dec_signature_header(acts[0].header, &ash) || ash.nonce.n == 0 || ash.creator.n == 0 ||
        !dec_action_payload(acts[0].payload, &ap) ||
        !ap.has_action /* Go dereferences a nil Action here */ ||
        !dec_prp(ap.action.prp))
      tx_status = BH_FAB_TX;
  }
  if (tx_status != BH_FAB_OK) {
    t->post_status = tx_status;
    return;
  }
  for (const Endorsement& en : ap.action.endorsements) {
    // SignedData{data: prp || endorser, identity: endorser, signature}
    // (validator_keylevel.go:246-260)
    SdEntry x;
    x.id_ser = en.endorser;
    x.seg[0] = ap.action.prp;
    x.seg[1] = en.endorser;
    x.nseg = 2;
    x.sig = en.signature;
    ends->push_back(x);
  }
  t->end_count = ends->size() - t->end_first;
}

// The sequential half of decode_tx: identities (the long-lived cache, through
// a per-block memo: a block repeats a few identities thousands of times).
// With `mu` set, several memos (one per decode chunk) share the session:
// their misses -- a block's few distinct identities per chunk -- go through it
// one at a time.
struct IdentMemo {
  IdentCache::Session& ic;
  std::mutex* mu = nullptr;
  std::unordered_multimap<uint64_t, std::pair<Span, IdentP>> m;
  explicit IdentMemo(IdentCache::Session& s, std::mutex* shared = nullptr) : ic(s), mu(shared) {
    m.reserve(256);
  }
  IdentP get(Span ser) {
    const uint64_t h = span_hash(ser.p, ser.n);
    auto r = m.equal_range(h);
    for (auto it = r.first; it != r.second; ++it) {
      const Span& k = it->second.first;
      if (k.n == ser.n && (k.p == ser.p || !memcmp(k.p, ser.p, ser.n))) return it->second.second;
    }
    IdentP id;
    if (mu) {
      std::lock_guard<std::mutex> g(*mu);
      id = ic.get(ser);
    } else {
      id = ic.get(ser);
    }
    m.emplace(h, std::make_pair(ser, id));
    return id;
  }
};

void resolve_tx(TxRec* t, SdEntry* ends, IdentMemo& memo) {
  if (t->resolve_creator) {
    t->creator = memo.get(t->creator_ser);
    if (!t->creator->ok) {
      t->status = BH_FAB_CREATOR_IDENTITY;
    } else {
      t->creator_check = true;
      if (t->status == BH_FAB_OK) t->status = t->post_status;
    }
  } else if (t->status == BH_FAB_OK) {
    t->status = t->post_status;
  }
  for (size_t k = 0; k < t->end_count; k++) ends[t->end_first + k].id = memo.get(ends[t->end_first + k].id_ser);
}

// Small persistent worker pool for the block decode (parallel_for over chunk
// indices; the calling thread takes chunks too). Size: BH_DECODE_THREADS, else
// 1 (measured below) -- the peer's validator shares the host.
class Pool {
 public:
  static Pool& get() {
    static Pool* p = new Pool();
    return *p;
  }
  size_t size() const { return th_.size() + 1; }
  void run(size_t tasks, const std::function<void(size_t)>& fn) {
    if (tasks <= 1 || th_.empty()) {
      for (size_t k = 0; k < tasks; k++) fn(k);
      return;
    }
    std::unique_lock<std::mutex> call(call_mu_);  // one parallel_for at a time
    uint64_t g;
    {
      std::lock_guard<std::mutex> l(mu_);
      fn_.store(&fn, std::memory_order_relaxed);
      tasks_.store(tasks, std::memory_order_relaxed);
      left_.store(tasks, std::memory_order_relaxed);
      g = ++gen_;
      claim_.store(g << 32, std::memory_order_release);
    }
    cv_.notify_all();
    work(g);
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [&] { return left_.load(std::memory_order_acquire) == 0; });
    fn_.store(nullptr, std::memory_order_relaxed);
  }

 private:
  Pool() {
    // default 1 (round 6, tools/r6_dec.sh on the box, decode-only p50 of the
    // config-3 block: 1 thread 0.25 ms, 2 / 4 / 8 threads 0.31-0.40 /
    // 0.17-0.37 / 0.37-0.53 ms -- waking workers across the box's 256 CPUs
    // costs more than the ~13 us chunks they would take)
    size_t n = 1;
    if (const char* e = getenv("BH_DECODE_THREADS")) n = std::max(1L, std::min(64L, atol(e)));
    for (size_t k = 1; k < n; k++) th_.emplace_back([this] { loop(); });
    for (auto& t : th_) t.detach();
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return gen_ != seen; });
        seen = gen_;
      }
      work(seen);
    }
  }
  // Round 6: a chunk is claimed with one compare-exchange on a word that
  // carries the run's generation (high half) and the next chunk (low half);
  // the mutex per claim before made the workers queue on futexes, and on the
  // box's 256 CPUs a futex hand-off costs tens of microseconds of a ~200 us
  // decode. A worker that wakes late sees another generation (or no chunk
  // left) and claims nothing -- it never consumes a later run's chunk nor
  // runs a finished run's function.
  void work(uint64_t g) {
    for (;;) {
      uint64_t c = claim_.load(std::memory_order_acquire);
      size_t k;
      do {
        if ((c >> 32) != g) return;
        k = (size_t)(c & 0xffffffffu);
        if (k >= tasks_.load(std::memory_order_relaxed)) return;
      } while (!claim_.compare_exchange_weak(c, c + 1, std::memory_order_acq_rel,
                                             std::memory_order_acquire));
      (*fn_.load(std::memory_order_relaxed))(k);  // run g is still open: its fn
      if (left_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> l(mu_);
        done_cv_.notify_all();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_cv_;
  std::atomic<const std::function<void(size_t)>*> fn_{nullptr};
  std::atomic<size_t> tasks_{0}, left_{0};
  std::atomic<uint64_t> claim_{0};
  uint64_t gen_ = 0;
};

// Decode every transaction and resolve its identities, in parallel chunks
// (round 6: the resolve ran serially after the parallel decode, ~200 us of
// 2,000 memo lookups -- a span hash and a ~1 KB compare each -- on one
// thread; each chunk now keeps its own memo, its misses shared through the
// session). ends gets each transaction's endorsements contiguously, in order.
// The outcome does not depend on the order identities are resolved in: a
// memo or the cache only returns what resolve() makes of the same bytes.
void decode_block_txs(const std::vector<Span>& data, std::vector<TxRec>* t,
                      std::vector<SdEntry>* ends) {
  const size_t n = data.size();
  Pool& pool = Pool::get();
  const size_t chunks = std::min<size_t>(n / 16 + 1, 4 * pool.size());
  std::vector<std::vector<SdEntry>> part(chunks);
  IdentCache::Session ic(ident_cache());
  std::mutex ic_mu;
  pool.run(chunks, [&](size_t c) {
    const size_t lo = n * c / chunks, hi = n * (c + 1) / chunks;
    part[c].reserve((hi - lo) * 4);
    for (size_t i = lo; i < hi; i++) decode_tx(data[i], &(*t)[i], &part[c]);
    IdentMemo memo(ic, &ic_mu);  // end_first is chunk-relative until the merge below
    for (size_t i = lo; i < hi; i++) resolve_tx(&(*t)[i], part[c].data(), memo);
  });
  size_t total = 0;
  for (auto& p : part) total += p.size();
  ends->reserve(total);
  for (size_t c = 0; c < chunks; c++) {
    const size_t lo = n * c / chunks, hi = n * (c + 1) / chunks, base = ends->size();
    for (size_t i = lo; i < hi; i++) (*t)[i].end_first += base;
    ends->insert(ends->end(), part[c].begin(), part[c].end());
  }
}

// ---------------------------------------------------------------- x509
// golang.org/x/crypto/cryptobyte (as used by Go 1.21 crypto/ecdsa
// parseSignature for VerifyASN1): readASN1 with DER length rules, tag exact.
bool cb_read(const uint8_t* b, size_t n, size_t* off, uint8_t want_tag, const uint8_t** out,
             size_t* out_n) {
  if (n - *off < 2) return false;
  const uint8_t tag = b[*off], lb = b[*off + 1];
  if ((tag & 0x1f) == 0x1f) return false;  // high-tag-number form unsupported
  size_t hl, len;
  if (!(lb & 0x80)) {
    hl = 2;
    len = lb;
  } else {
    const size_t ll = lb & 0x7f;
    if (ll == 0 || ll > 4 || n - *off < 2 + ll) return false;
    uint32_t l32 = 0;
    for (size_t i = 0; i < ll; i++) l32 = l32 << 8 | b[*off + 2 + i];
    if (l32 < 128) return false;                    // should be short form
    if ((l32 >> ((ll - 1) * 8)) == 0) return false; // leading zero octet
    hl = 2 + ll;
    len = l32;
  }
  if (len > n - *off - hl) return false;
  if (tag != want_tag) return false;
  *out = b + *off + hl;
  *out_n = len;
  *off += hl + len;
  return true;
}

// cryptobyte readASN1Bytes: minimal, non-negative INTEGER, leading zeros stripped
bool cb_uint(const uint8_t* b, size_t n, size_t* off, std::vector<uint8_t>* v) {
  const uint8_t* p;
  size_t l;
  if (!cb_read(b, n, off, 0x02, &p, &l)) return false;
  if (l == 0) return false;
  if (l > 1 && ((p[0] == 0 && !(p[1] & 0x80)) || (p[0] == 0xff && (p[1] & 0x80)))) return false;
  if (p[0] & 0x80) return false;
  while (l > 1 && p[0] == 0) {
    p++;
    l--;
  }
  v->assign(p, p + l);
  return true;
}

// crypto/ecdsa parseSignature: SEQUENCE { r INTEGER, s INTEGER }, nothing else
bool strict_sig(const uint8_t* b, size_t n, std::vector<uint8_t>* r, std::vector<uint8_t>* s) {
  size_t off = 0, io = 0;
  const uint8_t* in;
  size_t il;
  if (!cb_read(b, n, &off, 0x30, &in, &il) || off != n) return false;
  return cb_uint(in, il, &io, r) && cb_uint(in, il, &io, s) && io == il;
}

// DER length octets, any size (a certificate's signature BIT STRING is not
// bounded, so neither are r and s as cryptobyte reads them)
void der_len(std::vector<uint8_t>* o, size_t n) {
  if (n < 0x80) {
    o->push_back((uint8_t)n);
    return;
  }
  uint8_t b[8];
  int k = 0;
  for (; n; n >>= 8) b[k++] = (uint8_t)n;
  o->push_back((uint8_t)(0x80 | k));
  while (k) o->push_back(b[--k]);
}

void der_uint(std::vector<uint8_t>* o, const std::vector<uint8_t>& v) {
  const bool pad = v[0] & 0x80;
  o->push_back(0x02);
  der_len(o, v.size() + (pad ? 1 : 0));
  if (pad) o->push_back(0);
  o->insert(o->end(), v.begin(), v.end());
}

// canonical DER of (r, s): what the device's Go-asn1 parser reads back
// exactly (an r or s above 32 significant bytes parses as out of range there,
// as bigmod's SetBytes rejects it in Go)
void canon_sig(std::vector<uint8_t>* o, const std::vector<uint8_t>& r,
               const std::vector<uint8_t>& s) {
  std::vector<uint8_t> body;
  der_uint(&body, r);
  der_uint(&body, s);
  o->push_back(0x30);
  der_len(o, body.size());
  o->insert(o->end(), body.begin(), body.end());
}

}  // namespace

// Go crypto/x509 Certificate.CheckSignatureFrom for ECDSA (checkSignature:
// hash the raw TBSCertificate, ecdsa.VerifyASN1 = cryptobyte-strict DER, no
// low-S rule), the check msp/mspimpl.go:717-722 (cert.Verify chain building)
// and msp/cert.go:76-116 make per certificate of an identity's chain.
extern "C" int bh_verify_x509(const uint8_t* certs, const uint64_t* cert_off,
                              const uint32_t* cert_len, const uint8_t* issuer_pub, size_t n,
                              uint8_t* bitmap, uint8_t* reason) {
  if (n && (!certs || !cert_off || !cert_len || !issuer_pub || !bitmap || !reason))
    return bh::host_fail(BH_E_INVALID, "null argument");
  if (n > 0xffffffffull) return bh::host_fail(BH_E_INVALID, "batch too large");
  memset(bitmap, 0, (n + 7) / 8);
  std::vector<uint8_t> sigs;
  std::vector<size_t> which;
  std::vector<uint64_t> tbs_off;
  std::vector<uint32_t> tbs_len, sig_len;
  std::vector<uint64_t> sig_off;
  for (size_t i = 0; i < n; i++) {
    reason[i] = BH_R_UNSUPPORTED;
    const uint8_t* d = certs + cert_off[i];
    const size_t dn = cert_len[i];
    // Certificate ::= SEQUENCE { tbsCertificate, signatureAlgorithm,
    // signatureValue BIT STRING }; the algorithm OIDs of the outer field and
    // of the TBS signature field must match (x509.ParseCertificate)
    size_t off = 0, o = 0;
    Tlv cert, tbs, alg, sv, outer_oid;
    if (!tlv(d, dn, &off, &cert) || cert.tag != 0x30 || off != dn) continue;
    if (!tlv(cert.p, cert.n, &o, &tbs) || tbs.tag != 0x30) continue;
    if (!tlv(cert.p, cert.n, &o, &alg) || alg.tag != 0x30) continue;
    if (!tlv(cert.p, cert.n, &o, &sv) || sv.tag != 0x03 || sv.n < 1 || sv.p[0] != 0) continue;
    size_t ao = 0;
    if (!tlv(alg.p, alg.n, &ao, &outer_oid) || outer_oid.tag != 0x06) continue;
    size_t t = 0;
    Tlv f;
    if (!tlv(tbs.p, tbs.n, &t, &f)) continue;
    if (f.tag == 0xa0 && !tlv(tbs.p, tbs.n, &t, &f)) continue;
    if (f.tag != 0x02) continue;
    Tlv inner, inner_oid;
    if (!tlv(tbs.p, tbs.n, &t, &inner) || inner.tag != 0x30) continue;
    size_t io = 0;
    if (!tlv(inner.p, inner.n, &io, &inner_oid) || inner_oid.raw_n != outer_oid.raw_n ||
        memcmp(inner_oid.raw, outer_oid.raw, inner_oid.raw_n))
      continue;
    if (outer_oid.n != sizeof(kOidEcdsaSha256) ||
        memcmp(outer_oid.p, kOidEcdsaSha256, sizeof(kOidEcdsaSha256)))
      continue;  // SHA-384 / SHA-512 / RSA: Go's x509 path
    Cert c;
    c.tbs = tbs;
    c.sig = Tlv{0x03, sv.p + 1, sv.n - 1, sv.raw, sv.raw_n};
    std::vector<uint8_t> r, s;
    if (!strict_sig(c.sig.p, c.sig.n, &r, &s)) {
      reason[i] = BH_R_DER;  // parseSignature fails: VerifyASN1 false
      continue;
    }
    sig_off.push_back(sigs.size());
    canon_sig(&sigs, r, s);
    sig_len.push_back((uint32_t)(sigs.size() - sig_off.back()));
    tbs_off.push_back(cert_off[i] + (uint64_t)(c.tbs.raw - d));
    tbs_len.push_back((uint32_t)c.tbs.raw_n);
    which.push_back(i);
  }
  const size_t m = which.size();
  if (!m) return BH_OK;
  std::vector<uint8_t> pub(m * 64), bm((m + 7) / 8), rs(m);
  for (size_t k = 0; k < m; k++) memcpy(&pub[64 * k], issuer_pub + 64 * which[k], 64);
  sigs.push_back(0);
  // messages: the TBS bytes inside the caller's certificate buffer
  bh_batch bb{pub.data(), sigs.data(), sig_off.data(), sig_len.data(), certs, tbs_off.data(),
              tbs_len.data()};
  int rc = bh_verify(BH_CURVE_P256, &bb, m, BH_F_NO_LOW_S | BH_F_HASH_SHA256, bm.data(), rs.data());
  if (rc) return rc;
  for (size_t k = 0; k < m; k++) {
    const size_t i = which[k];
    reason[i] = rs[k];
    if (rs[k] == BH_R_OK) bitmap[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
  return BH_OK;
}

// The block's H2D queued while it is decoded (bdls_hip.cpp, "pre-staged block
// spans"): library-internal, hidden.
extern "C" int bhi_prestage_begin(const uint8_t* p, size_t len);
extern "C" void bhi_prestage_wait();
extern "C" void bhi_prestage_end();
struct Prestage {
  int on;
  Prestage(const uint8_t* p, size_t n, bool want) : on(want ? bhi_prestage_begin(p, n) : 0) {}
  void wait() const {
    if (on) bhi_prestage_wait();
  }
  ~Prestage() {
    if (on) bhi_prestage_end();
  }
};

static int block_preverify(const uint8_t* block, size_t len, uint32_t flags, bh_fab_tx* txs,
                           size_t tx_cap, size_t* n_tx, uint8_t* endorse, size_t endorse_cap,
                           size_t* n_endorse, bh_fab_sigref* refs, size_t ref_cap,
                           size_t* n_ref) {
  if (!n_tx || !n_endorse || (len && !block) || (n_ref && !refs && ref_cap))
    return bh::host_fail(BH_E_INVALID, "null argument");
  if (flags & ~(uint32_t)(BH_FAB_F_SHA3 | BH_FAB_F_KEEP_KEYS | BH_FAB_F_DECODE_ONLY))
    return bh::host_fail(BH_E_INVALID, "unknown flag");
  // BH_FAB_TIMING=1: the host phases of every call on stderr (a probe for
  // tools/r6_dec.sh; off by default)
  static const bool timing = getenv("BH_FAB_TIMING") != nullptr;
  const auto T0 = std::chrono::steady_clock::now();
  // the block goes up while it is decoded (round 6; not for decode-only calls)
  const Prestage pre(block, len, !(flags & BH_FAB_F_DECODE_ONLY));
  std::vector<Span> data;
  if (!dec_block(Span{block, len, true}, &data))
    return bh::host_fail(BH_E_INVALID, "block does not unmarshal (common.Block)");
  const auto T1 = std::chrono::steady_clock::now();
  std::vector<TxRec> t(data.size());
  std::vector<SdEntry> ends;
  decode_block_txs(data, &t, &ends);
  const auto T2 = std::chrono::steady_clock::now();
  *n_tx = t.size();
  *n_endorse = ends.size();
  if (n_ref) *n_ref = t.size() + ends.size();
  if ((t.size() && (!txs || tx_cap < t.size())) ||
      (ends.size() && (!endorse || endorse_cap < ends.size())) ||
      (n_ref && (t.size() + ends.size()) && (!refs || ref_cap < t.size() + ends.size())))
    return bh::host_fail(BH_E_INVALID, "result buffers too small (see *n_tx, *n_endorse, *n_ref)");
  const bool decode_only = (flags & BH_FAB_F_DECODE_ONLY) != 0;
  // one device batch: every creator signature and the first round of every
  // transaction's endorsement set
  Batch creators;
  creators.base = block;  // every signed span of the block's SignedData lies in the block
  creators.base_len = len;
  {
    size_t bytes = 0, sig_bytes = 0;
    for (const TxRec& x : t) {
      bytes += x.payload.n;
      sig_bytes += x.signature.n;
    }
    creators.reserve(t.size() + ends.size(), bytes + 2 * 1700 * ends.size(),
                     sig_bytes + 80 * ends.size());
  }
  std::vector<SetRange> sets;
  for (TxRec& x : t) {
    if (x.creator_check) creators.add(x.creator->pub, x.signature, &x.payload, 1, &x.creator_out);
    sets.push_back(SetRange{x.end_first, x.end_count});
  }
  std::vector<uint32_t> valid;
  pre.wait();  // its H2D is queued: the batch's upload indexes the device copy
  const auto T3 = std::chrono::steady_clock::now();
  if (int rc = verify_sets(ends, sets, verify_flags(flags), decode_only, &valid, &creators))
    return rc;
  if (timing) {
    auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::micro>(b - a).count();
    };
    fprintf(stderr, "bh_fab: block %.1f us, txs (decode + identities) %.1f, batch %.1f, "
                    "signatures %.1f (%s)\n", us(T0, T1), us(T1, T2), us(T2, T3),
            us(T3, std::chrono::steady_clock::now()), decode_only ? "decode only" : "device");
  }
  for (size_t i = 0; i < t.size(); i++) {
    TxRec& x = t[i];
    // the creator check precedes the endorser-transaction checks
    if (!decode_only && x.creator_check && x.creator_out != BH_R_OK &&
        (x.status == BH_FAB_OK || x.status == BH_FAB_TX || x.status == BH_FAB_UNSUPPORTED))
      x.status = BH_FAB_CREATOR_SIGNATURE;
    txs[i].status = x.status;
    txs[i].type = x.type;
    txs[i].creator = x.creator_out;
    txs[i].endorse_first = (uint32_t)x.end_first;
    txs[i].endorse_count = (uint32_t)x.end_count;
    txs[i].valid_endorsers = valid[i];
    for (size_t k = 0; k < x.end_count; k++) endorse[x.end_first + k] = ends[x.end_first + k].out;
  }
  if (n_ref) {
    auto off = [&](Span sp) -> uint64_t { return sp.n ? (uint64_t)(sp.p - block) : 0u; };
    const size_t nt = t.size();
    for (size_t i = 0; i < nt; i++) {
      const TxRec& x = t[i];
      bh_fab_sigref& r = refs[i];
      memset(&r, 0, sizeof(r));
      r.reason = x.creator_out;
      if (!x.creator_ser.n) continue;  // no creator reached (decode failed earlier)
      r.ident_off = off(x.creator_ser);
      r.ident_len = (uint32_t)x.creator_ser.n;
      r.sig_off = off(x.signature);
      r.sig_len = (uint32_t)x.signature.n;
      r.msg_off = off(x.payload);
      r.msg_len = (uint32_t)x.payload.n;
    }
    for (size_t j = 0; j < ends.size(); j++) {
      const SdEntry& e = ends[j];
      bh_fab_sigref& r = refs[nt + j];
      memset(&r, 0, sizeof(r));
      r.reason = e.out;
      r.ident_off = off(e.id_ser);
      r.ident_len = (uint32_t)e.id_ser.n;
      r.sig_off = off(e.sig);
      r.sig_len = (uint32_t)e.sig.n;
      r.msg_off = off(e.seg[0]);
      r.msg_len = (uint32_t)e.seg[0].n;
      if (e.nseg > 1) {
        r.msg2_off = off(e.seg[1]);
        r.msg2_len = (uint32_t)e.seg[1].n;
      }
    }
  }
  return BH_OK;
}

extern "C" int bh_fabric_block_preverify(const uint8_t* block, size_t len, uint32_t flags,
                                         bh_fab_tx* txs, size_t tx_cap, size_t* n_tx,
                                         uint8_t* endorse, size_t endorse_cap,
                                         size_t* n_endorse) {
  return block_preverify(block, len, flags, txs, tx_cap, n_tx, endorse, endorse_cap, n_endorse,
                         nullptr, 0, nullptr);
}

extern "C" int bh_fabric_block_preverify_refs(const uint8_t* block, size_t len, uint32_t flags,
                                              bh_fab_tx* txs, size_t tx_cap, size_t* n_tx,
                                              uint8_t* endorse, size_t endorse_cap,
                                              size_t* n_endorse, bh_fab_sigref* refs,
                                              size_t ref_cap, size_t* n_ref) {
  if (!n_ref) return bh::host_fail(BH_E_INVALID, "null argument");
  return block_preverify(block, len, flags, txs, tx_cap, n_tx, endorse, endorse_cap, n_endorse,
                         refs, ref_cap, n_ref);
}

// SignatureSetToValidIdentities over many signature sets in one device batch.
extern "C" int bh_signature_sets_verify(const bh_sd_batch* b, size_t n, const uint32_t* set_first,
                                        size_t n_sets, uint32_t flags, uint8_t* result,
                                        uint32_t* valid_identities) {
  if (!b || (n && (!b->identity || !b->identity_off || !b->identity_len || !b->data_off ||
                   !b->data_len || !b->sig_off || !b->sig_len || !result)) ||
      (n_sets && (!set_first || !valid_identities)))
    return bh::host_fail(BH_E_INVALID, "null argument");
  for (size_t i = 0; i < n; i++)  // a span with bytes needs a buffer (as bh_verify checks)
    if ((b->data_len[i] && !b->data) || (b->sig_len[i] && !b->sig))
      return bh::host_fail(BH_E_INVALID, "null data / sig buffer with nonzero lengths");
  if (flags & ~(uint32_t)(BH_FAB_F_SHA3 | BH_FAB_F_KEEP_KEYS | BH_FAB_F_DECODE_ONLY))
    return bh::host_fail(BH_E_INVALID, "unknown flag");
  std::vector<SetRange> sets;
  for (size_t k = 0; k < n_sets; k++) {
    const size_t f = set_first[k], l = k + 1 < n_sets ? set_first[k + 1] : n;
    if (f > l || l > n) return bh::host_fail(BH_E_INVALID, "set_first not ascending within n");
    sets.push_back(SetRange{f, l - f});
  }
  std::vector<SdEntry> e(n);
  {
    IdentCache::Session ic(ident_cache());  // released before the device work
    for (size_t i = 0; i < n; i++) {
      e[i].id = ic.get(Span{b->identity + b->identity_off[i], b->identity_len[i], true});
      e[i].seg[0] = Span{b->data ? b->data + b->data_off[i] : nullptr, b->data_len[i], true};
      e[i].nseg = 1;
      e[i].sig = Span{b->sig ? b->sig + b->sig_off[i] : nullptr, b->sig_len[i], true};
    }
  }
  std::vector<uint32_t> valid;
  if (int rc = verify_sets(e, sets, verify_flags(flags), (flags & BH_FAB_F_DECODE_ONLY) != 0,
                           &valid, nullptr))
    return rc;
  for (size_t i = 0; i < n; i++) result[i] = e[i].out;
  for (size_t k = 0; k < n_sets; k++) valid_identities[k] = valid[k];
  return BH_OK;
}

// Orderer broadcast SigFilter (orderer/common/msgprocessor/sigfilter.go:50-80)
// for n serialized envelopes: protoutil.EnvelopeAsSignedData
// (protoutil/signeddata.go:60-86: payload, "Missing Header", signature
// header) then the one-entry signature set of the policy evaluation.
extern "C" int bh_envelopes_preverify(const uint8_t* envs, const uint64_t* env_off,
                                      const uint32_t* env_len, size_t n, uint32_t flags,
                                      int32_t* status, uint8_t* reason) {
  if (n && (!envs || !env_off || !env_len || !status || !reason))
    return bh::host_fail(BH_E_INVALID, "null argument");
  if (flags & ~(uint32_t)(BH_FAB_F_SHA3 | BH_FAB_F_KEEP_KEYS | BH_FAB_F_DECODE_ONLY))
    return bh::host_fail(BH_E_INVALID, "unknown flag");
  std::vector<SdEntry> e(n);
  std::vector<SetRange> sets;
  std::unique_ptr<IdentCache::Session> ic(new IdentCache::Session(ident_cache()));
  for (size_t i = 0; i < n; i++) {
    status[i] = BH_FAB_OK;
    Envelope env;
    Payload pl;
    SignatureHeader sh;
    if (!dec_envelope(Span{envs + env_off[i], env_len[i], true}, &env)) {
      status[i] = BH_FAB_ENVELOPE;
    } else if (!dec_payload(env.payload, &pl)) {
      status[i] = BH_FAB_PAYLOAD;
    } else if (!pl.has_header || !dec_signature_header(pl.header.signature_header, &sh)) {
      status[i] = BH_FAB_HEADER;  // "Missing Header" / GetSignatureHeaderFromBytes failed
    } else {
      e[i].id = ic->get(sh.creator);
      e[i].seg[0] = env.payload;
      e[i].nseg = 1;
      e[i].sig = env.signature;
      if (!e[i].id->ok) status[i] = BH_FAB_CREATOR_IDENTITY;
      sets.push_back(SetRange{i, 1});
    }
  }
  ic.reset();  // release the cache before device work
  std::vector<uint32_t> valid;
  if (int rc = verify_sets(e, sets, verify_flags(flags), (flags & BH_FAB_F_DECODE_ONLY) != 0,
                           &valid, nullptr))
    return rc;
  for (size_t i = 0; i < n; i++) {
    reason[i] = status[i] == BH_FAB_OK ? e[i].out : (uint8_t)BH_SP_NOT_VERIFIED;
    if (status[i] == BH_FAB_OK && reason[i] != BH_R_OK && reason[i] != BH_SP_NOT_VERIFIED)
      status[i] = BH_FAB_CREATOR_SIGNATURE;
  }
  return BH_OK;
}

namespace {

// encoding/asn1 Marshal of protoutil's asn1Header{Number *big.Int,
// PreviousHash, DataHash []byte} (protoutil/blockutils.go:42-62)
void asn1_len(std::vector<uint8_t>* o, size_t n) {
  if (n < 0x80) {
    o->push_back((uint8_t)n);
    return;
  }
  uint8_t b[8];
  int k = 0;
  while (n) {
    b[k++] = (uint8_t)n;
    n >>= 8;
  }
  o->push_back((uint8_t)(0x80 | k));
  while (k) o->push_back(b[--k]);
}

std::vector<uint8_t> block_header_bytes(uint64_t number, Span prev, Span data_hash) {
  std::vector<uint8_t> num;  // big.Int two's complement, minimal
  for (int i = 7; i >= 0; i--) {
    const uint8_t v = (uint8_t)(number >> (8 * i));
    if (num.empty() && v == 0) continue;
    if (num.empty() && (v & 0x80)) num.push_back(0);
    num.push_back(v);
  }
  if (num.empty()) num.push_back(0);
  std::vector<uint8_t> body;
  body.push_back(0x02);
  asn1_len(&body, num.size());
  body.insert(body.end(), num.begin(), num.end());
  body.push_back(0x04);
  asn1_len(&body, prev.n);
  if (prev.n) body.insert(body.end(), prev.p, prev.p + prev.n);
  body.push_back(0x04);
  asn1_len(&body, data_hash.n);
  if (data_hash.n) body.insert(body.end(), data_hash.p, data_hash.p + data_hash.n);
  std::vector<uint8_t> out;
  out.push_back(0x30);
  asn1_len(&out, body.size());
  out.insert(out.end(), body.begin(), body.end());
  return out;
}

}  // namespace

namespace {

// protoutil.MarshalOrPanic(&msp.SerializedIdentity{Mspid, IdBytes})
// (protoutil/blockutils.go:298-308 searchConsenterIdentityByID): proto3
// fields in number order, each omitted when empty.
void pb_put_bytes(std::vector<uint8_t>* o, uint32_t num, const uint8_t* p, size_t n) {
  if (!n) return;
  o->push_back((uint8_t)(num << 3 | 2));
  size_t v = n;
  while (v >= 0x80) {
    o->push_back((uint8_t)(v | 0x80));
    v >>= 7;
  }
  o->push_back((uint8_t)v);
  o->insert(o->end(), p, p + n);
}

// The BFT consenter set as searchConsenterIdentityByID walks it: the FIRST
// consenter with the identifier, its marshalled SerializedIdentity (empty: Go
// treats the signature as outside the set).
struct Consenters {
  std::vector<uint32_t> id;
  std::vector<std::vector<uint8_t>> ser;
  const std::vector<uint8_t>* find(uint32_t ident) const {
    for (size_t k = 0; k < id.size(); k++)
      if (id[k] == ident) return &ser[k];
    return nullptr;
  }
};

int block_signatures(const uint8_t* blocks, const uint64_t* block_off, const uint32_t* block_len,
                     size_t n, uint32_t flags, const bh_consenter_set* cs, bh_blocksig_result* res,
                     uint8_t* sig_reason, size_t sig_cap, size_t* sig_total) {
  if (!sig_total || (n && (!blocks || !block_off || !block_len || !res)))
    return bh::host_fail(BH_E_INVALID, "null argument");
  if (flags & ~(uint32_t)(BH_FAB_F_SHA3 | BH_FAB_F_KEEP_KEYS | BH_FAB_F_DECODE_ONLY | BH_BLK_F_BFT))
    return bh::host_fail(BH_E_INVALID, "unknown flag");
  const bool bft = (flags & BH_BLK_F_BFT) != 0;
  Consenters cons;
  if (cs && cs->n) {
    if (!cs->id || !cs->msp_id_off || !cs->msp_id_len || !cs->identity_off || !cs->identity_len)
      return bh::host_fail(BH_E_INVALID, "null consenter array");
    for (size_t k = 0; k < cs->n; k++) {
      if ((cs->msp_id_len[k] && !cs->msp_id) || (cs->identity_len[k] && !cs->identity))
        return bh::host_fail(BH_E_INVALID, "null consenter bytes");
      std::vector<uint8_t> ser;
      if (cs->msp_id_len[k])
        pb_put_bytes(&ser, 1, cs->msp_id + cs->msp_id_off[k], cs->msp_id_len[k]);
      if (cs->identity_len[k])
        pb_put_bytes(&ser, 2, cs->identity + cs->identity_off[k], cs->identity_len[k]);
      cons.id.push_back(cs->id[k]);
      cons.ser.push_back(std::move(ser));
    }
  }
  std::vector<SdEntry> e;
  std::vector<uint8_t> not_in_set;  // per entry: a BFT signature outside the consenter set
  std::vector<SetRange> sets;
  std::vector<std::vector<uint8_t>> hdr_der(n);  // BlockHeaderBytes per block (kept alive)
  std::vector<size_t> set_of(n, SIZE_MAX);
  // entries outside the consenter set are not part of the policy's set: the
  // set handed to verify_sets is the in-set entries only (e_set indexes e)
  std::vector<size_t> e_set;
  std::unique_ptr<IdentCache::Session> ic(new IdentCache::Session(ident_cache()));
  for (size_t i = 0; i < n; i++) {
    res[i] = bh_blocksig_result{BH_BLK_OK, 0, 0, 0};
    bool has_header = false;
    std::vector<Span> mds;
    uint64_t number = 0;
    Span prev, dhash;
    const bool ok = pb_walk(blocks + block_off[i], block_len[i], [&](const Field& f) {
      if (is_bytes(f, 1)) {
        has_header = true;
        return pb_walk(f.s.p, f.s.n, [&](const Field& g) {
          if (is_varint(g, 1)) number = g.v;
          else if (is_bytes(g, 2)) prev = g.s;
          else if (is_bytes(g, 3)) dhash = g.s;
          return true;
        });
      }
      if (is_bytes(f, 2)) return pb_walk(f.s.p, f.s.n, [&](const Field&) { return true; });
      if (is_bytes(f, 3))
        return pb_walk(f.s.p, f.s.n, [&](const Field& g) {
          if (is_bytes(g, 1)) mds.push_back(g.s);
          return true;
        });
      return true;
    });
    if (!ok || !has_header) {  // Go dereferences the nil header
      res[i].status = BH_BLK_DECODE;
      continue;
    }
    if (mds.size() < 1) {  // "no signatures in block metadata"
      res[i].status = BH_BLK_NO_SIGNATURES;
      continue;
    }
    // cb.Metadata{1 value, 2 signatures: MetadataSignature{1 signature_header,
    // 2 signature, 3 identifier_header}}
    Span value;
    struct MSig {
      Span sh, sig, idh;
    };
    std::vector<MSig> sigs;
    const bool mok = pb_walk(mds[0].p, mds[0].n, [&](const Field& f) {
      if (is_bytes(f, 1)) {
        value = f.s;
      } else if (is_bytes(f, 2)) {
        MSig m;
        bool k = pb_walk(f.s.p, f.s.n, [&](const Field& g) {
          if (is_bytes(g, 1)) m.sh = g.s;
          else if (is_bytes(g, 2)) m.sig = g.s;
          else if (is_bytes(g, 3)) m.idh = g.s;
          return true;
        });
        sigs.push_back(m);
        return k;
      }
      return true;
    });
    if (!mok) {
      res[i].status = BH_BLK_METADATA;
      continue;
    }
    hdr_der[i] = block_header_bytes(number, prev, dhash);
    const size_t first = e.size(), first_set = e_set.size();
    for (const MSig& m : sigs) {
      SdEntry x;
      x.seg[0] = value;
      x.seg[2] = Span{hdr_der[i].data(), hdr_der[i].size(), true};
      x.nseg = 3;
      x.sig = m.sig;
      if (bft && m.sh.n == 0 && m.idh.n > 0) {
        // blockutils.go:261-272: the signer is the consenter with the
        // IdentifierHeader's identifier; signed = value || idh || header
        uint32_t ident = 0;
        if (!pb_walk(m.idh.p, m.idh.n, [&](const Field& g) {
              if (is_varint(g, 1)) ident = (uint32_t)g.v;  // uint32 field: low 32 bits
              return true;                                 // 2 nonce: bytes, no checks
            })) {
          res[i].status = BH_BLK_IDENTIFIER_HEADER;
          break;
        }
        const std::vector<uint8_t>* ser = cons.find(ident);
        if (!ser || ser->empty()) {  // "not within the consenter set": skipped
          x.out = BH_FAB_E_NOT_CONSENTER;
          e.push_back(x);
          not_in_set.push_back(1);
          continue;
        }
        x.id = ic->get(Span{ser->data(), ser->size(), true});
        x.seg[1] = m.idh;
      } else {
        SignatureHeader sh;
        if (!dec_signature_header(m.sh, &sh)) {  // fails the whole verifier
          res[i].status = BH_BLK_SIGNATURE_HEADER;
          break;
        }
        x.id = ic->get(sh.creator);
        x.seg[1] = m.sh;
      }
      e.push_back(x);
      not_in_set.push_back(0);
    }
    if (res[i].status != BH_BLK_OK) {
      e.resize(first);
      not_in_set.resize(first);
      continue;
    }
    for (size_t k = first; k < e.size(); k++)
      if (!not_in_set[k]) e_set.push_back(k);
    res[i].sig_first = (uint32_t)first;
    res[i].sig_count = (uint32_t)(e.size() - first);
    set_of[i] = sets.size();
    sets.push_back(SetRange{first_set, e_set.size() - first_set});
  }
  ic.reset();
  *sig_total = e.size();
  if (e.size() && (!sig_reason || sig_cap < e.size()))
    return bh::host_fail(BH_E_INVALID, "sig_reason too small (see *sig_total)");
  std::vector<SdEntry> in_set;
  in_set.reserve(e_set.size());
  for (size_t k : e_set) in_set.push_back(e[k]);
  std::vector<uint32_t> valid;
  if (int rc = verify_sets(in_set, sets, verify_flags(flags),
                           (flags & BH_FAB_F_DECODE_ONLY) != 0, &valid, nullptr))
    return rc;
  for (size_t j = 0; j < e_set.size(); j++) e[e_set[j]].out = in_set[j].out;
  for (size_t i = 0; i < n; i++)
    if (set_of[i] != SIZE_MAX) res[i].valid_identities = valid[set_of[i]];
  for (size_t k = 0; k < e.size(); k++) sig_reason[k] = e[k].out;
  return BH_OK;
}

}  // namespace

// Block signatures (protoutil/blockutils.go:245-300 BlockSignatureVerifier;
// called by orderer/common/cluster/util.go:300 VerifyBlockSignature and the
// peer's gossip MCS) for n serialized blocks in one device batch.
extern "C" int bh_block_signatures_preverify(const uint8_t* blocks, const uint64_t* block_off,
                                             const uint32_t* block_len, size_t n, uint32_t flags,
                                             bh_blocksig_result* res, uint8_t* sig_reason,
                                             size_t sig_cap, size_t* sig_total) {
  return block_signatures(blocks, block_off, block_len, n, flags, nullptr, res, sig_reason,
                          sig_cap, sig_total);
}

// The same with bftEnabled (flag BH_BLK_F_BFT) and the channel's consenter
// set (BlockSignatureVerifier(bftEnabled, consenters, policy)).
extern "C" int bh_block_signatures_preverify_bft(const uint8_t* blocks, const uint64_t* block_off,
                                                 const uint32_t* block_len, size_t n,
                                                 uint32_t flags, const bh_consenter_set* consenters,
                                                 bh_blocksig_result* res, uint8_t* sig_reason,
                                                 size_t sig_cap, size_t* sig_total) {
  return block_signatures(blocks, block_off, block_len, n, flags, consenters, res, sig_reason,
                          sig_cap, sig_total);
}
