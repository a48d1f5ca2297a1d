// BDLS drained-batch pre-verification (bh_bdls_preverify, include/bdls_hip.h).
//
// Host side of SURVEY.md 8(a) rows A15-A16: agent-tcp/tcp_peer.go:176-192
// drains the queued raw consensus messages and feeds them one by one to
// Consensus.ReceiveMessage, which verifies the outer SignedProto and, for
// <lock>/<select>/<decide>/<lock-release>, every embedded proof -- one
// btcec/nistec verify per SignedProto under the agent lock. Here the whole
// drained batch is decoded first, every reachable SignedProto that passes the
// participant gate goes into ONE bh_verify_bdls device batch, and the
// per-message verdict is then evaluated from the per-record results in the
// order Go runs its checks.
//
// Wire decoding restates the gogo/protobuf generated code of
// vendor/github.com/BDLS-bft/bdls/message.pb.go (SignedProto.Unmarshal :516-755,
// Message.Unmarshal :757-970, skipMessage :972-1049) including its corner
// cases: last occurrence of a scalar/bytes field wins, PubKeyAxis.Unmarshal
// (message.go:45-55) rejects > 32 bytes and copies a short value into the TAIL
// without clearing the head, a repeated LockRelease merges into the first,
// narrow varints keep the low bits, unknown fields are skipped.
#include <array>
#include <cstdint>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/bdls_hip.h"

namespace bh {
int host_fail(int code, const char* msg);
}

namespace {

constexpr uint32_t kProtocolVersion = 1;  // consensus.go:22
constexpr int kMaxResyncDepth = 8;

enum MsgType : int32_t {  // message.proto MessageType
  T_NOP = 0,
  T_ROUNDCHANGE = 1,
  T_LOCK = 2,
  T_SELECT = 3,
  T_COMMIT = 4,
  T_LOCKRELEASE = 5,
  T_DECIDE = 6,
  T_RESYNC = 7,
};

struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
  bool set = false;  // field present (Go: non-nil slice)
};

struct SProto {  // message.proto SignedProto
  uint32_t version = 0;
  Span message;
  uint8_t x[32] = {0};
  uint8_t y[32] = {0};
  Span r, s;
};

struct Msg {  // message.proto Message
  int32_t type = 0;
  uint64_t height = 0, round = 0;
  Span state;
  std::vector<SProto> proofs;
  bool has_lr = false;
  SProto lr;
};

// ---- wire format (message.pb.go) -------------------------------------------
bool varint(const uint8_t* d, size_t l, size_t& i, uint64_t& v) {
  v = 0;
  for (unsigned shift = 0;; shift += 7) {
    if (shift >= 64) return false;  // ErrIntOverflowMessage
    if (i >= l) return false;       // io.ErrUnexpectedEOF
    const uint8_t b = d[i++];
    v |= (uint64_t)(b & 0x7f) << shift;
    if (b < 0x80) return true;
  }
}

// bytes field: byteLen as Go int (negative -> ErrInvalidLengthMessage),
// postIndex > l -> io.ErrUnexpectedEOF.
bool len_field(const uint8_t* d, size_t l, size_t& i, Span& out) {
  uint64_t v;
  if (!varint(d, l, i, v)) return false;
  const int64_t bl = (int64_t)v;
  if (bl < 0 || (uint64_t)bl > l - i) return false;
  out.p = d + i;
  out.n = (size_t)bl;
  out.set = true;
  i += (size_t)bl;
  return true;
}

// skipMessage (:972-1049): length of the field starting at d[0], or false.
bool skip_field(const uint8_t* d, size_t l, uint64_t& out) {
  int64_t i = 0;
  int depth = 0;
  while ((uint64_t)i < l) {
    uint64_t wire;
    size_t ii = (size_t)i;
    if (!varint(d, l, ii, wire)) return false;
    i = (int64_t)ii;
    switch (wire & 7) {
      case 0:
        for (unsigned shift = 0;; shift += 7) {
          if (shift >= 64) return false;
          if ((uint64_t)i >= l) return false;
          i++;
          if (d[i - 1] < 0x80) break;
        }
        break;
      case 1:
        i += 8;
        break;
      case 2: {
        uint64_t v;
        ii = (size_t)i;
        if (!varint(d, l, ii, v)) return false;
        i = (int64_t)ii;
        const int64_t len = (int64_t)v;
        if (len < 0) return false;
        if (__builtin_add_overflow(i, len, &i)) return false;
        break;
      }
      case 3:
        depth++;
        break;
      case 4:
        if (depth == 0) return false;  // ErrUnexpectedEndOfGroupMessage
        depth--;
        break;
      case 5:
        i += 4;
        break;
      default:
        return false;  // illegal wireType
    }
    if (i < 0) return false;
    if (depth == 0) {
      out = (uint64_t)i;
      return true;
    }
  }
  return false;
}

// Common tag prologue; returns false on a decode error. fn/wt set on success.
bool read_tag(const uint8_t* d, size_t l, size_t& i, int32_t& fn, int& wt) {
  uint64_t wire;
  if (!varint(d, l, i, wire)) return false;
  fn = (int32_t)(uint32_t)(wire >> 3);
  wt = (int)(wire & 7);
  if (wt == 4) return false;  // wiretype end group for non-group
  if (fn <= 0) return false;  // illegal tag
  return true;
}

bool skip_unknown(const uint8_t* d, size_t l, size_t pre, size_t& i) {
  uint64_t sk;
  if (!skip_field(d + pre, l - pre, sk)) return false;
  if (sk > l - pre) return false;
  i = pre + (size_t)sk;
  return true;
}

bool axis(const Span& s, uint8_t out[32]) {  // PubKeyAxis.Unmarshal
  if (s.n > 32) return false;                // ErrPubKey
  if (s.n) std::memcpy(out + 32 - s.n, s.p, s.n);
  return true;
}

// SignedProto.Unmarshal into an existing value (no reset: merge semantics).
bool un_sproto(const uint8_t* d, size_t l, SProto& m) {
  size_t i = 0;
  while (i < l) {
    const size_t pre = i;
    int32_t fn;
    int wt;
    if (!read_tag(d, l, i, fn, wt)) return false;
    Span sp;
    uint64_t v;
    switch (fn) {
      case 1:
        if (wt != 0 || !varint(d, l, i, v)) return false;
        m.version = (uint32_t)v;
        break;
      case 2:
        if (wt != 2 || !len_field(d, l, i, m.message)) return false;
        break;
      case 3:
        if (wt != 2 || !len_field(d, l, i, sp) || !axis(sp, m.x)) return false;
        break;
      case 4:
        if (wt != 2 || !len_field(d, l, i, sp) || !axis(sp, m.y)) return false;
        break;
      case 5:
        if (wt != 2 || !len_field(d, l, i, m.r)) return false;
        break;
      case 6:
        if (wt != 2 || !len_field(d, l, i, m.s)) return false;
        break;
      default:
        if (!skip_unknown(d, l, pre, i)) return false;
    }
  }
  return true;
}

bool un_message(const uint8_t* d, size_t l, Msg& m) {
  size_t i = 0;
  while (i < l) {
    const size_t pre = i;
    int32_t fn;
    int wt;
    if (!read_tag(d, l, i, fn, wt)) return false;
    Span sp;
    uint64_t v;
    switch (fn) {
      case 1:
        if (wt != 0 || !varint(d, l, i, v)) return false;
        m.type = (int32_t)(uint32_t)v;
        break;
      case 2:
        if (wt != 0 || !varint(d, l, i, v)) return false;
        m.height = v;
        break;
      case 3:
        if (wt != 0 || !varint(d, l, i, v)) return false;
        m.round = v;
        break;
      case 4:
        if (wt != 2 || !len_field(d, l, i, m.state)) return false;
        break;
      case 5:
        if (wt != 2 || !len_field(d, l, i, sp)) return false;
        m.proofs.emplace_back();
        if (!un_sproto(sp.p, sp.n, m.proofs.back())) return false;
        break;
      case 6:
        if (wt != 2 || !len_field(d, l, i, sp)) return false;
        if (!m.has_lr) {
          m.has_lr = true;
          m.lr = SProto{};
        }
        if (!un_sproto(sp.p, sp.n, m.lr)) return false;
        break;
      default:
        if (!skip_unknown(d, l, pre, i)) return false;
    }
  }
  return true;
}

// ---- per-message plan ---------------------------------------------------------
using Ident = std::array<uint8_t, 64>;

Ident ident_of(const SProto& s) {  // DefaultPubKeyToIdentity(PublicKey()) == X || Y
  Ident id;
  std::memcpy(id.data(), s.x, 32);
  std::memcpy(id.data() + 32, s.y, 32);
  return id;
}

struct Node {  // one SignedProto occurrence
  SProto sp;
  uint32_t idx = 0;  // position in the flattened SignedProto list
  bool gate = false;
  bool decoded = false;
  Msg m;
};

struct Plan {
  bool decode_ok = false;
  Node outer;
  std::vector<Node> proofs;     // <lock>/<select>/<decide>
  bool has_lr = false;
  Node lr;                      // <lock-release>
  std::vector<Node> lr_proofs;
  std::vector<Plan> subs;       // <resync> loopback
};

struct Ctx {
  std::set<Ident> parts;
  const uint8_t* part_list;
  size_t np;
  size_t n_ident;  // distinct participants (numIdentities, consensus.go:362-367)
  bool quorum;
  std::vector<const SProto*> flat;  // every decoded SignedProto, in order
  std::vector<uint8_t> verify;      // 1 = goes to the device batch
};

void add_node(Ctx& c, Node& nd, bool verify_it) {
  nd.idx = (uint32_t)c.flat.size();
  nd.gate = c.parts.count(ident_of(nd.sp)) != 0;
  c.flat.push_back(&nd.sp);
  c.verify.push_back(verify_it && nd.gate);
  nd.decoded = un_message(nd.sp.message.p, nd.sp.message.n, nd.m);
}

// Plan for one SignedProto handled by receiveMessage (outer or resync loopback).
void plan_signed(Ctx& c, Plan& p, int depth) {
  p.decode_ok = true;
  const bool vok = p.outer.sp.version == kProtocolVersion;
  add_node(c, p.outer, vok);
  if (!vok || !p.outer.gate || !p.outer.decoded) return;
  Msg& m = p.outer.m;
  switch (m.type) {
    case T_LOCK:
    case T_SELECT:
    case T_DECIDE:
      p.proofs.resize(m.proofs.size());
      for (size_t k = 0; k < m.proofs.size(); k++) {
        p.proofs[k].sp = m.proofs[k];
        add_node(c, p.proofs[k], true);
      }
      break;
    case T_LOCKRELEASE:
      if (!m.has_lr) break;
      p.has_lr = true;
      p.lr.sp = m.lr;
      add_node(c, p.lr, true);
      if (p.lr.gate && p.lr.decoded) {
        p.lr_proofs.resize(p.lr.m.proofs.size());
        for (size_t k = 0; k < p.lr_proofs.size(); k++) {
          p.lr_proofs[k].sp = p.lr.m.proofs[k];
          add_node(c, p.lr_proofs[k], true);
        }
      }
      break;
    case T_RESYNC:
      if (depth >= kMaxResyncDepth) break;
      p.subs.resize(m.proofs.size());
      for (size_t k = 0; k < m.proofs.size(); k++) {
        p.subs[k].outer.sp = m.proofs[k];
        plan_signed(c, p.subs[k], depth + 1);
      }
      break;
    default:
      break;
  }
}

// Node references stay valid: vectors are sized before add_node takes addresses,
// and Plans are not moved after planning (the top-level vector is reserved).

struct Verdict {
  int32_t status = BH_BDLS_OK;
  int32_t bad = -1;
  uint32_t distinct = 0;
};

bool states_equal(const Span& a, const Span& b) {  // stateHash(a) == stateHash(b), default hash
  return a.n == b.n && (a.n == 0 || std::memcmp(a.p, b.p, a.n) == 0);
}

bool is_leader(const Ctx& c, uint64_t round, const SProto& signer) {  // roundLeader :1148-1154
  if (c.np == 0) return false;
  const int64_t r = (int64_t)round;  // int(round) % len: negative panics in Go
  if (r < 0) return false;
  const uint8_t* l = c.part_list + 64 * (size_t)(r % (int64_t)c.np);
  const Ident id = ident_of(signer);
  return std::memcmp(l, id.data(), 64) == 0;
}

// verifyMessage (:449-493) of a proof, as seen from the enclosing check.
bool proof_sig(const Node& nd, const uint8_t* rs, uint32_t base, Verdict& v) {
  const int32_t rel = (int32_t)(nd.idx - base);
  if (!nd.gate) {
    v = {BH_BDLS_PROOF_UNKNOWN_PARTICIPANT, rel, v.distinct};
    return false;
  }
  if (rs[nd.idx] != BH_R_OK) {
    v = {BH_BDLS_PROOF_BAD_SIGNATURE, rel, v.distinct};
    return false;
  }
  if (!nd.decoded) {
    v = {BH_BDLS_PROOF_DECODE, rel, v.distinct};
    return false;
  }
  return true;
}

// Proof loops of verifyLockMessage (:520-600), verifySelectMessage (:628-728)
// and verifyDecideMessage (:829-902), after their state-dependent prologues.
void check_proofs(const Ctx& c, const Msg& m, const Node& signer, const std::vector<Node>& proofs,
                  int kind, const uint8_t* rs, uint32_t base, Verdict& v) {
  if ((kind == T_LOCK || kind == T_DECIDE) && !m.state.set) {
    v.status = BH_BDLS_EMPTY_STATE;
    return;
  }
  if (!is_leader(c, m.round, signer.sp)) {
    v.status = BH_BDLS_NOT_LEADER;
    return;
  }
  const int32_t want = kind == T_DECIDE ? T_COMMIT : T_ROUNDCHANGE;
  std::map<Ident, Span> signers;  // map[Identity]State, last wins
  for (const Node& pf : proofs) {
    if (!proof_sig(pf, rs, base, v)) return;
    const int32_t rel = (int32_t)(pf.idx - base);
    if (pf.m.type != want) {
      v.status = BH_BDLS_PROOF_TYPE_MISMATCH, v.bad = rel;
      return;
    }
    if (pf.m.height != m.height) {
      v.status = BH_BDLS_PROOF_HEIGHT_MISMATCH, v.bad = rel;
      return;
    }
    if (pf.m.round != m.round) {
      v.status = BH_BDLS_PROOF_ROUND_MISMATCH, v.bad = rel;
      return;
    }
    signers[ident_of(pf.sp)] = pf.m.state;
  }
  v.distinct = (uint32_t)signers.size();
  if (!c.quorum) return;
  const size_t need = 2 * ((c.n_ident - 1) / 3) + 1;  // 2t+1, t() :1173
  if (kind == T_SELECT) {
    if (signers.size() < need) {
      v.status = BH_BDLS_PROOF_INSUFFICIENT;
      return;
    }
    std::vector<std::pair<Span, size_t>> props;  // dataProposals[stateHash(data)]++
    for (const auto& kv : signers) {
      if (!kv.second.set) continue;
      bool found = false;
      for (auto& pr : props)
        if (states_equal(pr.first, kv.second)) pr.second++, found = true;
      if (!found) props.push_back({kv.second, 1});
    }
    if (!m.state.set && !props.empty()) {
      v.status = BH_BDLS_SELECT_STATE_MISMATCH;
      return;
    }
    size_t mx = 0;
    for (const auto& pr : props) mx = pr.second > mx ? pr.second : mx;
    if (mx >= need) v.status = BH_BDLS_SELECT_PROOF_EXCEEDED;
    return;
  }
  size_t cnt = 0;
  for (const auto& kv : signers)
    if (states_equal(kv.second, m.state)) cnt++;
  if (cnt < need) v.status = BH_BDLS_PROOF_INSUFFICIENT;
}

// receiveMessage (:1209-1226) + verifyMessage + the type switch's proof checks.
Verdict evaluate(const Ctx& c, const Plan& p, const uint8_t* rs, uint32_t base) {
  Verdict v;
  if (!p.decode_ok) {
    v.status = BH_BDLS_DECODE;
    return v;
  }
  v.bad = 0;
  if (p.outer.sp.version != kProtocolVersion) v.status = BH_BDLS_VERSION;
  else if (!p.outer.gate) v.status = BH_BDLS_UNKNOWN_PARTICIPANT;
  else if (rs[p.outer.idx] != BH_R_OK) v.status = BH_BDLS_BAD_SIGNATURE;
  else if (!p.outer.decoded) v.status = BH_BDLS_MSG_DECODE;
  if (v.status != BH_BDLS_OK) return v;
  v.bad = -1;
  const Msg& m = p.outer.m;
  switch (m.type) {
    case T_NOP:
    case T_ROUNDCHANGE:
    case T_COMMIT:
    case T_RESYNC:  // loopback errors are ignored (ReceiveMessage :1197-1204)
      break;
    case T_LOCK:
    case T_SELECT:
    case T_DECIDE:
      check_proofs(c, m, p.outer, p.proofs, m.type, rs, base, v);
      break;
    case T_LOCKRELEASE:
      if (!p.has_lr) {
        v.status = BH_BDLS_LOCKRELEASE_EMPTY;
        break;
      }
      if (!proof_sig(p.lr, rs, base, v)) break;
      check_proofs(c, p.lr.m, p.lr, p.lr_proofs, T_LOCK, rs, base, v);
      break;
    default:
      v.status = BH_BDLS_UNKNOWN_TYPE;
  }
  return v;
}

}  // namespace

extern "C" int bh_bdls_preverify(int curve, const uint8_t* msgs, const uint64_t* msg_off,
                                 const uint32_t* msg_len, size_t n, const uint8_t* participants,
                                 size_t n_participants, uint32_t flags,
                                 bh_bdls_msg_result* results, uint8_t* sp_reason, size_t sp_cap,
                                 size_t* sp_total) {
  if (curve != BH_CURVE_P256 && curve != BH_CURVE_SECP256K1)
    return bh::host_fail(BH_E_INVALID, "unknown curve");
  if (flags & ~(BH_BDLS_F_GIVEN_REASONS | BH_BDLS_F_NO_QUORUM))
    return bh::host_fail(BH_E_INVALID, "unknown flag");
  if (!sp_total || (n && (!msgs || !msg_off || !msg_len || !results)) ||
      (n_participants && !participants))
    return bh::host_fail(BH_E_INVALID, "null pointer");
  if (n > 0xffffffffull) return bh::host_fail(BH_E_INVALID, "batch too large");
  Ctx c;
  c.part_list = participants;
  c.np = n_participants;
  for (size_t k = 0; k < n_participants; k++) {
    Ident id;
    std::memcpy(id.data(), participants + 64 * k, 64);
    c.parts.insert(id);
  }
  c.n_ident = c.parts.size();
  c.quorum = (flags & BH_BDLS_F_NO_QUORUM) == 0;

  std::vector<Plan> plans(n);
  std::vector<uint32_t> first(n), count(n);
  for (size_t i = 0; i < n; i++) {
    first[i] = (uint32_t)c.flat.size();
    SProto sp;
    if (un_sproto(msgs + msg_off[i], msg_len[i], sp)) {
      plans[i].outer.sp = sp;
      plan_signed(c, plans[i], 0);
    }
    count[i] = (uint32_t)(c.flat.size() - first[i]);
    if (c.flat.size() > 0xffffffffull) return bh::host_fail(BH_E_INVALID, "too many records");
  }
  const size_t total = c.flat.size();
  *sp_total = total;
  const bool given = (flags & BH_BDLS_F_GIVEN_REASONS) != 0;
  if (given && !sp_reason) return bh::host_fail(BH_E_INVALID, "BH_BDLS_F_GIVEN_REASONS needs sp_reason");
  if (sp_reason && sp_cap < total) return bh::host_fail(BH_E_INVALID, "sp_cap smaller than sp_total");

  std::vector<uint8_t> rs(total, BH_SP_NOT_VERIFIED);
  if (given) {
    for (size_t k = 0; k < total; k++)
      if (c.verify[k]) rs[k] = sp_reason[k];
  } else {
    // one device batch over every gated record (offsets into the caller's buffer)
    std::vector<uint32_t> sel;
    for (size_t k = 0; k < total; k++)
      if (c.verify[k]) sel.push_back((uint32_t)k);
    const size_t m = sel.size();
    if (m) {
      std::vector<uint8_t> xy(m * 64);
      std::vector<uint64_t> ro(m), so(m), mo(m);
      std::vector<uint32_t> rl(m), sl(m), ml(m), ver(m);
      auto off = [&](const Span& s) -> uint64_t { return s.n ? (uint64_t)(s.p - msgs) : 0; };
      for (size_t j = 0; j < m; j++) {
        const SProto& s = *c.flat[sel[j]];
        std::memcpy(&xy[64 * j], s.x, 32);
        std::memcpy(&xy[64 * j + 32], s.y, 32);
        ro[j] = off(s.r), rl[j] = (uint32_t)s.r.n;
        so[j] = off(s.s), sl[j] = (uint32_t)s.s.n;
        mo[j] = off(s.message), ml[j] = (uint32_t)s.message.n;
        ver[j] = s.version;
      }
      bh_bdls_batch b{xy.data(), msgs, ro.data(), rl.data(), msgs, so.data(), sl.data(),
                      ver.data(), msgs, mo.data(), ml.data()};
      std::vector<uint8_t> bitmap((m + 7) / 8), reason(m);
      const int rc = bh_verify_bdls(curve, &b, m, bitmap.data(), reason.data());
      if (rc) return rc;
      for (size_t j = 0; j < m; j++) rs[sel[j]] = reason[j];
    }
  }
  for (size_t i = 0; i < n; i++) {
    const Verdict v = evaluate(c, plans[i], rs.data(), first[i]);
    bh_bdls_msg_result& o = results[i];
    o.status = v.status;
    o.bad_sp = v.bad;
    const bool dec = plans[i].decode_ok && plans[i].outer.decoded;
    o.type = dec ? (uint32_t)plans[i].outer.m.type : 0u;
    o.height = dec ? plans[i].outer.m.height : 0u;
    o.round = dec ? plans[i].outer.m.round : 0u;
    o.distinct_signers = v.distinct;
    o.sp_first = first[i];
    o.sp_count = count[i];
  }
  if (sp_reason && !given) std::memcpy(sp_reason, rs.data(), total);
  return BH_OK;
}
