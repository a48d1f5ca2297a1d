// libbdlship.so host runtime: device contexts, workspaces, C ABI (include/bdls_hip.h).
//
// One context per initialised GPU: a HIP stream, the fixed-base G tables (one
// per curve) and a growable workspace. The host-buffer API shards a batch
// into contiguous record ranges (multiples of 64 so bitmap words concatenate)
// and drives each device from its own host thread -- no collective, since
// records are independent.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bdls_hip.h"
#include "verify.h"

namespace bh {
hipError_t launch_gtab_build(int curve, uint32_t* gtab, hipStream_t s);
hipError_t launch_verify(int curve, const BatchIn& in, const Work& w, const Plan& pl,
                         const uint32_t* gtab, uint32_t n, uint32_t chunk, uint64_t* bitmap,
                         uint8_t* reason, hipStream_t s, hipEvent_t* ev);
hipError_t launch_verify_bdls(int curve, const BdlsIn& in, const Work& w, const Plan& pl,
                              const uint32_t* gtab, uint32_t n, uint32_t chunk, uint64_t* bitmap,
                              uint8_t* reason, hipStream_t s, hipEvent_t* ev);
}  // namespace bh

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(BH_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));        \
  } while (0)

constexpr size_t kMaxChunk = size_t(1) << 22;  // records per kernel pass (workspace bound)
constexpr size_t kGtabWords = size_t(bh::kCombWindows) * bh::kCombEntries * bh::kGEntry;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return BH_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) return fail(BH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    cap = want;
    return BH_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct Dev {
  int id = -1;
  hipStream_t stream = nullptr;
  uint32_t* gtab[2] = {nullptr, nullptr};
  DevBuf ws;        // Work arrays
  DevBuf in_fix;    // host-API staging: pub, offsets, lengths
  DevBuf in_sig, in_msg, out;
  hipEvent_t ev[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  std::mutex mu;
};

std::mutex g_mu;
std::vector<Dev*> g_devs;

size_t round64(size_t n) { return (n + 63) & ~size_t(63); }

size_t pow2_at_least(size_t v) {
  size_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

size_t max_tables_for(size_t ns) {
  return std::min<size_t>(ns / bh::kMinUses, size_t(1) << 16);
}

size_t work_bytes(size_t ns) {
  // 4 scalar SoA arrays (8 limbs) + 4 base-field SoA arrays (9 limbs) + status
  // + per-lane Q tables; then the key plan (fingerprint table, lists, key
  // tables). Every carve is rounded to 256 bytes.
  const size_t hc = pow2_at_least(2 * ns);
  const size_t mt = max_tables_for(ns);
  return 4 * 32 * ns + 4 * 36 * ns + ns + (ns / 64) * 64 * bh::kQTab * bh::kQPt * 4 +
         hc * (8 + 4 + 4 + 4) + ns * 12 + 16 + mt * 4 + mt * (size_t)bh::kKTabWords * 4 +
         256 * 24;
}

int carve_work(Dev& d, size_t n, bh::Work* w, bh::Plan* pl) {
  const size_t ns = round64(n);
  int rc = d.ws.ensure(work_bytes(ns));
  if (rc) return rc;
  char* p = (char*)d.ws.p;
  auto take = [&](size_t bytes) {
    char* q = p;
    p += (bytes + 255) & ~size_t(255);
    return q;
  };
  w->ns = (uint32_t)ns;
  w->e = (uint32_t*)take(32 * ns);
  w->r = (uint32_t*)take(32 * ns);
  w->sm = (uint32_t*)take(32 * ns);
  w->pre = (uint32_t*)take(32 * ns);
  w->qx = (uint32_t*)take(36 * ns);
  w->qy = (uint32_t*)take(36 * ns);
  w->rm = (uint32_t*)take(36 * ns);
  w->r2m = (uint32_t*)take(36 * ns);
  w->st = (uint8_t*)take(ns);
  w->qtab = (uint32_t*)take((ns / 64) * 64 * bh::kQTab * bh::kQPt * 4);
  const size_t hc = pow2_at_least(2 * ns);
  const size_t mt = max_tables_for(ns);
  pl->hc = (uint32_t)hc;
  pl->max_tables = (uint32_t)mt;
  pl->slot_hash = (uint64_t*)take(hc * 8);
  pl->slot_rep = (uint32_t*)take(hc * 4);
  pl->slot_cnt = (uint32_t*)take(hc * 4);
  pl->slot_tab = (uint32_t*)take(hc * 4);
  pl->rec_slot = (uint32_t*)take(ns * 4);
  pl->comb_list = (uint32_t*)take(ns * 4);
  pl->ladder_list = (uint32_t*)take(ns * 4);
  pl->counters = (uint32_t*)take(16);
  pl->tab_rec = (uint32_t*)take(mt * 4 + 4);
  pl->tables = (uint32_t*)take(mt * (size_t)bh::kKTabWords * 4 + 4);
  return BH_OK;
}

int dev_init(Dev& d, int id) {
  d.id = id;
  HIPCHK(hipSetDevice(id));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, id));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(BH_E_NODEV, std::string("device ") + std::to_string(id) + " is " +
                                prop.gcnArchName + ", this build targets gfx950 only");
  HIPCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  for (int c = 0; c < 2; c++) {
    HIPCHK(hipMalloc(&d.gtab[c], kGtabWords * 4));
    HIPCHK(bh::launch_gtab_build(c, d.gtab[c], d.stream));
  }
  for (auto& e : d.ev) HIPCHK(hipEventCreate(&e));
  HIPCHK(hipStreamSynchronize(d.stream));
  return BH_OK;
}

void dev_free(Dev& d) {
  (void)hipSetDevice(d.id);
  if (d.stream) (void)hipStreamSynchronize(d.stream);
  for (auto& g : d.gtab)
    if (g) (void)hipFree(g);
  d.ws.release();
  d.in_fix.release();
  d.in_sig.release();
  d.in_msg.release();
  d.out.release();
  for (auto& e : d.ev)
    if (e) (void)hipEventDestroy(e);
  if (d.stream) (void)hipStreamDestroy(d.stream);
}

Dev* get_dev(int device) {
  std::lock_guard<std::mutex> g(g_mu);
  for (Dev* d : g_devs)
    if (d->id == device) return d;
  return nullptr;
}

uint32_t inv_chunk(size_t n) {
  size_t c = n / 65536;
  return (uint32_t)std::max<size_t>(1, std::min<size_t>(16, c));
}

// Record-range views of the two input kinds (for kMaxChunk passes).
bh::BatchIn slice(const bh_batch* b, size_t base, uint32_t flags) {
  return bh::BatchIn{b->pub + base * 64, b->sig, b->sig_off + base, b->sig_len + base,
                     b->msg, b->msg_off + base, b->msg_len + base, flags};
}
bh::BdlsIn slice(const bh_bdls_batch* b, size_t base, uint32_t flags) {
  return bh::BdlsIn{b->xy + base * 64, b->r, b->r_off + base, b->r_len + base,
                    b->s, b->s_off + base, b->s_len + base, b->version + base,
                    b->msg, b->msg_off + base, b->msg_len + base, flags};
}
hipError_t launch(int curve, const bh::BatchIn& in, const bh::Work& w, const bh::Plan& pl,
                  const uint32_t* gtab, uint32_t n, uint32_t chunk, uint64_t* bm, uint8_t* rs,
                  hipStream_t s, hipEvent_t* ev) {
  return bh::launch_verify(curve, in, w, pl, gtab, n, chunk, bm, rs, s, ev);
}
hipError_t launch(int curve, const bh::BdlsIn& in, const bh::Work& w, const bh::Plan& pl,
                  const uint32_t* gtab, uint32_t n, uint32_t chunk, uint64_t* bm, uint8_t* rs,
                  hipStream_t s, hipEvent_t* ev) {
  return bh::launch_verify_bdls(curve, in, w, pl, gtab, n, chunk, bm, rs, s, ev);
}

// Core device-resident pass (caller holds d.mu and has set the device).
// With t != nullptr, events bracket every stage and the call synchronises.
template <class B>
int run_dev(Dev& d, int curve, const B* b, size_t n, uint32_t flags, uint64_t* bitmap,
            uint8_t* reason, hipStream_t s, bh_timing* t) {
  if (t) *t = bh_timing{};
  for (size_t base = 0; base < n; base += kMaxChunk) {
    const size_t m = std::min(kMaxChunk, n - base);
    bh::Work w;
    bh::Plan pl;
    int rc = carve_work(d, m, &w, &pl);
    if (rc) return rc;
    HIPCHK(launch(curve, slice(b, base, flags), w, pl, d.gtab[curve], (uint32_t)m, inv_chunk(m),
                  bitmap + base / 64, reason + base, s, t ? d.ev : nullptr));
    if (t) {
      HIPCHK(hipEventSynchronize(d.ev[6]));
      float ms[6];
      for (int k = 0; k < 6; k++) HIPCHK(hipEventElapsedTime(&ms[k], d.ev[k], d.ev[k + 1]));
      t->prep_ms += ms[0];
      t->inv_ms += ms[1];
      t->plan_ms += ms[2];
      t->ktab_ms += ms[3];
      t->keycomb_ms += ms[4];
      t->ladder_ms += ms[5];
      uint32_t cnt[4];
      HIPCHK(hipMemcpy(cnt, pl.counters, 16, hipMemcpyDeviceToHost));
      t->n_keycomb += cnt[0];
      t->n_ladder += cnt[1];
      t->n_keytables += std::min<uint32_t>(cnt[2], pl.max_tables);
    }
  }
  return BH_OK;
}

}  // namespace


extern "C" {

const char* bh_last_error(void) { return g_err.c_str(); }
const char* bh_version(void) { return "bdls-hip 0.1.0 (gfx950)"; }

int bh_init(uint32_t device_mask, uint32_t flags) {
  (void)flags;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) return fail(BH_E_NODEV, "no HIP device visible");
  std::lock_guard<std::mutex> g(g_mu);
  for (int id = 0; id < count && id < 32; id++) {
    if (device_mask && !(device_mask & (1u << id))) continue;
    bool have = false;
    for (Dev* d : g_devs) have |= (d->id == id);
    if (have) continue;
    Dev* d = new Dev();
    int rc = dev_init(*d, id);
    if (rc) {
      dev_free(*d);
      delete d;
      return rc;
    }
    g_devs.push_back(d);
  }
  if (g_devs.empty()) return fail(BH_E_NODEV, "device_mask selects no visible device");
  return BH_OK;
}

int bh_shutdown(void) {
  std::lock_guard<std::mutex> g(g_mu);
  for (Dev* d : g_devs) {
    dev_free(*d);
    delete d;
  }
  g_devs.clear();
  return BH_OK;
}

int bh_device_count(void) {
  std::lock_guard<std::mutex> g(g_mu);
  return (int)g_devs.size();
}

size_t bh_workspace_bytes(size_t n) { return work_bytes(round64(std::min(n, kMaxChunk))); }

int bh_verify_dev(int device, int curve, const bh_batch* b, size_t n, uint32_t flags,
                  uint64_t* bitmap_words, uint8_t* reason, void* stream, int sync,
                  bh_timing* timing) {
  if (!b || (n && (!b->pub || !b->sig || !b->sig_off || !b->sig_len || !b->msg ||
                   !b->msg_off || !b->msg_len || !bitmap_words || !reason)))
    return fail(BH_E_INVALID, "null pointer in batch");
  if (curve != BH_CURVE_P256) return fail(BH_E_INVALID, "curve not supported by bh_verify_dev");
  if (n > 0xffffffffull) return fail(BH_E_INVALID, "batch too large");
  Dev* d = get_dev(device);
  if (!d) return fail(BH_E_NOT_INIT, "device not initialised (call bh_init)");
  std::lock_guard<std::mutex> g(d->mu);
  HIPCHK(hipSetDevice(d->id));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  if (n == 0) return BH_OK;
  int rc = run_dev(*d, curve, b, n, flags, bitmap_words, reason, s, timing);
  if (rc) return rc;
  if (sync && !timing) HIPCHK(hipStreamSynchronize(s));
  return BH_OK;
}

int bh_verify(int curve, const bh_batch* b, size_t n, uint32_t flags, uint8_t* bitmap,
              uint8_t* reason) {
  if (!b || (n && (!b->pub || !b->sig_off || !b->sig_len || !b->msg_off || !b->msg_len ||
                   !bitmap || !reason)))
    return fail(BH_E_INVALID, "null pointer in batch");
  if (curve != BH_CURVE_P256) return fail(BH_E_INVALID, "curve not supported by bh_verify");
  std::vector<Dev*> devs;
  {
    std::lock_guard<std::mutex> g(g_mu);
    devs = g_devs;
  }
  if (devs.empty()) return fail(BH_E_NOT_INIT, "bh_init not called");
  std::memset(bitmap, 0, (n + 7) / 8);
  if (n == 0) return BH_OK;
  // contiguous shards, 64-record aligned
  const size_t nd = std::min(devs.size(), (n + 63) / 64);
  const size_t per = round64((n + nd - 1) / nd);
  std::vector<int> rcs(nd, BH_OK);
  std::vector<std::string> errs(nd);
  auto work = [&](size_t k) {
    const size_t lo = k * per, hi = std::min(n, lo + per);
    if (lo >= hi) return;
    const size_t m = hi - lo;
    Dev& d = *devs[k];
    std::lock_guard<std::mutex> g(d.mu);
    auto body = [&]() -> int {
      HIPCHK(hipSetDevice(d.id));
      // byte ranges of sig / msg used by this shard; offsets rebased
      uint64_t smin = UINT64_MAX, smax = 0, mmin = UINT64_MAX, mmax = 0;
      for (size_t i = lo; i < hi; i++) {
        smin = std::min<uint64_t>(smin, b->sig_off[i]);
        smax = std::max<uint64_t>(smax, b->sig_off[i] + b->sig_len[i]);
        mmin = std::min<uint64_t>(mmin, b->msg_off[i]);
        mmax = std::max<uint64_t>(mmax, b->msg_off[i] + b->msg_len[i]);
      }
      std::vector<uint64_t> so(m), mo(m);
      for (size_t i = 0; i < m; i++) {
        so[i] = b->sig_off[lo + i] - smin;
        mo[i] = b->msg_off[lo + i] - mmin;
      }
      const size_t fix = m * 64 + m * 8 * 2 + m * 4 * 2;
      int rc;
      if ((rc = d.in_fix.ensure(fix + 1024))) return rc;
      if ((rc = d.in_sig.ensure(smax - smin + 16))) return rc;
      if ((rc = d.in_msg.ensure(mmax - mmin + 16))) return rc;
      if ((rc = d.out.ensure(round64(m) / 8 + m + 1024))) return rc;
      char* f = (char*)d.in_fix.p;
      uint8_t* dpub = (uint8_t*)f;
      uint64_t* dso = (uint64_t*)(f + ((m * 64 + 255) & ~size_t(255)));
      uint64_t* dmo = dso + m;
      uint32_t* dsl = (uint32_t*)(dmo + m);
      uint32_t* dml = dsl + m;
      uint64_t* dbm = (uint64_t*)d.out.p;
      uint8_t* drs = (uint8_t*)(dbm + round64(m) / 64);
      hipStream_t s = d.stream;
      HIPCHK(hipMemcpyAsync(dpub, b->pub + lo * 64, m * 64, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(dso, so.data(), m * 8, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(dmo, mo.data(), m * 8, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(dsl, b->sig_len + lo, m * 4, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(dml, b->msg_len + lo, m * 4, hipMemcpyHostToDevice, s));
      if (smax > smin)
        HIPCHK(hipMemcpyAsync(d.in_sig.p, b->sig + smin, smax - smin, hipMemcpyHostToDevice, s));
      if (mmax > mmin)
        HIPCHK(hipMemcpyAsync(d.in_msg.p, b->msg + mmin, mmax - mmin, hipMemcpyHostToDevice, s));
      bh_batch db{dpub, (const uint8_t*)d.in_sig.p, dso, dsl, (const uint8_t*)d.in_msg.p, dmo, dml};
      rc = run_dev(d, curve, &db, m, flags, dbm, drs, s, nullptr);
      if (rc) return rc;
      std::vector<uint64_t> words(round64(m) / 64);
      HIPCHK(hipMemcpyAsync(words.data(), dbm, words.size() * 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(reason + lo, drs, m, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      // lo is a multiple of 64 -> byte-aligned splice
      uint8_t* dst = bitmap + lo / 8;
      const size_t nbytes = (m + 7) / 8;
      std::memcpy(dst, words.data(), nbytes);
      return BH_OK;
    };
    rcs[k] = body();
    if (rcs[k]) errs[k] = g_err;
  };
  if (nd == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (size_t k = 0; k < nd; k++) th.emplace_back(work, k);
    for (auto& t : th) t.join();
  }
  for (size_t k = 0; k < nd; k++)
    if (rcs[k]) return fail(rcs[k], errs[k]);
  return BH_OK;
}

int bh_csp_verify_p256(const uint8_t pub[64], const uint8_t* sig, size_t sig_len,
                       const uint8_t* digest, size_t digest_len, int* valid, int* reason) {
  if (!pub || !valid || !reason) return fail(BH_E_INVALID, "null argument");
  static const uint8_t empty = 0;
  uint64_t so = 0, mo = 0;
  uint32_t sl = (uint32_t)sig_len, ml = (uint32_t)digest_len;
  bh_batch b{pub, sig ? sig : &empty, &so, &sl, digest ? digest : &empty, &mo, &ml};
  uint8_t bm = 0, rs = 0;
  int rc = bh_verify(BH_CURVE_P256, &b, 1, 0, &bm, &rs);
  if (rc) return rc;
  *valid = bm & 1;
  *reason = rs;
  return BH_OK;
}

int bh_parse_der_sig(const uint8_t* der, size_t len, uint8_t r[32], uint8_t s[32], int* r_big,
                     int* s_big) {
  if ((!der && len) || !r || !s || !r_big || !s_big) return fail(BH_E_INVALID, "null argument");
  if (len > 0xffffffffull) return BH_R_DER;
  bh::DerSig ds;
  std::memset(&ds, 0, sizeof(ds));
  uint8_t rc = bh::der_parse_sig(der, (uint32_t)len, &ds);
  std::memset(r, 0, 32);
  std::memset(s, 0, 32);
  *r_big = *s_big = 0;
  if (rc == BH_R_OK) {
    bh::limbs_to_be32(r, ds.r);
    bh::limbs_to_be32(s, ds.s);
    *r_big = (int)ds.r_big;
    *s_big = (int)ds.s_big;
  }
  return rc;
}

int bh_dev_alloc(int device, size_t bytes, void** ptr) {
  if (!ptr) return fail(BH_E_INVALID, "null ptr");
  Dev* d = get_dev(device);
  if (!d) return fail(BH_E_NOT_INIT, "device not initialised (call bh_init)");
  HIPCHK(hipSetDevice(d->id));
  hipError_t e = hipMalloc(ptr, bytes ? bytes : 1);
  if (e != hipSuccess) return fail(BH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return BH_OK;
}

int bh_dev_free(int device, void* ptr) {
  Dev* d = get_dev(device);
  if (!d) return fail(BH_E_NOT_INIT, "device not initialised (call bh_init)");
  HIPCHK(hipSetDevice(d->id));
  HIPCHK(hipFree(ptr));
  return BH_OK;
}

static int copy_sync(int device, void* dst, const void* src, size_t bytes, hipMemcpyKind k) {
  Dev* d = get_dev(device);
  if (!d) return fail(BH_E_NOT_INIT, "device not initialised (call bh_init)");
  if (!bytes) return BH_OK;
  if (!dst || !src) return fail(BH_E_INVALID, "null pointer");
  std::lock_guard<std::mutex> g(d->mu);
  HIPCHK(hipSetDevice(d->id));
  HIPCHK(hipMemcpyAsync(dst, src, bytes, k, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return BH_OK;
}

int bh_memcpy_h2d(int device, void* dst, const void* src, size_t bytes) {
  return copy_sync(device, dst, src, bytes, hipMemcpyHostToDevice);
}

int bh_memcpy_d2h(int device, void* dst, const void* src, size_t bytes) {
  return copy_sync(device, dst, src, bytes, hipMemcpyDeviceToHost);
}

int bh_sync(int device) {
  Dev* d = get_dev(device);
  if (!d) return fail(BH_E_NOT_INIT, "device not initialised (call bh_init)");
  HIPCHK(hipSetDevice(d->id));
  HIPCHK(hipStreamSynchronize(d->stream));
  return BH_OK;
}

// ---- BDLS consensus messages (SignedProto.Verify) --------------------------
int bh_verify_bdls_dev(int device, int curve, const bh_bdls_batch* b, size_t n,
                       uint64_t* bitmap_words, uint8_t* reason, void* stream, int sync,
                       bh_timing* timing) {
  if (!b || (n && (!b->xy || !b->r || !b->r_off || !b->r_len || !b->s || !b->s_off ||
                   !b->s_len || !b->version || !b->msg || !b->msg_off || !b->msg_len ||
                   !bitmap_words || !reason)))
    return fail(BH_E_INVALID, "null pointer in batch");
  if (curve != BH_CURVE_P256 && curve != BH_CURVE_SECP256K1)
    return fail(BH_E_INVALID, "unknown curve");
  if (n > 0xffffffffull) return fail(BH_E_INVALID, "batch too large");
  Dev* d = get_dev(device);
  if (!d) return fail(BH_E_NOT_INIT, "device not initialised (call bh_init)");
  std::lock_guard<std::mutex> g(d->mu);
  HIPCHK(hipSetDevice(d->id));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  if (n == 0) return BH_OK;
  int rc = run_dev(*d, curve, b, n, 0u, bitmap_words, reason, s, timing);
  if (rc) return rc;
  if (sync && !timing) HIPCHK(hipStreamSynchronize(s));
  return BH_OK;
}

int bh_verify_bdls(int curve, const bh_bdls_batch* b, size_t n, uint8_t* bitmap,
                   uint8_t* reason) {
  if (!b || (n && (!b->xy || !b->r_off || !b->r_len || !b->s_off || !b->s_len || !b->version ||
                   !b->msg_off || !b->msg_len || !bitmap || !reason)))
    return fail(BH_E_INVALID, "null pointer in batch");
  Dev* d = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_devs.empty()) d = g_devs[0];
  }
  if (!d) return fail(BH_E_NOT_INIT, "bh_init not called");
  std::memset(bitmap, 0, (n + 7) / 8);
  if (n == 0) return BH_OK;
  // stage: one contiguous device buffer per host array (BDLS rounds are small)
  auto span = [&](const uint64_t* off, const uint32_t* len, uint64_t* lo) {
    uint64_t a = UINT64_MAX, z = 0;
    for (size_t i = 0; i < n; i++) {
      a = std::min<uint64_t>(a, off[i]);
      z = std::max<uint64_t>(z, off[i] + len[i]);
    }
    *lo = a;
    return z - a;
  };
  uint64_t rlo, slo, mlo;
  const uint64_t rsz = span(b->r_off, b->r_len, &rlo), ssz = span(b->s_off, b->s_len, &slo),
                 msz = span(b->msg_off, b->msg_len, &mlo);
  std::vector<uint64_t> ro(n), so(n), mo(n);
  for (size_t i = 0; i < n; i++) {
    ro[i] = b->r_off[i] - rlo;
    so[i] = b->s_off[i] - slo;
    mo[i] = b->msg_off[i] - mlo;
  }
  std::vector<void*> bufs;
  auto cleanup = [&]() {
    for (void* p : bufs) (void)hipFree(p);
  };
  auto up = [&](const void* src, size_t bytes, void** dst) -> int {
    hipError_t e = hipMalloc(dst, bytes + 16);
    if (e != hipSuccess) return fail(BH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    bufs.push_back(*dst);
    if (bytes) {
      e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) return fail(BH_E_DEVICE, std::string("hipMemcpy: ") + hipGetErrorString(e));
    }
    return BH_OK;
  };
  std::lock_guard<std::mutex> g(d->mu);
  HIPCHK(hipSetDevice(d->id));
  void *dxy, *dr, *ds, *dm, *dro, *dso, *dmo, *drl, *dsl, *dml, *dver, *dbm, *drs;
  int rc = 0;
  if (!rc) rc = up(b->xy, n * 64, &dxy);
  if (!rc) rc = up(b->r ? b->r + rlo : nullptr, b->r ? rsz : 0, &dr);
  if (!rc) rc = up(b->s ? b->s + slo : nullptr, b->s ? ssz : 0, &ds);
  if (!rc) rc = up(b->msg ? b->msg + mlo : nullptr, b->msg ? msz : 0, &dm);
  if (!rc) rc = up(ro.data(), n * 8, &dro);
  if (!rc) rc = up(so.data(), n * 8, &dso);
  if (!rc) rc = up(mo.data(), n * 8, &dmo);
  if (!rc) rc = up(b->r_len, n * 4, &drl);
  if (!rc) rc = up(b->s_len, n * 4, &dsl);
  if (!rc) rc = up(b->msg_len, n * 4, &dml);
  if (!rc) rc = up(b->version, n * 4, &dver);
  if (!rc) rc = up(nullptr, round64(n) / 8, &dbm);
  if (!rc) rc = up(nullptr, n, &drs);
  if (!rc) {
    bh_bdls_batch db{(const uint8_t*)dxy, (const uint8_t*)dr, (const uint64_t*)dro,
                     (const uint32_t*)drl, (const uint8_t*)ds, (const uint64_t*)dso,
                     (const uint32_t*)dsl, (const uint32_t*)dver, (const uint8_t*)dm,
                     (const uint64_t*)dmo, (const uint32_t*)dml};
    rc = run_dev(*d, curve, &db, n, 0u, (uint64_t*)dbm, (uint8_t*)drs, d->stream, nullptr);
  }
  if (!rc) {
    std::vector<uint64_t> words(round64(n) / 64);
    hipError_t e = hipStreamSynchronize(d->stream);
    if (e == hipSuccess) e = hipMemcpy(words.data(), dbm, words.size() * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(reason, drs, n, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(BH_E_DEVICE, std::string("hipMemcpy: ") + hipGetErrorString(e));
    else std::memcpy(bitmap, words.data(), (n + 7) / 8);
  }
  cleanup();
  return rc;
}

}  // extern "C"

